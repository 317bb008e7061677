"""Host cost of enqueueing one bs=256 train step (eager launch path): time from step() call to
return with the GPU idle beforehand, vs the step's GPU time.  If the host is slower than the GPU
(e.g. a loaded box), the eager step becomes launch-bound."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vit-project_amd")]
import torch  # noqa: E402
import vit_amd  # noqa: E402

dev = torch.device("cuda", 0)
model = vit_amd.create_model("vit_base_patch16_224", num_classes=1000, compute_dtype=torch.bfloat16).to(dev)
model.use_flat_grads(True)
opt = vit_amd.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
x = torch.randn(256, 3, 224, 224, device=dev)
y = torch.randint(0, 1000, (256,), device=dev)


def step():
    loss = vit_amd.cross_entropy(model(x), y)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)


for _ in range(5):
    step()
torch.cuda.synchronize()
enq, tot = [], []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq.append(t1 - t0)
    tot.append(t2 - t0)
enq.sort(); tot.sort()
print({"host_enqueue_ms_median": round(enq[5] * 1e3, 2), "step_ms_median": round(tot[5] * 1e3, 2),
       "load_avg": os.getloadavg()})
