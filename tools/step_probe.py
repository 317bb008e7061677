"""The bench step alone (bench.py's ViT-B/16 bs=256 bf16 configuration: flat gradients,
deferred join, side-stream weight gradients, FusedSGD), W + K steps and nothing else -- the
program rocprofv3 counter passes run (tools/gpu_job.sh pmc), so no other leg's launches mix
into the per-kernel averages.

    python tools/step_probe.py [steps] [warmup] [batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402
import vit_amd  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = vit_amd.create_model("vit_base_patch16_224", num_classes=1000, compute_dtype=torch.bfloat16).to(dev)
    model.use_flat_grads(True)
    model.set_deferred_grad_join(True)
    vit_amd.set_wgrad_overlap(True)
    opt = vit_amd.FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(B, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (B,), device=dev)
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream(dev))
        for _ in range(warmup + steps):
            loss = vit_amd.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(dev)
    print("steps", warmup + steps, "loss", float(loss.item()), flush=True)


if __name__ == "__main__":
    main()
