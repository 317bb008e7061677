"""fc1-forward (bias+GELU epilogue) kernel time vs operand data: the bench's roofline leg uses the
model's trunc-normal weights and zero bias; tools/bench_kernels.py uses 0.05*randn weights and a
randn bias.  Same shapes (M = 256*197, N = 3072, K = 768), HIP events, 20 reps each (3 warm-up launches), in an
order that measures each operand set twice, first and later in the run (--first-cold: the original order)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vit-project_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
import vit_amd  # noqa: E402
from vit_amd import ops  # noqa: E402
from vit_amd import _lib as L  # noqa: E402
from bench_kernels import timeit  # noqa: E402

dev = "cuda"
M = 256 * 197
model = vit_amd.create_model("vit_base_patch16_224", num_classes=1000, compute_dtype=torch.bfloat16).to(dev)
model.shadow_params()
fc1 = model.blocks[0].mlp.fc1
wm = fc1.weight._vit_shadow
h = torch.randn(M, 768, device=dev).to(torch.bfloat16)
pre = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
act = torch.empty_like(pre)
cases = {
    "model_w_zero_bias": (wm, torch.zeros(3072, device=dev)),
    "model_w_randn_bias": (wm, torch.randn(3072, device=dev)),
    "randn005_w_randn_bias": ((torch.randn(3072, 768, device=dev) * 0.05).to(torch.bfloat16), torch.randn(3072, device=dev)),
    "randn005_w_zero_bias": ((torch.randn(3072, 768, device=dev) * 0.05).to(torch.bfloat16), torch.zeros(3072, device=dev)),
    "randn002_w_zero_bias": ((torch.randn(3072, 768, device=dev) * 0.02).to(torch.bfloat16), torch.zeros(3072, device=dev)),
}
order = ["randn002_w_zero_bias", "model_w_zero_bias", "model_w_zero_bias", "randn002_w_zero_bias",
         "model_w_randn_bias", "randn005_w_randn_bias", "randn005_w_zero_bias"]
if "--first-cold" in sys.argv:  # the original order: model weights first, right after model creation
    order = list(cases)
for name in order:
    w, b = cases[name]
    t = timeit(lambda: ops.linear_fwd(h, w, b, epi=L.EPI_BIAS_GELU, out=pre, act_out=act), 20)
    print(name, round(t * 1e3, 4), "ms")
