"""Run one GEMM shape/layout N times (for rocprofv3 counter passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
which = sys.argv[1] if len(sys.argv) > 1 else "wgrad_fc1"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
M, D, F = 256 * 197, 768, 3072
bf = torch.bfloat16
dev = "cuda"
x = torch.randn(M, D, device=dev).to(bf)
dy = torch.randn(M, F, device=dev).to(bf)
w = (torch.randn(F, D, device=dev) * 0.05).to(bf)
for _ in range(reps):
    if which == "wgrad_fc1":
        ops.linear_wgrad(dy, x)
    elif which == "fwd_fc1":
        ops.linear_fwd(x, w, None, out_dtype=bf)
    elif which == "dgrad_fc1":
        ops.linear_dgrad(dy, w, out_dtype=bf)
torch.cuda.synchronize()
print("done", which)
if which in ("sdpa_bwd", "sdpa_fwd"):
    B, H, N = 256, 12, 197
    qkv = torch.randn(B * N, 3 * 768, device=dev).to(bf)
    o, lse = ops.sdpa_fwd(qkv, B, H, N)
    do = torch.randn(B * N, 768, device=dev).to(bf)
    for _ in range(reps):
        if which == "sdpa_bwd":
            ops.sdpa_bwd(qkv, o, do, lse, B, H, N)
        else:
            ops.sdpa_fwd(qkv, B, H, N)
    torch.cuda.synchronize()
    print("done attn")
