"""Run one GEMM shape/layout N times (for rocprofv3 counter passes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
which = sys.argv[1] if len(sys.argv) > 1 else "wgrad_fc1"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
if len(sys.argv) > 3:  # force a GEMM tile configuration (big::V<n> / ping-pong 8, 9)
    L.lib().vit_gemm_variant(int(sys.argv[3]))
M, D, F = 256 * 197, 768, 3072
bf = torch.bfloat16
dev = "cuda"
x = torch.randn(M, D, device=dev).to(bf)
dy = torch.randn(M, F, device=dev).to(bf)
w = (torch.randn(F, D, device=dev) * 0.05).to(bf)
for _ in range(reps):
    if which == "wgrad_fc1":
        ops.linear_wgrad(dy, x)
    elif which == "wgrad_pair":  # the step's MLP weight-gradient pair + its slab sums (one batch launch)
        if _ == 0:
            dy2, act = torch.randn(M, D, device=dev).to(bf), torch.randn(M, F, device=dev).to(bf)
            dw2, dw1 = torch.empty(D, F, device=dev), torch.empty(F, D, device=dev)
        cb = ops.ColBatch()
        ops.linear_wgrad_pair((dy2, act, dw2), (dy, x, dw1), cb)
        cb.launch()
    elif which == "fwd_fc2":
        if _ == 0:
            a2 = torch.randn(M, F, device=dev).to(bf)
            w2 = (torch.randn(D, F, device=dev) * 0.05).to(bf)
        ops.linear_fwd(a2, w2, None, out_dtype=bf)
    elif which == "fwd_fc1":
        ops.linear_fwd(x, w, None, out_dtype=bf)
    elif which == "fwd_fc1_gelu":
        b = torch.zeros(F, device=dev)
        pre = torch.empty(M, F, device=dev, dtype=bf)
        act = torch.empty_like(pre)
        ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU, out=pre, act_out=act)
    elif which == "ln_fwd":  # calibration: reads M*768*4 B, writes M*768*2 B (+ 8 B/row stats)
        if _ == 0:
            xf = torch.randn(M, D, device=dev)
            lw, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
            y = torch.empty(M, D, device=dev, dtype=bf)
        ops.layer_norm_fwd(xf, lw, lb, 1e-6, bf, out=y)
    elif which in ("sdpa_fwd", "sdpa_bwd"):  # bs=256 ViT-B/16 attention (12 heads, N=197)
        if _ == 0:
            B, H, N = 256, 12, 197
            qkv = torch.randn(M, 3 * D, device=dev).to(bf)
            o, lse = ops.sdpa_fwd(qkv, B, H, N)
            do = torch.randn(M, D, device=dev).to(bf)
            dq = torch.empty_like(qkv)
        if which == "sdpa_fwd":
            ops.sdpa_fwd(qkv, B, H, N, o=o)
        else:
            ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq)
    elif which == "dgrad_fc1":
        ops.linear_dgrad(dy, w, out_dtype=bf)
    elif which in ("dgrad_fc2_gelu", "dgrad_fc2_plain"):  # the step's fc2 input gradient, with / without GELU'
        if _ == 0:
            dy2 = torch.randn(M, D, device=dev).to(bf)
            w2 = (torch.randn(D, F, device=dev) * 0.05).to(bf)
            pre = torch.randn(M, F, device=dev).to(bf)
            dpre = torch.empty(M, F, device=dev, dtype=bf)
        if which == "dgrad_fc2_gelu":
            ops.linear_dgrad(dy2, w2, out_dtype=bf, epi=L.EPI_GELU_BWD, pre=pre, out=dpre)
        else:
            ops.linear_dgrad(dy2, w2, out_dtype=bf, out=dpre)
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
