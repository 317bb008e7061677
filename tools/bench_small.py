"""Time the step's small critical-path kernels at bs=256 (HIP events): patch unfold,
pos_embed gradient, and the fp32 classifier-head GEMMs (forward, dgrad, wgrad).
Checks each against torch on the same inputs.  VIT_HIP_LIB selects the library (A/B)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vit-project_amd"), os.path.dirname(os.path.abspath(__file__))]
import torch  # noqa: E402
from vit_amd import ops  # noqa: E402
from bench_kernels import timeit  # noqa: E402


def main():
    dev = "cuda"
    B, S, D, C = 256, 197, 768, 1000
    torch.manual_seed(0)
    img = torch.randn(B, 3, 224, 224, device=dev)
    U = ops.patch_unfold(img, 16, torch.bfloat16)
    ref = img.unfold(2, 16, 16).unfold(3, 16, 16).permute(0, 2, 3, 1, 4, 5).reshape(B * 196, 768).to(torch.bfloat16)
    assert torch.equal(U, ref)
    t = timeit(lambda: ops.patch_unfold(img, 16, torch.bfloat16), 50)
    print(json.dumps({"name": "patch_unfold", "ms": round(t * 1e3, 4), "GBps": round(B * 3 * 224 * 224 * 6 / t / 1e9, 1)}))

    dx = torch.randn(B, S, D, device=dev)
    dpos, dcls = torch.empty(S, D, device=dev), torch.empty(D, device=dev)
    ops.pos_grad(dx, B, S, D, dpos, dcls)
    r = dx.double().sum(0).float()
    assert torch.allclose(dpos, r, rtol=1e-5, atol=1e-4) and torch.allclose(dcls, r[0], rtol=1e-5, atol=1e-4)
    t = timeit(lambda: ops.pos_grad(dx, B, S, D, dpos, dcls), 50)
    print(json.dumps({"name": "pos_grad", "ms": round(t * 1e3, 4), "GBps": round(B * S * D * 4 / t / 1e9, 1)}))

    h = torch.randn(B, D, device=dev)
    w, b = torch.randn(C, D, device=dev) * 0.02, torch.randn(C, device=dev)
    y = ops.linear_fwd(h, w, b, out_dtype=torch.float32)
    assert torch.allclose(y, h @ w.t() + b, rtol=1e-4, atol=1e-4)
    t = timeit(lambda: ops.linear_fwd(h, w, b, out_dtype=torch.float32), 50)
    print(json.dumps({"name": "head_fwd_f32", "ms": round(t * 1e3, 4)}))
    dy = torch.randn(B, C, device=dev)
    g = ops.linear_dgrad(dy, w)
    assert torch.allclose(g, dy @ w, rtol=1e-4, atol=1e-4)
    t = timeit(lambda: ops.linear_dgrad(dy, w), 50)
    print(json.dumps({"name": "head_dgrad_f32", "ms": round(t * 1e3, 4)}))
    gw = ops.linear_wgrad(dy, h)
    assert torch.allclose(gw, dy.t() @ h, rtol=1e-4, atol=1e-3)
    t = timeit(lambda: ops.linear_wgrad(dy, h), 50)
    print(json.dumps({"name": "head_wgrad_f32", "ms": round(t * 1e3, 4)}))


if __name__ == "__main__":
    main()
