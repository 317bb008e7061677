"""Bit-for-bit check of the fc1 GELU pair epilogue across two builds of the library (e.g. a change to the
epilogue's arithmetic that must not change a bit): each run writes the pair (GELU'(pre), GELU(pre)) of the
8-wave V5 kernel and of the default dispatch for fixed inputs; `cmp` compares two runs with torch.equal.

    VIT_HIP_LIB=<lib a> python tools/gelu_pair_bitcheck.py run a.pt
    VIT_HIP_LIB=<lib b> python tools/gelu_pair_bitcheck.py run b.pt
    python tools/gelu_pair_bitcheck.py cmp a.pt b.pt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch  # noqa: E402

SHAPES = [(27580, 3072, 768), (1000, 3072, 768), (257, 136, 192)]


def run(out):
    from vit_amd import ops, _lib as L
    lib = L.lib()
    res = {}
    for M, N, K in SHAPES:
        g = torch.Generator().manual_seed(M + N + K)
        x = (torch.randn(M, K, generator=g) * 2).to(torch.bfloat16).cuda()
        w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).cuda()
        b = torch.randn(N, generator=g).cuda()
        for v in (5, -1):
            lib.vit_gemm_variant(v)
            d, a = ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU)
            torch.cuda.synchronize()
            res[f"{M}x{N}x{K}/v{v}"] = (d.cpu(), a.cpu())
        lib.vit_gemm_variant(-1)
    torch.save(res, out)
    print("wrote", out, len(res))


def cmp(a, b):
    ra, rb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [k for k in ra if not (torch.equal(ra[k][0], rb[k][0]) and torch.equal(ra[k][1], rb[k][1]))]
    print("identical" if not bad else f"DIFFER: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
