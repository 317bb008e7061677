"""The plain bf16 GEMM classes of the step on the 4-wave g4 kernel (csrc/gemm_g4.hip) against the 8-wave
kernels it replaced (V5 forward, V1 / V3 input gradients, forced through vit_gemm_variant) and against
hipBLASLt behind torch (F.linear with bias / matmul) -- the vendor kernels round 5 dispatched to --
at the step's shapes: forwards of qkv / proj / fc2 at the two forward chains' row counts (140 / 116
images), input gradients of qkv / fc1 / proj at the full batch.  Interleaved rounds, HIP events, TFLOP/s.

    python tools/bench_g4.py [--reps 20] [--rounds 2] [--walks]   (--walks: every g4 tile walk too)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vit_amd import ops, _lib as L  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--walks", action="store_true")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--wt", action="store_true", help="also time the input gradient as RC x RC on W^T")
    ap.add_argument("--gelu", action="store_true", help="only the fc2 GELU' input gradient: g4 vs V1")
    a = ap.parse_args()
    if a.gelu:
        return gelu(a)
    lib = L.lib()
    dev, bf = "cuda", torch.bfloat16
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    D, Fh = 768, 3072
    B = 256
    m_half = (B // 2 + 3 * B // 64) * 197, (B - (B // 2 + 3 * B // 64)) * 197
    cases = []
    for M in m_half:
        for nm, (K, N) in (("qkv", (D, 3 * D)), ("proj", (D, D)), ("fc2", (Fh, D))):
            cases.append(("fwd", nm, M, N, K))
    for nm, (N, K) in (("qkv", (3 * D, D)), ("fc1", (Fh, D)), ("proj", (D, D))):
        cases.append(("dgrad", nm, B * 197, N, K))
    if a.shapes:
        keep = set(a.shapes.split(","))
        cases = [c for c in cases if f"{c[0]}_{c[1]}" in keep]
    for kind, nm, M, N, K in cases:
        g = torch.Generator(device=dev).manual_seed(M + N + K)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(bf)
        flop = 2.0 * M * N * K
        rec = {"class": kind, "shape": nm, "M": M, "N": N, "K": K}
        if kind == "fwd":
            x = torch.randn(M, K, device=dev, generator=g).to(bf)
            b = torch.randn(N, device=dev, generator=g)
            bb = b.to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: ops.linear_fwd(x, w, b, out=y)  # noqa: E731
            lib_fn = lambda: F.linear(x, w, bb)  # noqa: E731
            old = [5]
        else:
            dy = torch.randn(M, N, device=dev, generator=g).to(bf)
            dx = torch.empty(M, K, device=dev, dtype=bf)
            ours = lambda: ops.linear_dgrad(dy, w, out_dtype=bf, out=dx)  # noqa: E731
            lib_fn = lambda: torch.matmul(dy, w)  # noqa: E731
            old = [1, 3]
            if a.wt:  # the same product as a forward (RC x RC) on a transposed copy of W
                wt = w.t().contiguous()
                for fm in (1, 0):
                    lib.vit_gemm_g4_config(fm, -1, -1, -1)
                    rec[f"g4_wt_walk{fm}"] = round(flop / timeit(lambda: ops.linear_fwd(dy, wt, None, out=dx), a.reps) / 1e12, 1)
                lib.vit_gemm_g4_config(0, 2, 0, 1)
        walks = [(0, 2, 0)]
        if a.walks:
            walks = [(0, 2, 0), (1, 2, 0)] if kind == "fwd" else [(0, 2, 0), (0, 1, 0), (0, 0, 0)]
        for _ in range(a.rounds):
            for wk in walks:
                lib.vit_gemm_g4_config(*wk, -1)
                key = "g4" if wk == (0, 2, 0) else f"g4_walk{wk[0] if kind == 'fwd' else wk[1]}"
                rec.setdefault(key, []).append(round(flop / timeit(ours, a.reps) / 1e12, 1))
            lib.vit_gemm_g4_config(0, 2, 0, 1)
            for v in old:
                lib.vit_gemm_variant(v)
                rec.setdefault(f"V{v}", []).append(round(flop / timeit(ours, a.reps) / 1e12, 1))
                lib.vit_gemm_variant(-1)
            rec.setdefault("hipblaslt", []).append(round(flop / timeit(lib_fn, a.reps) / 1e12, 1))
        print(json.dumps(rec), flush=True)


def gelu(a):
    lib = L.lib()
    dev, bf = "cuda", torch.bfloat16
    M, K, N = 256 * 197, 3072, 768  # dx [M, 3072] = dy [M, 768] @ W2 [768, 3072] * act'
    g = torch.Generator(device=dev).manual_seed(5)
    dy = torch.randn(M, N, device=dev, generator=g).to(bf)
    w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(bf)
    pre = torch.rand(M, K, device=dev, generator=g).to(bf)
    out = torch.empty(M, K, device=dev, dtype=bf)
    db = torch.empty(K, device=dev)
    flop = 2.0 * M * N * K
    fn = lambda: ops.linear_dgrad(dy, w, out_dtype=bf, epi=L.EPI_GELU_BWD, pre=pre, dbias=db, out=out)  # noqa: E731
    rec = {"class": "gelu_dgrad", "M": M, "N": K, "K": N}
    for _ in range(a.rounds):
        for tag, on in (("g4", 1), ("V1", 0)):
            prev = lib.vit_gemm_g4_gelu(on)
            rec.setdefault(tag, []).append(round(flop / timeit(fn, a.reps) / 1e12, 1))
            lib.vit_gemm_g4_gelu(prev)
    print(json.dumps(rec), flush=True)
    for Mf in (27580, 22852):  # the fc1 GELU pair forward at the two chains' rows: g4 (mask 3) vs V5 (mask 1)
        x = torch.randn(Mf, N, device=dev, generator=g).to(bf)
        w1 = (torch.randn(K, N, device=dev, generator=g) * 0.05).to(bf)
        b1 = torch.randn(K, device=dev, generator=g)
        d, act = torch.empty(Mf, K, device=dev, dtype=bf), torch.empty(Mf, K, device=dev, dtype=bf)
        fn = lambda: ops.linear_fwd(x, w1, b1, epi=L.EPI_BIAS_GELU, out=d, act_out=act)  # noqa: E731
        flop = 2.0 * Mf * N * K
        rec = {"class": "gelu_pair_fwd", "M": Mf, "N": K, "K": N}
        for _ in range(a.rounds):
            for tag, on in (("g4", 3), ("V5", 1)):
                prev = lib.vit_gemm_g4_gelu(on)
                rec.setdefault(tag, []).append(round(flop / timeit(fn, a.reps) / 1e12, 1))
                lib.vit_gemm_g4_gelu(prev)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
