"""The step's forward / input-gradient GEMM shapes on our kernels against the vendor libraries behind
torch (hipBLASLt, rocBLAS, CK via torch.backends.cuda.preferred_blas_library), bf16 in / out, at the
full batch and at the forward chains' row counts (140 / 116 images).  Ours with the epilogue the step
runs (bias; bias + GELU pair for fc1), the libraries with the bias epilogue (F.linear) where it
exists; interleaved rounds, HIP events, TFLOP/s.

    python tools/bench_vs_lib.py [--reps 20] [--rows 50432,27580,22852]
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
    ap.add_argument("--rows", default="50432,27580,22852")
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    libs = []
    for name in ("hipblaslt", "rocblas", "ck"):
        try:
            torch.backends.cuda.preferred_blas_library(name)
            libs.append(name)
        except Exception as ex:  # noqa: BLE001
            print(json.dumps({"lib": name, "unavailable": str(ex)[:120]}), flush=True)
    D, Fh = 768, 3072
    for M in [int(r) for r in a.rows.split(",")]:
        for nm, (K, N) in {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, Fh), "fc2": (Fh, D)}.items():
            x = torch.randn(M, K, device=dev).to(bf)
            w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
            b = torch.randn(N, device=dev)
            bb = b.to(bf)
            dy = torch.randn(M, N, device=dev).to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            act = torch.empty(M, N, device=dev, dtype=bf)
            dx = torch.empty(M, K, device=dev, dtype=bf)
            flop = 2.0 * M * N * K
            rec = {"M": M, "shape": nm}
            if nm == "fc1":
                ours_fwd = lambda: ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU, out=y, act_out=act)  # noqa: E731
            else:
                ours_fwd = lambda: ops.linear_fwd(x, w, b, out=y)  # noqa: E731
            ours_dgrad = lambda: ops.linear_dgrad(dy, w, out_dtype=bf, out=dx)  # noqa: E731
            for rnd in range(2):
                rec.setdefault("ours_fwd", []).append(round(flop / timeit(ours_fwd, a.reps) / 1e12, 1))
                rec.setdefault("ours_dgrad", []).append(round(flop / timeit(ours_dgrad, a.reps) / 1e12, 1))
                for lib in libs:
                    torch.backends.cuda.preferred_blas_library(lib)
                    fl = (lambda: F.gelu(F.linear(x, w, bb))) if nm == "fc1" else (lambda: F.linear(x, w, bb))
                    rec.setdefault(f"{lib}_fwd_bias", []).append(round(flop / timeit(fl, a.reps) / 1e12, 1))
                    rec.setdefault(f"{lib}_fwd_plain", []).append(
                        round(flop / timeit(lambda: torch.matmul(x, w.t()), a.reps) / 1e12, 1))
                    rec.setdefault(f"{lib}_dgrad", []).append(
                        round(flop / timeit(lambda: torch.matmul(dy, w), a.reps) / 1e12, 1))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
