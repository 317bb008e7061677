"""Sustained power and clock of the plain bf16 GEMMs: the g4 kernel (csrc/gemm_g4.hip) against hipBLASLt
behind torch, each run back to back for `--secs` seconds at one step shape, with the GPU's metrics sampled
by amdsmi on a thread.  Under the board's power cap the clock a kernel sustains is set by its energy per
unit of work, which a short HIP-event timing does not see:

    python tools/power_g4.py [--secs 3] [--shapes fwd_qkv,dgrad_fc1]

Per case: TFLOP/s, mean gfx clock (MHz), socket power (W), flop per clock (TFLOP/s / GHz) and pJ/flop.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from bench import GpuTelemetry  # noqa: E402
from vit_amd import ops, _lib as L  # noqa: E402


def sustained(fn, flop, secs, tel_dev):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    # one batch size that takes ~0.1 s, repeated until `secs` have elapsed
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 10 * 1e-3
    n = max(10, int(0.1 / per))
    for _ in range(int(1.0 / (n * per)) + 1):  # 1 s of heat first
        for _ in range(n):
            fn()
    torch.cuda.synchronize()
    tel = GpuTelemetry(tel_dev).start()
    t0 = time.time()
    e0.record()
    reps = 0
    while time.time() - t0 < secs:
        for _ in range(n):
            fn()
        reps += n
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    box = tel.stop()
    dt = e0.elapsed_time(e1) * 1e-3 / reps
    tf = flop / dt / 1e12
    clk = box.get("current_gfxclk", {}).get("mean")
    pw = box.get("current_socket_power", {}).get("mean")
    return {"tflops": round(tf, 1), "mhz": clk, "watts": pw,
            "tflop_per_ghz": round(tf / (clk / 1000), 1) if clk else None,
            "pj_per_flop": round(pw / (tf * 1e12) * 1e12, 3) if pw else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=3.0)
    ap.add_argument("--shapes", default="fwd_qkv,fwd_fc2,dgrad_qkv,dgrad_fc1")
    a = ap.parse_args()
    L.lib()
    dev, bf = "cuda", torch.bfloat16
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    D, Fh, M = 768, 3072, 256 * 197
    shapes = {"fwd_qkv": ("fwd", D, 3 * D), "fwd_fc2": ("fwd", Fh, D), "fwd_proj": ("fwd", D, D),
              "dgrad_qkv": ("dgrad", 3 * D, D), "dgrad_fc1": ("dgrad", Fh, D), "dgrad_proj": ("dgrad", D, D)}
    for nm in a.shapes.split(","):
        kind, A, B = shapes[nm]
        g = torch.Generator(device=dev).manual_seed(A + B)
        if kind == "fwd":
            K, N = A, B
            w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(bf)
            x = torch.randn(M, K, device=dev, generator=g).to(bf)
            b = torch.randn(N, device=dev, generator=g)
            bb = b.to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            ours = lambda: ops.linear_fwd(x, w, b, out=y)  # noqa: E731
            lib_fn = lambda: torch.addmm(bb, x, w.t(), out=y)  # noqa: E731
        else:
            N, K = A, B
            w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(bf)
            dy = torch.randn(M, N, device=dev, generator=g).to(bf)
            dx = torch.empty(M, K, device=dev, dtype=bf)
            ours = lambda: ops.linear_dgrad(dy, w, out_dtype=bf, out=dx)  # noqa: E731
            lib_fn = lambda: torch.matmul(dy, w, out=dx)  # noqa: E731
        flop = 2.0 * M * N * K
        rec = {"shape": nm, "M": M, "N": N, "K": K}
        for tag, fn in (("g4", ours), ("hipblaslt", lib_fn), ("g4_again", ours)):
            rec[tag] = sustained(fn, flop, a.secs, 0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
