"""fp32 MFMA GEMM timing at config C3's shapes (CLIP ViT-L/14 visual tower, B=64: M = 64 x 257 rows),
with and without the stream's stream-K workspace (f32m::gemm_sk_kernel vs one tile per workgroup).

    python tools/bench_f32.py [--batch 64] [--reps 20] [--json out.jsonl]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402

from vit_amd import _lib as L, ops  # noqa: E402

PEAK_F32 = 256 * 4 * 64 * 2.4e9 / 1e12


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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, D = a.batch * 257, 1024
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, D, device=dev, generator=g)
    h = torch.randn(M, 4 * D, device=dev, generator=g)
    w = {n: torch.randn(o, i, device=dev, generator=g) * 0.03
         for n, (o, i) in {"qkv": (3 * D, D), "proj": (D, D), "fc1": (4 * D, D), "fc2": (D, 4 * D)}.items()}
    b = {n: torch.zeros(t.shape[0], device=dev) for n, t in w.items()}
    dy4 = torch.randn(M, 4 * D, device=dev, generator=g)
    dy1 = torch.randn(M, D, device=dev, generator=g)
    pre = torch.empty(M, 4 * D, device=dev)
    act = torch.empty_like(pre)
    cases = {
        "fwd qkv (bias)": (lambda: ops.linear_fwd(x, w["qkv"], b["qkv"]), 2 * M * 3 * D * D),
        "fwd proj (bias)": (lambda: ops.linear_fwd(x, w["proj"], b["proj"]), 2 * M * D * D),
        "fwd fc1 (bias + QuickGELU pair)": (lambda: ops.linear_fwd(x, w["fc1"], b["fc1"], epi=L.EPI_BIAS_QGELU,
                                                                   out=pre, act_out=act), 2 * M * 4 * D * D),
        "fwd fc2 (bias)": (lambda: ops.linear_fwd(h, w["fc2"], b["fc2"]), 2 * M * 4 * D * D),
        "dgrad fc2 -> dh": (lambda: ops.linear_dgrad(dy1, w["fc2"], out_dtype=torch.float32), 2 * M * 4 * D * D),
        "dgrad fc1 -> dx": (lambda: ops.linear_dgrad(dy4, w["fc1"], out_dtype=torch.float32), 2 * M * 4 * D * D),
    }
    st = L.stream_ptr(dev)
    out = []
    for name, (fn, flop) in cases.items():
        row = {"case": name, "M": M, "gflop": round(flop / 1e9, 2)}
        for mode in ("plain", "streamk"):
            if mode == "plain":  # unregistered, and marked registered so the ops do not register it
                L.lib().vit_gemm_streamk_workspace(st, None, 0, None, 0)
                ops._SK[st] = None
            else:
                ops._SK.pop(st, None)
                ops._streamk(dev)
            t = timeit(fn, a.reps)
            row[mode + "_us"] = round(t * 1e6, 1)
            row[mode + "_tf"] = round(flop / t / 1e12, 1)
        row["frac_streamk"] = round(row["streamk_tf"] / PEAK_F32, 3)
        print(json.dumps(row), flush=True)
        out.append(row)
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
