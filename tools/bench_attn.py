"""Attention forward / backward timing at the ViT-B/16 bs=256 step shape (B*H = 3072 heads of
197 x 64), with the qkv-bias gradient as the step runs it.  VIT_ATTN_BWD_SPLIT=1 selects the
two-kernel backward.  Prints one JSON line.

    python tools/bench_attn.py [--batch 256] [--reps 50] [--n 197]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import torch  # noqa: E402

from vit_amd import ops  # noqa: E402
from tools.bench_kernels import PEAK, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--n", type=int, default=197)
    a = ap.parse_args()
    B, N, H = a.batch, a.n, 12
    D = H * 64
    dev = "cuda"
    qkv = torch.randn(B * N, 3 * D, device=dev).to(torch.bfloat16)
    do = torch.randn(B * N, D, device=dev).to(torch.bfloat16)
    o, lse = ops.sdpa_fwd(qkv, B, H, N)
    dq = torch.empty_like(qkv)
    dbias = torch.empty(3 * D, device=dev)
    fl = 4.0 * B * H * N * N * 64
    tf = timeit(lambda: ops.sdpa_fwd(qkv, B, H, N, o=o), a.reps)
    tb = timeit(lambda: ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq, dbias=dbias), a.reps)
    # minimal HBM bytes of the backward: q, k, v, o, dO read once, dq, dk, dv written once (bf16) + lse
    byts = B * N * D * 2 * 8 + B * H * N * 4
    print(json.dumps({"N": N, "batch": B, "split": os.environ.get("VIT_ATTN_BWD_SPLIT", "0"),
                      "fwd_ms": round(tf * 1e3, 4), "fwd_tflops": round(fl / tf / 1e12, 1),
                      "bwd_ms": round(tb * 1e3, 4), "bwd_tflops": round(2.5 * fl / tb / 1e12, 1),
                      "bwd_frac_mfma": round(2.5 * fl / tb / 1e12 / PEAK, 4),
                      "bwd_min_bytes": byts, "bwd_GBps_min_bytes": round(byts / tb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
