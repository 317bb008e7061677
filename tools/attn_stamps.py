"""Phase stamps of the bf16 attention kernels at the ViT-B/16 bs=256 step shape (diagnostic build
variant selected by vit_debug_attn_stamps; the product launches never record).

Forward stamps:  0 start, 1 K/V images in LDS, 2 wave 0's last query tile done, 6 stores drained.
Backward stamps: 0 start, 1 prologue (Q/dO images, delta) done, 2 phase 1 (dK/dV) done,
                 3 K image written, 4 phase 2 (dQ) + bias partials done, 6 stores drained.
Slot 5 / 7 hold s_memrealtime (100 MHz) at start / end.

    python tools/attn_stamps.py [--batch 256] [--n 197] [--variant 1]

--variant selects the backward form (vit_sdpa_bwd_variant); "bwd_us" is the standalone backward time
(HIP events, mean of 50 launches after warm-up); the two-kernel form (2) records no stamps.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vit_amd import _lib as L, ops  # noqa: E402


def summarize(st, names):
    st = st.astype(np.int64)
    out = {}
    prev = 0
    for i, nm in names:
        d = st[:, i] - st[:, prev]
        out[nm] = {"mean_cyc": round(float(d.mean()), 0), "p10": int(np.percentile(d, 10)),
                   "p90": int(np.percentile(d, 90))}
        prev = i
    tot = st[:, 6] - st[:, 0]
    rt = (st[:, 7] - st[:, 5]) / 100.0  # us
    span = (st[:, 7].max() - st[:, 5].min()) / 100.0
    out["total"] = {"mean_cyc": round(float(tot.mean()), 0), "mean_us": round(float(rt.mean()), 2),
                    "clock_GHz": round(float(tot.sum() / (rt.sum() * 1e3)), 3)}
    out["span_us"] = round(float(span), 1)
    out["mean_concurrent_wgs"] = round(float(rt.sum() / span), 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--n", type=int, default=197)
    ap.add_argument("--variant", type=int, default=-1)
    a = ap.parse_args()
    B, N, H = a.batch, a.n, 12
    D = H * 64
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B * N, 3 * D, device=dev).to(torch.bfloat16)
    do = torch.randn(B * N, D, device=dev).to(torch.bfloat16)
    o, lse = ops.sdpa_fwd(qkv, B, H, N)
    dq = torch.empty_like(qkv)
    dbias = torch.empty(3 * D, device=dev)
    lib = L.lib()
    lib.vit_debug_attn_stamps.argtypes = [ctypes.c_void_p]
    assert lib.vit_sdpa_bwd_variant(a.variant) == 0
    buf = torch.zeros(B * H * 8, dtype=torch.int64, device=dev)
    res = {"N": N, "batch": B, "variant": a.variant}
    for _ in range(10):
        ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq, dbias=dbias)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq, dbias=dbias)
    e1.record()
    torch.cuda.synchronize()
    res["bwd_us"] = round(e0.elapsed_time(e1) * 1e3 / 50, 1)
    buf.zero_()
    for name, fn, names in (
            ("fwd", lambda: ops.sdpa_fwd(qkv, B, H, N, o=o), [(1, "kv_load"), (2, "compute"), (6, "drain")]),
            ("bwd", lambda: ops.sdpa_bwd(qkv, o, do, lse, B, H, N, dqkv=dq, dbias=dbias),
             [(1, "prologue"), (2, "phase1"), (3, "k_image"), (4, "phase2"), (6, "drain")])):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        buf.zero_()
        torch.cuda.synchronize()
        lib.vit_debug_attn_stamps(ctypes.c_void_p(buf.data_ptr()))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        lib.vit_debug_attn_stamps(ctypes.c_void_p(0))
        st = buf.cpu().numpy().reshape(B * H, 8)
        st = st[st[:, 7] != 0]  # workgroups that ran (the backward may walk several items per workgroup)
        res[name] = summarize(st, names)
        res[name]["workgroups"] = int(st.shape[0])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
