"""Where the g4 kernel's cycles go (diagnostic stamped instance, vit_debug_g4_stamps): per workgroup the
prologue, every k-step and every epilogue in s_memtime cycles, and the in-kernel clock (s_memtime over
s_memrealtime), for the step's plain GEMM shapes run alone.

    python tools/g4_stamps.py [--tpw 0] [--shapes fwd_qkv,...]

Output per shape: k-step cycles (mean / p10 / p90 over every workgroup's k-steps after the first of a tile,
and the first k-step of a tile separately), epilogue cycles, prologue cycles, MFMA floor per k-step
(128 x 16 = 2048), clock in GHz, kernel us.
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

from vit_amd import ops, _lib as L  # noqa: E402


def analyse(st, nk, ntiles_max):
    """st: [G, 64] stamps.  Events from slot 2: prologue done, then per tile: nk k-step starts, epilogue
    start, epilogue end (zero_acc included)."""
    ks, k0, ep, pro, tot, rt = [], [], [], [], [], []
    for row in st.astype(np.int64):
        if row[1] == 0:
            continue
        pro.append(row[2] - row[1])
        slot = 3
        for q in range(ntiles_max):
            starts = []
            for k in range(nk):
                if slot >= 62 or row[slot] == 0:
                    break
                starts.append(row[slot])
                slot += 1
            if slot + 1 >= 62 or len(starts) < nk or row[slot] == 0:
                break
            e0, e1 = row[slot], row[slot + 1]
            slot += 2
            d = np.diff(np.array(starts + [e0]))
            k0.append(d[0])
            ks.extend(d[1:].tolist())
            ep.append(e1 - e0)
        tot.append(row[62] - row[1])
        rt.append((row[63] - row[0]) / 100.0)
    f = lambda a: {"mean": round(float(np.mean(a)), 0), "p10": int(np.percentile(a, 10)),
                   "p90": int(np.percentile(a, 90))} if len(a) else None
    return {"kstep": f(ks), "kstep_first": f(k0), "epilogue": f(ep), "prologue": f(pro),
            "clock_GHz": round(float(np.sum(tot) / (np.sum(rt) * 1e3)), 3), "wg_us": round(float(np.mean(rt)), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tpw", type=int, default=1)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--dbg", type=int, default=0, help="timing switches: 1 no in-loop loads, 2 no barriers, 4 no stores")
    ap.add_argument("--sched", type=int, default=0, help="k-step schedule (g4::Sched<n>; 0 = the product's)")
    a = ap.parse_args()
    lib = L.lib()
    dev, bf = "cuda", torch.bfloat16
    D, Fh, B = 768, 3072, 256
    m0 = (B // 2 + 3 * B // 64) * 197
    cases = [("fwd", "qkv", m0, 3 * D, D), ("fwd", "proj", m0, D, D), ("fwd", "fc2", m0, D, Fh),
             ("dgrad", "qkv", B * 197, 3 * D, D), ("dgrad", "fc1", B * 197, Fh, D), ("dgrad", "proj", B * 197, D, D),
             ("gelu", "fc2", B * 197, D, Fh),  # gelu: the fc2 GELU' input gradient with its column sums
             ("pair", "fc1", m0, Fh, D)]  # pair: the fc1 GELU pair forward (vit_gemm_g4_gelu bit 1)
    if a.shapes:
        keep = set(a.shapes.split(","))
        cases = [c for c in cases if f"{c[0]}_{c[1]}" in keep]
    buf = torch.zeros(4096 * 64, dtype=torch.int64, device=dev)
    lib.vit_debug_g4_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.vit_gemm_g4_config(-1, -1, -1, a.tpw)  # 0 = no per-workgroup tile limit
    for kind, nm, M, N, K in cases:
        g = torch.Generator(device=dev).manual_seed(1)
        w = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(bf)
        if kind == "pair":
            x = torch.randn(M, K, device=dev, generator=g).to(bf)
            b = torch.randn(N, device=dev, generator=g)
            lib.vit_gemm_g4_gelu(3)
            run = lambda: ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU)  # noqa: E731
            nk, tiles = K // 64, ((M + 255) // 256) * (N // 256)
        elif kind == "fwd":
            x = torch.randn(M, K, device=dev, generator=g).to(bf)
            b = torch.randn(N, device=dev, generator=g)
            run = lambda: ops.linear_fwd(x, w, b)  # noqa: E731
            nk, tiles = K // 64, ((M + 255) // 256) * (N // 256)
        else:
            dy = torch.randn(M, N, device=dev, generator=g).to(bf)
            if kind == "gelu":
                pre = torch.rand(M, K, device=dev, generator=g).to(bf)
                db = torch.empty(K, device=dev)
                run = lambda: ops.linear_dgrad(dy, w, out_dtype=bf, epi=L.EPI_GELU_BWD, pre=pre, dbias=db)  # noqa: E731
            else:
                run = lambda: ops.linear_dgrad(dy, w, out_dtype=bf)  # noqa: E731
            nk, tiles = N // 64, ((M + 255) // 256) * (K // 256)
        for _ in range(30):  # warm clocks
            run()
        torch.cuda.synchronize()
        buf.zero_()
        lib.vit_debug_g4_stamps(buf.data_ptr(), a.dbg | (a.sched << 4))
        run()
        torch.cuda.synchronize()
        lib.vit_debug_g4_stamps(None, 0)
        st = buf.view(-1, 64).cpu().numpy()
        st = st[st[:, 1] != 0]
        rec = {"class": kind, "shape": nm, "M": M, "nk": nk, "tiles": tiles, "wgs": int(st.shape[0]), "tpw": a.tpw,
               "dbg": a.dbg, "sched": a.sched}
        rec.update(analyse(st, nk, 64))
        if kind == "gelu":  # epilogue phases (slots 50, 51): act' landed, products + column sums done
            ok = st[:, 50] != 0
            e0 = st[ok, 3 + nk]
            rec["gelu_wait"] = int(np.mean(st[ok, 50] - e0))
            rec["gelu_mul_csum"] = int(np.mean(st[ok, 51] - st[ok, 50]))
            rec["gelu_sweep"] = int(np.mean(st[ok, 4 + nk] - st[ok, 51]))
            ks = np.diff(st[ok, 3:4 + nk].astype(np.int64), axis=1)  # k-step k's cycles (k = 0 .. nk-1)
            rec["kstep_by_k"] = [int(x) for x in ks.mean(axis=0)]
        span = (st[:, 63].max() - st[:, 0].min()) / 100.0
        rec["span_us"] = round(float(span), 1)
        print(json.dumps(rec), flush=True)
    lib.vit_gemm_g4_config(-1, -1, -1, 1)


if __name__ == "__main__":
    main()
