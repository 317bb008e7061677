"""Lab bench for the multi-tile deferred-store forward GEMM (csrc/gemm_ms.hip) against the
library's default forward path (V5) on the step's shapes: bit-exact check + HIP-event timing.

    python tools/lab/ms_lab.py [--lab <hipcc -shared build of csrc/gemm_ms.hip>] [--reps 20] [--grids 0,256,512]

Measured negative in the step (profiles/r04/ab_gemm_ms_instep_negative.txt): the route stays opt-in.
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L


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
    ap.add_argument("--lab", default="", help="a separately built gemm_ms.hip (fast iteration); default: libvit_hip.so")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--grids", default="0,256,512")
    ap.add_argument("--cfgs", default="0,1,2,3")
    ap.add_argument("--rows", default="50432,27580")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    lab = ctypes.CDLL(a.lab) if a.lab else L.lib()
    f = lab.vit_gemm_ms
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    f.argtypes = [i32, i32, i32, i32, i32, i32, vp, i64, vp, i64, vp, vp, i64, vp, i32, vp]
    if hasattr(L.lib(), "vit_gemm_ms_config"):  # the reference is the one-tile V* path
        L.lib().vit_gemm_ms_config(0, -1, -1)
    dev, bf = "cuda", torch.bfloat16
    D, F = 768, 3072
    out = []
    for M in [int(v) for v in a.rows.split(",")]:
        cases = {"qkv": (D, 3 * D, 0, 0), "proj": (D, D, 0, 0), "fc1_gelu": (D, F, 1, 0), "fc2": (F, D, 0, 0),
                 "dg_qkv": (3 * D, D, 0, 1), "dg_fc1": (F, D, 0, 1), "dg_proj": (D, D, 0, 1)}
        for nm, (K, N, epi, wl) in cases.items():
            if a.only and nm not in a.only.split(","):
                continue
            x = torch.randn(M, K, device=dev).to(bf)
            w = (torch.randn(K, N, device=dev) * 0.05).to(bf) if wl else (torch.randn(N, K, device=dev) * 0.05).to(bf)
            b = None if wl else torch.randn(N, device=dev)
            y0, y1 = torch.empty(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf)
            z0, z1 = torch.zeros_like(y0), torch.zeros_like(y1)
            flop = 2.0 * M * N * K
            if wl:
                ref = lambda: ops.linear_dgrad(x, w, out_dtype=bf, out=y0)
            elif epi:
                ref = lambda: ops.linear_fwd(x, w, b, epi=L.EPI_BIAS_GELU, out=y0, act_out=y1)
            else:
                ref = lambda: ops.linear_fwd(x, w, b, out=y0)
            ref(); torch.cuda.synchronize()
            t0 = timeit(ref, a.reps)
            rec = {"M": M, "shape": nm, "ref_ms": round(t0 * 1e3, 4), "ref_tf": round(flop / t0 / 1e12, 1)}
            st = torch.cuda.current_stream().cuda_stream
            for bm in [int(v) for v in a.cfgs.split(",")]:
                for g in [int(v) for v in a.grids.split(",")]:
                    def run():
                        rc = f(epi, wl, bm, M, N, K, x.data_ptr(), K, w.data_ptr(), N if wl else K,
                               None if b is None else b.data_ptr(), z0.data_ptr(), N,
                               z1.data_ptr() if epi else None, g, st)
                        assert rc == 0, rc
                    z0.zero_(); z1.zero_()
                    run(); torch.cuda.synchronize()
                    exact = bool(torch.equal(z0, y0)) and (not epi or bool(torch.equal(z1, y1)))
                    if not exact:
                        d = (z0.float() - y0.float()).abs()
                        print("MISMATCH", nm, M, bm, g, d.max().item(), (d > 0).float().mean().item(), flush=True)
                    t = timeit(run, a.reps)
                    rec[f"c{bm}_g{g}"] = {"ms": round(t * 1e3, 4), "tf": round(flop / t / 1e12, 1), "exact": exact}
            print(json.dumps(rec), flush=True)
            out.append(rec)


if __name__ == "__main__":
    main()
