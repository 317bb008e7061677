"""Lab: tools/lab/w4b_lab.hip (the w4 loop on 4 waves of 128 x 64, two workgroups per CU) against the
library's forward (V5) and plain input-gradient (V1 / V3) GEMMs with bf16 output, on the step's shapes at
the full batch and at the two forward chains' row counts; bias on the forwards.  Interleaved rounds, HIP
events; the lab output is compared with the library's (same k order: expect bit equality).

    python tools/lab/w4b_lab.py [--cfgs 1,2,3] [--reps 20]
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.ms_lab import timeit

ap = argparse.ArgumentParser()
ap.add_argument("--cfgs", default="1,2,3")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rows", default="50432,27580")
a = ap.parse_args()
cfgs = [int(c) for c in a.cfgs.split(",")]
lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libw4b_lab.so"))
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lab.lab_w4b.argtypes = [i32, i32, vp, i64, vp, i64, i32, i32, i32, vp, vp, i32, vp]
dev, bf = "cuda", torch.bfloat16
st = torch.cuda.current_stream().cuda_stream
lib = L.lib()
for M in [int(r) for r in a.rows.split(",")]:
    for nm, (K, N) in {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}.items():
        x = torch.randn(M, K, device=dev).to(bf)
        w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
        b = torch.randn(N, device=dev)
        dy = torch.randn(M, N, device=dev).to(bf)
        flop = 2.0 * M * N * K
        y, z = torch.empty(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf)
        dx, dz = torch.empty(M, K, device=dev, dtype=bf), torch.empty(M, K, device=dev, dtype=bf)
        rec = {"M": M, "shape": nm}
        for rnd in range(2):
            t = timeit(lambda: ops.linear_fwd(x, w, b, out=y), a.reps)
            rec.setdefault("fwd_lib", []).append(round(flop / t / 1e12, 1))
            t = timeit(lambda: ops.linear_dgrad(dy, w, out_dtype=bf, out=dx), a.reps)
            rec.setdefault("dgrad_lib", []).append(round(flop / t / 1e12, 1))
            for cfg in cfgs:
                t = timeit(lambda: lab.lab_w4b(0, cfg, x.data_ptr(), K, w.data_ptr(), K, M, N, K, b.data_ptr(),
                                               z.data_ptr(), 0, st), a.reps)
                rec.setdefault(f"fwd_c{cfg}", []).append(round(flop / t / 1e12, 1))
                t = timeit(lambda: lab.lab_w4b(1, cfg, dy.data_ptr(), N, w.data_ptr(), K, M, K, N, None,
                                               dz.data_ptr(), 0, st), a.reps)
                rec.setdefault(f"dgrad_c{cfg}", []).append(round(flop / t / 1e12, 1))
        ops.linear_fwd(x, w, b, out=y)
        ops.linear_dgrad(dy, w, out_dtype=bf, out=dx)
        for cfg in cfgs:
            lab.lab_w4b(0, cfg, x.data_ptr(), K, w.data_ptr(), K, M, N, K, b.data_ptr(), z.data_ptr(), 0, st)
            lab.lab_w4b(1, cfg, dy.data_ptr(), N, w.data_ptr(), K, M, K, N, None, dz.data_ptr(), 0, st)
            torch.cuda.synchronize()
            rec[f"fwd_c{cfg}_err"] = float((z.float() - y.float()).abs().max() / y.float().abs().max())
            rec[f"dgrad_c{cfg}_err"] = float((dz.float() - dx.float()).abs().max() / dx.float().abs().max())
        print(json.dumps(rec), flush=True)
