"""Lab: register-staged operand stages (tools/lab/w4r_lab.hip) against the library's LDS-DMA w4 weight
gradient (variant 11; +400 no epilogue, +500 no loads / no epilogue), on the step's weight-gradient shapes
at the split for 256 and 128 workgroups; the lab's slab sum is checked against the library's dW.

    python tools/lab/w4r_lab.py [--cfgs 40,52,60] [--reps 20]
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.ms_lab import timeit

ap = argparse.ArgumentParser()
ap.add_argument("--cfgs", default="40,52,60")
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
cfgs = [int(c) for c in a.cfgs.split(",")]
lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libw4r_lab.so"))
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lab.lab_w4r.argtypes = [i32, vp, i64, vp, i64, i32, i32, i32, i32, vp, i32, vp]
lib = L.lib()
dev, bf = "cuda", torch.bfloat16
st = torch.cuda.current_stream().cuda_stream
Mtok = 50432
for wgs in (256, 128):
    for nm, (K, Nout) in {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}.items():
        x = torch.randn(Mtok, K, device=dev).to(bf)
        dy = torch.randn(Mtok, Nout, device=dev).to(bf)
        flop = 2.0 * Mtok * Nout * K
        split = ops._wgrad_split(Mtok, Nout, K, wgs)
        rec = {"shape": nm, "wgs": wgs, "split": split}
        dw = torch.empty(Nout, K, device=dev)
        slab = torch.empty(split, Nout, K, device=dev)
        for rnd in range(2):
            for v, tag in ((11, "w4"), (411, "w4_noepi"), (511, "w4_ceil")):
                lib.vit_gemm_variant(v)
                t = timeit(lambda: ops.linear_wgrad(dy, x, out=dw, split=split), a.reps)
                rec.setdefault(tag, []).append(round(flop / t / 1e12, 1))
            lib.vit_gemm_variant(-1)
            for cfg in cfgs:
                for dbg, tag in ((0, ""), (4, "_noepi")):
                    t = timeit(lambda: lab.lab_w4r(cfg, dy.data_ptr(), Nout, x.data_ptr(), K, Nout, K, Mtok, split,
                                                   slab.data_ptr(), dbg, st), a.reps)
                    rec.setdefault(f"w4r{cfg}{tag}", []).append(round(flop / t / 1e12, 1))
        lib.vit_gemm_variant(11)
        ops.linear_wgrad(dy, x, out=dw, split=split)
        lib.vit_gemm_variant(-1)
        for cfg in cfgs:
            lab.lab_w4r(cfg, dy.data_ptr(), Nout, x.data_ptr(), K, Nout, K, Mtok, split, slab.data_ptr(), 0, st)
            torch.cuda.synchronize()
            rec[f"w4r{cfg}_err"] = float(((slab.sum(0) - dw).abs().max() / dw.abs().max()).item())
        print(json.dumps(rec), flush=True)
