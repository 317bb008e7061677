"""Lab: the 4-wave 256x256 tile with 128x128 wave tiles (tools/lab/w4_lab.hip) against the library's
ping-pong weight-gradient kernel (variant 8) and V5 forward, on the step's shapes: main-loop ceiling
(no ring loads, no epilogue: lab dbg 5, library variant +500) and the loop with loads (lab dbg 4, library
+400), plus a check of the lab's f32 output against the library's.

    python tools/lab/w4_lab.py [--cfgs 41,40,42,31,51] [--reps 20] [--wgs 256]
"""
import argparse, ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.ms_lab import timeit

ap = argparse.ArgumentParser()
ap.add_argument("--cfgs", default="41,40,42,31,51")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--wgs", type=int, default=256, help="weight-gradient workgroups (split-K target)")
ap.add_argument("--only", default="")
a = ap.parse_args()
cfgs = [int(c) for c in a.cfgs.split(",")]

lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libw4_lab.so"))
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lab.lab_w4.argtypes = [i32, i32, vp, i64, vp, i64, i32, i32, i32, i32, vp, i32, vp]
lib = L.lib()
dev, bf = "cuda", torch.bfloat16
Mtok = 50432
st = torch.cuda.current_stream().cuda_stream


def split_for(m, n, r, wgs):
    tiles = ((m + 255) // 256) * ((n + 255) // 256)
    s = max(1, wgs // tiles)
    while s > 1 and (r // s) < 256:
        s -= 1
    return s


def run_lab(lay, cfg, P, ldp, Q, ldq, m, n, r, split, C, dbg):
    rc = lab.lab_w4(lay, cfg, P.data_ptr(), ldp, Q.data_ptr(), ldq, m, n, r, split, C.data_ptr(), dbg, st)
    assert rc == 0, rc


shapes = {"qkv": (768, 2304), "proj": (768, 768), "fc1": (768, 3072), "fc2": (3072, 768)}
for nm, (K, Nout) in shapes.items():
    if a.only and nm not in a.only.split(","):
        continue
    flop = 2.0 * Mtok * Nout * K
    x = torch.randn(Mtok, K, device=dev).to(bf)
    w = (torch.randn(Nout, K, device=dev) * 0.05).to(bf)
    dy = torch.randn(Mtok, Nout, device=dev).to(bf)
    rec = {"shape": nm}
    # weight gradient: P = dy (CR over tokens), Q = x
    m, n, r = Nout, K, Mtok
    split = split_for(m, n, r, a.wgs)
    rec["split"] = split
    slab = torch.empty(split, m, n, device=dev)
    dw = torch.empty(Nout, K, device=dev)
    lib.vit_gemm_variant(8)
    ops.linear_wgrad(dy, x, out=dw)
    torch.cuda.synchronize()
    ref = dw.clone()
    for v, tag in ((8, "lib_pp"), (408, "lib_pp_noepi"), (508, "lib_pp_ceil")):
        lib.vit_gemm_variant(v)
        t = timeit(lambda: ops.linear_wgrad(dy, x, out=dw), a.reps)
        rec[f"wgrad_{tag}"] = round(flop / t / 1e12, 1)
    lib.vit_gemm_variant(-1)
    for cfg in cfgs:
        for dbg, tag in ((0, ""), (4, "_noepi"), (5, "_ceil")):
            t = timeit(lambda: run_lab(1, cfg, dy, Nout, x, K, m, n, r, split, slab, dbg), a.reps)
            rec[f"wgrad_w4c{cfg}{tag}"] = round(flop / t / 1e12, 1)
        slab.zero_()
        run_lab(1, cfg, dy, Nout, x, K, m, n, r, split, slab, 0)
        torch.cuda.synchronize()
        got = slab.sum(0)
        rec[f"wgrad_w4c{cfg}_relerr"] = float(((got - ref).abs().max() / ref.abs().max()).item())
    # forward: P = x (RC), Q = w (RC), f32 out [Mtok, Nout]
    y = torch.empty(Mtok, Nout, device=dev)
    yb = torch.empty(Mtok, Nout, device=dev, dtype=bf)
    for v, tag in ((5, "lib_v5"), (405, "lib_v5_noepi"), (505, "lib_v5_ceil"), (508, "lib_pp_ceil")):
        lib.vit_gemm_variant(v)
        t = timeit(lambda: ops.linear_fwd(x, w, None, out=yb), a.reps)
        rec[f"fwd_{tag}"] = round(flop / t / 1e12, 1)
    lib.vit_gemm_variant(-1)
    ops.linear_fwd(x, w, None, out=yb)
    for cfg in cfgs:
        for dbg, tag in ((0, "_f32out"), (4, "_noepi"), (5, "_ceil")):
            t = timeit(lambda: run_lab(0, cfg, x, K, w, K, Mtok, Nout, K, 1, y, dbg), a.reps)
            rec[f"fwd_w4c{cfg}{tag}"] = round(flop / t / 1e12, 1)
        run_lab(0, cfg, x, K, w, K, Mtok, Nout, K, 1, y, 0)
        torch.cuda.synchronize()
        rec[f"fwd_w4c{cfg}_relerr"] = float(((y - yb.float()).abs().max() / yb.float().abs().max()).item())
    print(json.dumps(rec), flush=True)
