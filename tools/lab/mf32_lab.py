"""Lab: 32x32x16 vs 16x16x32 MFMA in the V5 forward main loop (tools/lab/mf32_lab.hip), per mode
(0 store, 1 no epilogue, 2 no loads + no epilogue), on the step's forward shapes; the library's V5
(vit_gemm_variant 5 / 405 / 505) alongside.  Checks the MF=32 store against the V5 output."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch
from vit_amd import ops, _lib as L
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.ms_lab import timeit

lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libmf32_lab.so"))
vp, i32 = ctypes.c_void_p, ctypes.c_int
lab.lab_gemm.argtypes = [i32, i32, i32, i32, vp, vp, vp, vp, i32, vp]
lib = L.lib()
if hasattr(lib, "vit_gemm_ms_config"):
    lib.vit_gemm_ms_config(0, -1, -1)
dev, bf = "cuda", torch.bfloat16
M = 50432
for nm, (K, N) in {"qkv": (768, 2304), "fc1": (768, 3072), "fc2": (3072, 768)}.items():
    x = torch.randn(M, K, device=dev).to(bf)
    w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=bf)
    z = torch.empty_like(y)
    flop = 2.0 * M * N * K
    st = torch.cuda.current_stream().cuda_stream
    rec = {"shape": nm}
    for rep in range(2):
        for v in (405,):
            lib.vit_gemm_variant(v)
            t = timeit(lambda: ops.linear_fwd(x, w, b, out=y), 20)
            rec[f"V{v}#{rep}"] = round(flop / t / 1e12, 1)
        lib.vit_gemm_variant(-1)
        for mf in (16, 17, 19, 20):
            for mode in (0, 1):
                t = timeit(lambda: lab.lab_gemm(mf, M, N, K, x.data_ptr(), w.data_ptr(), b.data_ptr(), z.data_ptr(), mode, st), 20)
                rec[f"mf{mf}m{mode}#{rep}"] = round(flop / t / 1e12, 1)
    ops.linear_fwd(x, w, b, out=y)
    for mf in (16, 17, 19, 20):
        z.zero_()
        lab.lab_gemm(mf, M, N, K, x.data_ptr(), w.data_ptr(), b.data_ptr(), z.data_ptr(), 0, st)
        torch.cuda.synchronize()
        rec[f"mf{mf}_exact"] = bool(torch.equal(z, y))
        rec[f"mf{mf}_maxdiff"] = (z.float() - y.float()).abs().max().item()
    print(json.dumps(rec), flush=True)
