"""Lab diagnostic: which configurations of tools/lab/w4_lab.hip are wrong, and how (repeatability,
error pattern by tile / wave quadrant / fragment)."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
import torch

lab = ctypes.CDLL(os.path.join(ROOT, "tools/lab/libw4_lab.so"))
vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lab.lab_w4.argtypes = [i32, i32, vp, i64, vp, i64, i32, i32, i32, i32, vp, i32, vp]
dev, bf = "cuda", torch.bfloat16
st = torch.cuda.current_stream().cuda_stream
cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "41,40,42").split(",")]
torch.manual_seed(0)
for lay, (m, n, r, split) in ((0, (4096, 768, 768, 1)), (1, (768, 768, 50432, 28)), (0, (50432, 3072, 768, 1))):
    if lay == 0:
        P = torch.randn(m, r, device=dev).to(bf); Q = torch.randn(n, r, device=dev).to(bf)
        ref = P.float() @ Q.float().t()
        ldp, ldq = r, r
    else:
        P = torch.randn(r, m, device=dev).to(bf); Q = torch.randn(r, n, device=dev).to(bf)
        ref = P.float().t() @ Q.float()
        ldp, ldq = m, n
    for cfg in cfgs:
        outs = []
        for rep in range(3):
            C = torch.zeros(split, m, n, device=dev)
            rc = lab.lab_w4(lay, cfg, P.data_ptr(), ldp, Q.data_ptr(), ldq, m, n, r, split, C.data_ptr(), 0, st)
            assert rc == 0
            torch.cuda.synchronize()
            outs.append(C.sum(0))
        err = (outs[0] - ref).abs() > 1e-2 * ref.abs().max()
        rec = {"lay": lay, "shape": [m, n, r], "cfg": cfg, "bad_frac": err.float().mean().item(),
               "repeat_equal": all(torch.equal(outs[0], o) for o in outs[1:])}
        if err.any():
            idx = err.nonzero()
            ri, cj = idx[:, 0], idx[:, 1]
            rec["bad_tiles"] = sorted(set(((ri // 256) * 1000 + cj // 256).tolist()))[:12]
            rec["row_mod256_hist"] = torch.bincount((ri % 256) // 16, minlength=16).tolist()
            rec["col_mod256_hist"] = torch.bincount((cj % 256) // 16, minlength=16).tolist()
            # relative magnitude of the error on bad elements
            rec["err_ratio_med"] = ((outs[0] - ref)[err] / ref.abs().max()).abs().median().item()
        print(json.dumps(rec), flush=True)
