"""HBM traffic of the plain GEMMs on the g4 kernel against hipBLASLt (behind torch) at the step's shapes,
from rocprofv3 counter passes (FETCH_SIZE and WRITE_SIZE in separate runs):

    rocprofv3 --pmc FETCH_SIZE -d D/fetch -o r -- python3 tools/pmc_g4_lib.py run
    rocprofv3 --pmc WRITE_SIZE -d D/write -o r -- python3 tools/pmc_g4_lib.py run
    python3 tools/pmc_g4_lib.py sum D

`run`: every operand is allocated first; then per case REPS launches of g4, then REPS of hipBLASLt, so
the GEMM dispatches after the setup come in blocks of REPS in CASES order.  `sum`: per case and
implementation the mean HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
MI355X_MICROARCH.md) against the algorithmic bytes (each operand read once, C written once).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D, FH, B = 768, 3072, 256
MF = (B // 2 + 3 * B // 64) * 197  # the larger forward chain's rows
CASES = [("fwd_qkv", "fwd", MF, 3 * D, D), ("fwd_fc2", "fwd", MF, D, FH), ("fwd_proj", "fwd", MF, D, D),
         ("dgrad_qkv", "dgrad", B * 197, D, 3 * D), ("dgrad_fc1", "dgrad", B * 197, D, FH),
         ("dgrad_proj", "dgrad", B * 197, D, D)]  # (name, kind, M, N out columns, K reduction)
REPS = 3


def run():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "vit-project_amd"))
    import torch
    from vit_amd import ops, _lib as L
    L.lib()
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    dev, bf = "cuda", torch.bfloat16
    fns = []
    for name, kind, M, N, K in CASES:
        if kind == "fwd":
            x = torch.randn(M, K, device=dev).to(bf)
            w = (torch.randn(N, K, device=dev) * 0.05).to(bf)
            b = torch.randn(N, device=dev)
            bb = b.to(bf)
            y = torch.empty(M, N, device=dev, dtype=bf)
            fns.append((lambda x=x, w=w, b=b, y=y: ops.linear_fwd(x, w, b, out=y),
                        lambda x=x, w=w, bb=bb, y=y: torch.addmm(bb, x, w.t(), out=y)))
        else:
            w = (torch.randn(K, N, device=dev) * 0.05).to(bf)  # the layer's weight [out = K, in = N]
            dy = torch.randn(M, K, device=dev).to(bf)
            dx = torch.empty(M, N, device=dev, dtype=bf)
            fns.append((lambda dy=dy, w=w, dx=dx: ops.linear_dgrad(dy, w, out_dtype=bf, out=dx),
                        lambda dy=dy, w=w, dx=dx: torch.matmul(dy, w, out=dx)))
    torch.cuda.synchronize()
    for ours, lib in fns:
        for fn in (ours, lib):
            for _ in range(REPS):
                fn()
            torch.cuda.synchronize()


def summarize(d):
    per = {}
    for pas in ("fetch", "write"):
        rows = defaultdict(dict)
        for f in glob.glob(os.path.join(d, pas, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    n = r["Kernel_Name"]
                    if "g4::kernel" in n or "Cijk" in n:
                        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
                        rows[int(r["Dispatch_Id"])]["name"] = n
        per[pas] = [rows[k] for k in sorted(rows)]
    out = []
    for ci, (name, kind, M, N, K) in enumerate(CASES):
        alg = (M * K + N * K + M * N) * 2
        rec = {"case": name, "M": M, "N": N, "K": K, "alg_MB": round(alg / 1e6, 1)}
        for ii, impl in enumerate(("g4", "hipblaslt")):
            lo = (2 * ci + ii) * REPS
            fe = [r.get("FETCH_SIZE", 0) for r in per["fetch"][lo:lo + REPS]]
            wr = [r.get("WRITE_SIZE", 0) for r in per["write"][lo:lo + REPS]]
            names = {r["name"][:40] for r in per["fetch"][lo:lo + REPS]}
            if len(fe) < REPS or len(wr) < REPS:
                rec[impl] = None
                continue
            fb, wb = 2 * 1024 * sum(fe) / REPS, 1024 * sum(wr) / REPS
            rec[impl] = {"kernel": sorted(names), "fetch_MB": round(fb / 1e6, 1), "write_MB": round(wb / 1e6, 1),
                         "hbm_over_alg": round((fb + wb) / alg, 3)}
        out.append(rec)
        print(json.dumps(rec))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
