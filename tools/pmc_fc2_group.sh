#!/bin/bash
# fc2 GELU' input gradient (V1): operand FETCH and duration per tile-walk band (VIT_GEMM_GROUP_DGRAD = row
# tiles per band, 0 = row-major), the round-4 verdict's re-read item; one FETCH_SIZE pass (+ kernel trace) each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_fc2g
mkdir -p $O
for g in 0 4 8 16; do
  VIT_GEMM_GROUP_DGRAD=$g timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/g$g -o r \
    -- python3 tools/kernel_probe.py dgrad_fc2_gelu 5 > $O/g$g.log 2>&1 || { tail -5 $O/g$g.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
out = {}
for g in (0, 4, 8, 16):
    d = f"gpurun_out/pmc_fc2g/g{g}"
    cc = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    f = [float(r["Counter_Value"]) for r in csv.DictReader(open(cc[0])) if "gemm_kernel" in r["Kernel_Name"]]
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(kt[0])) if "gemm_kernel" in r["Kernel_Name"]]
    out[g] = {"fetch_raw_MB_per_launch": round(sum(f) / len(f) * 1024 / 1e6, 1), "us_per_launch": round(sum(t[1:]) / max(1, len(t) - 1), 1)}
out["note"] = "FETCH_SIZE raw (KiB x 1024); act' read 310 MB of it; operands algorithmic 82 MB (dY 77.5 + W 4.7)"
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/pmc_fc2g/summary.json", "w"), indent=1)
PY
