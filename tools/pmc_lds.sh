#!/bin/bash
# LDS / issue counters of single GEMM shapes (tools/kernel_probe.py), one rocprofv3 pass per shape:
#   bash tools/pmc_lds.sh <out dir> <shape[:variant]> ...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
for sv in "$@"; do
  s=${sv%%:*}; v=${sv#*:}; [ "$v" = "$sv" ] && v=""
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS \
    SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d "$O/$sv" -o r \
    -- python3 tools/kernel_probe.py "$s" 4 $v > "$O/$sv.log" 2>&1 || { tail -5 "$O/$sv.log"; exit 1; }
  python3 - "$O/$sv" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
if not f: print("no counter csv", sys.argv[1]); sys.exit(0)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "gemm" not in r["Kernel_Name"] and "pp_kernel" not in r["Kernel_Name"] and "w4" not in r["Kernel_Name"]: continue
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(sys.argv[1].split("/")[-1], k, {a: int(b) for a, b in d.items()})
PY
done
