#!/bin/bash
# HBM traffic of the fc2 input gradient with and without its GELU' epilogue (act' read, VIT r04 verdict
# item 4): FETCH_SIZE / WRITE_SIZE in separate passes per case; the difference of the two FETCHes is the
# act' read, a known 310 MB (50432 x 3072 bf16, 16-B row-contiguous loads), which calibrates the x2
# FETCH correction for this kernel's access widths.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_fc2dg
for c in dgrad_fc2_gelu dgrad_fc2_plain; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$c/fetch -o r -- python3 tools/kernel_probe.py $c 5 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$c/write -o r -- python3 tools/kernel_probe.py $c 5 > /dev/null 2>&1 || exit 1
  python3 tools/pmc_traffic.py $O/$c gemm_kernel --out $O/$c.json > /dev/null || exit 1
done
python3 - <<'PY'
import json
g = json.load(open("gpurun_out/pmc_fc2dg/dgrad_fc2_gelu.json")); p = json.load(open("gpurun_out/pmc_fc2dg/dgrad_fc2_plain.json"))
raw = lambda d: d["FETCH_SIZE_KiB_avg"] * 1024
act = 50432 * 3072 * 2
res = {"gelu_fetch_raw": raw(g), "plain_fetch_raw": raw(p), "act_prime_bytes": act,
       "fetch_raw_diff": raw(g) - raw(p), "diff_over_act_raw": (raw(g) - raw(p)) / act,
       "gelu_write": g["write_bytes"], "plain_write": p["write_bytes"],
       "operand_bytes_algorithmic": 50432 * 768 * 2 + 3072 * 768 * 2}
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/pmc_fc2dg/calibration.json", "w"), indent=1)
PY
