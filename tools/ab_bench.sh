#!/bin/bash
# A/B of an environment knob on the step bench: tools/ab_bench.sh VAR "v1 v2" [rounds]
# Each run is time-limited; the script stops at the first failing run.
set -e
var=$1; vals=$2; rounds=${3:-2}
mkdir -p gpurun_out
for i in $(seq 1 "$rounds"); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 200 python -u bench.py --no-cpu --steps 30 > "gpurun_out/ab_${var}_${v}_$i.json"
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      "gpurun_out/ab_${var}_${v}_$i.json" "$var=$v#$i"
  done
done
