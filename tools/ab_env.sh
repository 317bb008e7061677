#!/bin/bash
# Interleaved same-box A/B of environment settings on the step bench (bench.py --no-cpu --no-c3):
#   bash tools/ab_env.sh <out dir> <rounds> "<env assignments A>" "<env assignments B>" ...
# e.g. bash tools/ab_env.sh gpurun_out/ab 2 "VIT_COL_BATCH=0" "VIT_COL_BATCH=1"
# ("-" = no extra environment).  Stops at the first failing run.
set -o pipefail
O=$1; R=$2; shift 2
mkdir -p "$O"
for i in $(seq 1 "$R"); do
  k=0
  for cfg in "$@"; do
    k=$((k + 1))
    envs=(); [ "$cfg" != "-" ] && read -r -a envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --no-cpu --no-c3 --steps 40 --warmup 10 > "$O/ab_${k}_$i.json" 2> "$O/ab_${k}_$i.err" || { tail -5 "$O/ab_${k}_$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); b=d.get('box',{}); print(sys.argv[2], d['value'], d['ms_per_step'], 'MHz', b.get('current_gfxclk',{}).get('mean'), 'W', b.get('current_socket_power',{}).get('mean'))" "$O/ab_${k}_$i.json" "[$cfg]#$i"
  done
done
