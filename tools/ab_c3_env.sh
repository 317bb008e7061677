#!/bin/bash
# Interleaved same-box A/B of environment settings on config C3 (tools/bench_clip.py), fp32 and bf16:
#   bash tools/ab_c3_env.sh <rounds> "<env assignments A>" "<env assignments B>" ...   ("-" = none)
set -o pipefail
R=$1; shift
O=gpurun_out/ab_c3_env
mkdir -p "$O"
for i in $(seq 1 "$R"); do
  k=0
  for cfg in "$@"; do
    k=$((k + 1))
    envs=(); [ "$cfg" != "-" ] && read -r -a envs <<< "$cfg"
    for dt in f32 bf16; do
      env "${envs[@]}" timeout -k 10 300 python -u tools/bench_clip.py --dtype $dt > "$O/c3_${k}_${dt}_$i.json" 2> "$O/c3_${k}_${dt}_$i.err" || { tail -5 "$O/c3_${k}_${dt}_$i.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['final_loss'])" "$O/c3_${k}_${dt}_$i.json" "[$cfg] $dt #$i"
    done
  done
done
