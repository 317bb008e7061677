#!/bin/bash
# GEMM kernel table under several environments (library builds via VIT_HIP_LIB, VIT_GEMM_* knobs),
# interleaved on one box:  bash tools/sched_sweep.sh <out dir> <variants> "<env A>" "<env B>" ...
# ("-" = no extra environment; variants as bench_kernels.py --sweep, -1 = per-shape default)
set -o pipefail
O=gpurun_out/$1; V=$2; shift 2
mkdir -p "$O"
k=0
for cfg in "$@"; do
  k=$((k + 1))
  envs=(); [ "$cfg" != "-" ] && read -r -a envs <<< "$cfg"
  env "${envs[@]}" timeout -k 10 200 python tools/bench_kernels.py --sweep="$V" > "$O/kern_$k.jsonl" 2>&1 || { tail -5 "$O/kern_$k.jsonl"; exit 1; }
  echo "[$cfg] $(tail -1 "$O/kern_$k.jsonl")"
done
