#!/bin/bash
# Same-box A/B of whole environment settings on the step bench, interleaved:
#   bash tools/ab_envs.sh rounds "NAME1:VAR=v,VAR=v" "NAME2:..." ...   (an empty setting list = defaults)
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out/ab_envs
for i in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%:*}; vars=${spec#*:}
    envs=()
    IFS=',' read -ra kv <<< "$vars"
    for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --no-cpu --no-c3 --steps 30 --warmup 8 \
      > "gpurun_out/ab_envs/${name}_$i.json" 2> "gpurun_out/ab_envs/${name}_$i.err" || { tail -5 "gpurun_out/ab_envs/${name}_$i.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      "gpurun_out/ab_envs/${name}_$i.json" "$name#$i"
  done
done
