#!/bin/bash
# Same-box A/B of the bench step between another source tree (its own bench.py and library, e.g. the
# previous round's closing commit extracted with git archive and built in place) and this tree:
#   bash tools/ab_tree.sh <other tree dir> [rounds]
set -o pipefail
OTHER=$1; ROUNDS=${2:-3}
mkdir -p gpurun_out/ab_tree
export PYTHONUNBUFFERED=1
ROOT=$(pwd)
TW="python3 $ROOT/tools/telemetry_wrap.py"
unset VIT_HIP_LIB
for i in $(seq 1 $ROUNDS); do
  ( cd "$OTHER" && timeout -k 10 300 $TW $ROOT/gpurun_out/ab_tree/other_$i.tel -- python -u bench.py --no-cpu --no-c3 --steps 40 --warmup 10 ) \
    > gpurun_out/ab_tree/other_$i.json 2> gpurun_out/ab_tree/other_$i.err || { tail -5 gpurun_out/ab_tree/other_$i.err; exit 1; }
  timeout -k 10 300 $TW gpurun_out/ab_tree/this_$i.tel -- python -u bench.py --no-cpu --no-c3 --steps 40 --warmup 10 \
    > gpurun_out/ab_tree/this_$i.json 2> gpurun_out/ab_tree/this_$i.err || { tail -5 gpurun_out/ab_tree/this_$i.err; exit 1; }
  for t in other this; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[3])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('final_loss'), t)" \
      gpurun_out/ab_tree/${t}_$i.json "$t#$i" gpurun_out/ab_tree/${t}_$i.tel
  done
done
