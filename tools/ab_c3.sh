#!/bin/bash
# Same-box A/B of two library builds on config C3 (CLIP-HBA ViT-L/14 + DoRA step, tools/bench_clip.py):
#   bash tools/ab_c3.sh <base .so> [rounds]
set -o pipefail
BASE=$1; ROUNDS=${2:-2}
NEW=vit-project_amd/vit_amd/lib/libvit_hip.so
mkdir -p gpurun_out/ab_c3
for i in $(seq 1 $ROUNDS); do
  for lib in $BASE $NEW; do
    VIT_HIP_LIB=$lib timeout -k 10 300 python -u tools/bench_clip.py > gpurun_out/ab_c3/c3_$(basename $lib)_$i.json 2> gpurun_out/ab_c3/c3_$(basename $lib)_$i.err || { tail -5 gpurun_out/ab_c3/c3_$(basename $lib)_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['final_loss'])" gpurun_out/ab_c3/c3_$(basename $lib)_$i.json "$(basename $lib)#$i"
  done
done
