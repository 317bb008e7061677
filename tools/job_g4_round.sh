#!/bin/bash
# g4 iteration job: kernel tests, stamps (normal and with timing switches), standalone step-shape bench,
# then in-step A/Bs: $AB (tools/ab_envs.sh arguments) and $ABTREE rounds against gpurun_ab/r05.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/g4
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "${TESTK:-g4}" > gpurun_out/g4/pytest_g4.log 2>&1 || { tail -30 gpurun_out/g4/pytest_g4.log; exit 1; }
tail -1 gpurun_out/g4/pytest_g4.log
: > gpurun_out/g4/stamps.jsonl
for d in ${STAMPS:-0:0}; do  # dbg:sched pairs
  timeout -k 10 200 python -u tools/g4_stamps.py --dbg ${d%%:*} --sched ${d##*:} --shapes ${STAMP_SHAPES:-fwd_qkv,fwd_fc2,dgrad_fc1,dgrad_qkv} >> gpurun_out/g4/stamps.jsonl || exit 1
done
cat gpurun_out/g4/stamps.jsonl
timeout -k 10 300 python -u tools/bench_g4.py --rounds 1 > gpurun_out/g4/bench_g4.jsonl || exit 1
cat gpurun_out/g4/bench_g4.jsonl
if [ -n "$AB" ]; then eval bash tools/ab_envs.sh $AB || exit 1; fi
if [ -n "$ABTREE" ]; then bash tools/ab_tree.sh gpurun_ab/r05 $ABTREE || exit 1; fi
exit 0
