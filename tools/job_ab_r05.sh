#!/bin/bash
# Same-box A/B: the round-5 closing tree (hipBLASLt for the plain GEMMs, gpurun_ab/r05) against this tree
# (g4), interleaved, then this tree's input-gradient walk (band vs stride) and a kernel trace of the step.
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/ab_tree.sh gpurun_ab/r05 ${ROUNDS:-3} || exit 1
if [ -n "$MODES" ]; then
  bash tools/ab_bench.sh VIT_G4_MODE_DGRAD "0 1" 2 || exit 1
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g4 -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-c3 > gpurun_out/bench_g4_underprof.json 2> gpurun_out/prof_g4.err || exit 1
python3 tools/step_classes.py "$(find gpurun_out/prof_g4 -name "*kernel_trace.csv" | head -1)" 3
