#!/bin/bash
# Kernel traces of the bench step for this tree and the round-5 tree (gpurun_ab/r05), same box, plus the
# g4 input gradient on W^T (tools/bench_g4.py --wt).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_this -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-c3 > gpurun_out/bench_this_underprof.json 2> gpurun_out/prof_this.err || exit 1
( cd gpurun_ab/r05 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r05" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-c3 > "$GRAFT_REPO_ROOT/gpurun_out/bench_r05_underprof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_r05.err" ) || exit 1
echo "== this"; python3 tools/trace_kernels.py "$(find gpurun_out/prof_this -name "*kernel_trace.csv" | head -1)" 16
echo "== r05"; python3 tools/trace_kernels.py "$(find gpurun_out/prof_r05 -name "*kernel_trace.csv" | head -1)" 16
