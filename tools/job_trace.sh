#!/bin/bash
# Kernel trace of the bench step under the current environment (tag = $1), per-kernel summary printed.
set -o pipefail
tag=${1:-t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-c3 > gpurun_out/bench_${tag}_underprof.json 2> gpurun_out/prof_$tag.err || exit 1
python3 tools/trace_kernels.py "$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)"
