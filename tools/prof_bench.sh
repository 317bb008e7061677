#!/bin/bash
# Bench line + rocprofv3 kernel trace/stats of the same bench command (outputs under gpurun_out/).
#   bash tools/prof_bench.sh <tag>
set -o pipefail
tag=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python3 -u bench.py > "gpurun_out/bench_$tag.json" 2> "gpurun_out/bench_$tag.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$tag" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu > "gpurun_out/bench_${tag}_underprof.json" 2> "gpurun_out/prof_$tag.err"
