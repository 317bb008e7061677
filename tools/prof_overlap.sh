# kernel trace of the default (two-stream) bench step; outputs under gpurun_out/prof_ovl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ovl -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu > gpurun_out/bench_ovl.json 2> gpurun_out/prof_ovl.err
