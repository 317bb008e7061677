set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_novl -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu --no-overlap > gpurun_out/bench_novl.json 2> gpurun_out/prof_novl.err
