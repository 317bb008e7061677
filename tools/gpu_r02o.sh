# step kernel trace: forward / backward split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu > $O/bench_prof.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -1)
python3 tools/step_phases.py $T 3 --json $O/step_phases.json
python3 tools/trace_overlap.py $T 3 > $O/step_summary.txt
python3 tools/step_classes.py $T 3 --json $O/step_classes.json > /dev/null
head -3 $O/step_summary.txt
