# round-2 pass E: PMC traffic of the roofline kernel (fc1 weight gradient: pp_kernel + slab reduce),
# step kernel trace of the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r -- python3 tools/kernel_probe.py wgrad_fc1 5 > /dev/null 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r -- python3 tools/kernel_probe.py wgrad_fc1 5 > /dev/null 2>&1 || { echo write failed; exit 1; }
python3 tools/pmc_traffic.py $O pp_kernel,splitk_reduce --out $O/pmc_traffic_wgrad_fc1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu > $O/bench_prof.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
python3 tools/trace_overlap.py $(ls $O/prof/*kernel_trace.csv | head -1) 3 > $O/step_summary.txt
python3 tools/step_classes.py $(ls $O/prof/*kernel_trace.csv | head -1) 3 --json $O/step_classes.json > /dev/null
head -12 $O/step_summary.txt
