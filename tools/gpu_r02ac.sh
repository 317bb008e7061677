# round-2 final pass: full GPU suite, forward split re-tune, default bench line, step kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu > $O/bench_prof.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -1)
python3 tools/step_phases.py $T 3 --json $O/step_phases.json > /dev/null
python3 tools/trace_overlap.py $T 3 > $O/step_summary.txt
python3 tools/step_classes.py $T 3 --json $O/step_classes.json > /dev/null
head -3 $O/step_summary.txt
