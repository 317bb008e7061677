# round-2 GPU pass A: full GPU test suite, default bench line, kernel trace of the bench step,
# standalone kernel table (ours vs hipBLASLt).  Outputs under gpurun_out/r02a/.
set -o pipefail
O=gpurun_out/r02a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu --no-probe > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
timeout -k 10 200 python tools/bench_kernels.py > $O/kernels.jsonl 2>&1 || exit 1
timeout -k 10 200 python tools/bench_kernels.py --torch > $O/kernels_torch.jsonl 2>&1 || exit 1
echo done
