set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider -x > gpurun_out/t9.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
tail -5 gpurun_out/t9.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bk9.log 2>&1
  echo "bk rc=$?"; grep -v amdgpu.ids gpurun_out/bk9.log | cut -c1-100
  timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench9.log 2>&1
  echo "bench rc=$?"; tail -1 gpurun_out/bench9.log | cut -c1-260
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof9 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-graph > $GRAFT_REPO_ROOT/gpurun_out/prof9.log 2>&1
  echo "prof rc=$?"
fi
