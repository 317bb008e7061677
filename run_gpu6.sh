set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider -x > gpurun_out/t6.log 2>&1
rc=$?
echo "gpu tests rc=$rc"
tail -5 gpurun_out/t6.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bk6.log 2>&1
  echo "bk rc=$?"; cat gpurun_out/bk6.log | grep -v amdgpu.ids
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench6.log 2>&1
  echo "bench rc=$?"; tail -1 gpurun_out/bench6.log
fi
