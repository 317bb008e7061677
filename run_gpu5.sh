set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -x > gpurun_out/t5.log 2>&1
rc=$?
echo "kernel tests rc=$rc"
tail -5 gpurun_out/t5.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bk5.log 2>&1
  echo "bk rc=$?"; cat gpurun_out/bk5.log | grep -v amdgpu.ids
fi
