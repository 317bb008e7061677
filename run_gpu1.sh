set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/k.log 2>&1
rc=$?
echo "kernels rc=$rc"
tail -30 gpurun_out/k.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider > gpurun_out/p.log 2>&1
  rc2=$?
  echo "parity rc=$rc2"
  tail -30 gpurun_out/p.log
  if [ $rc2 -le 1 ]; then
    timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
    echo "bench rc=$?"
    tail -5 gpurun_out/bench.log
  fi
fi
