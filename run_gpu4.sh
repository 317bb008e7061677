set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -x > gpurun_out/t4.log 2>&1
rc=$?
echo "kernel tests rc=$rc"
tail -15 gpurun_out/t4.log
if [ $rc -eq 0 ]; then
  timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/t4p.log 2>&1
  echo "parity rc=$?"; tail -3 gpurun_out/t4p.log
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench4.log 2>&1
  rc3=$?
  echo "bench rc=$rc3"
  tail -1 gpurun_out/bench4.log
  if [ $rc3 -eq 0 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-graph > $GRAFT_REPO_ROOT/gpurun_out/prof4.log 2>&1
    echo "prof rc=$?"
  fi
fi
