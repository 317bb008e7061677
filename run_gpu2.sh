set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/p.log 2>&1
rc2=$?
echo "parity rc=$rc2"
tail -40 gpurun_out/p.log
if [ $rc2 -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
  rc3=$?
  echo "bench rc=$rc3"
  tail -3 gpurun_out/bench.log
  if [ $rc3 -eq 0 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-graph > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
    echo "prof rc=$?"
    tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof1.log
  fi
fi
