set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/t3.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -15 gpurun_out/t3.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/bench3.log 2>&1
  rc3=$?
  echo "bench rc=$rc3"
  tail -2 gpurun_out/bench3.log
  if [ $rc3 -eq 0 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-graph > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1
    echo "prof rc=$?"
  fi
fi
