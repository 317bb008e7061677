set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
