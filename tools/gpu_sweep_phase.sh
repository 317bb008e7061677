set -o pipefail
mkdir -p gpurun_out/sw3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_config" > gpurun_out/sw3/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/sw3/pytest.log | head -20; exit 1; }
tail -1 gpurun_out/sw3/pytest.log
for ph in 0 2 6; do
  VIT_GEMM_PHASE=$ph timeout -k 10 300 python tools/bench_kernels.py --sweep=5,1605,11,12 > gpurun_out/sw3/sweep_ph$ph.jsonl 2>&1 || exit 1
done
