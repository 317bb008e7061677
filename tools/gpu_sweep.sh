# GEMM configuration sweep: correctness of every forced variant, then per-shape timings.
#   bash tools/gpu_sweep.sh <out dir> <comma variant list>
set -o pipefail
O=$1; V=$2
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_config or f32_mfma or linear" > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/bench_kernels.py --sweep="$V" > $O/sweep.jsonl 2>&1 || { tail -5 $O/sweep.jsonl; exit 1; }
grep SUMMARY $O/sweep.jsonl
