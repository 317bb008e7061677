# Fused attention backward: parity tests, standalone timing (fused vs two-kernel), in-step A/B.
#   bash tools/gpu_attn.sh <out dir>
set -o pipefail
O=$1
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sdpa" > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAILED|rel" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for S in 0 1 0 1; do
  VIT_ATTN_BWD_SPLIT=$S timeout -k 10 120 python tools/bench_attn.py >> $O/attn.jsonl 2>&1 || { tail -5 $O/attn.jsonl; exit 1; }
done
cat $O/attn.jsonl
bash tools/ab_bench.sh VIT_ATTN_BWD_SPLIT "0 1" 2
