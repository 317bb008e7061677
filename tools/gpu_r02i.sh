# two-tiles-per-wave fused attention backward: parity, A/B timing vs the one-tile form, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sdpa" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
for v in 1 0; do
  VIT_ATTN_BWD_ONE_TILE=$v timeout -k 10 120 python -u tools/bench_attn.py > $O/bench_attn_$v.json 2>/dev/null || exit 1
  echo "one_tile=$v $(cat $O/bench_attn_$v.json)"
done
done
for v in 1 0; do
VIT_ATTN_BWD_ONE_TILE=$v timeout -k 10 120 python -u tools/attn_stamps.py > $O/stamps_$v.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
echo "one_tile=$v"; cat $O/stamps_$v.json
done
