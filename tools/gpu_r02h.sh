# fused attention backward over several (b, h) items per workgroup: parity + timing + stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sdpa" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for it in 1 2 4 3 6; do
  VIT_ATTN_BWD_ITEMS=$it timeout -k 10 120 python -u tools/bench_attn.py > $O/bench_attn_$it.json 2>/dev/null || exit 1
  echo "items=$it $(cat $O/bench_attn_$it.json)"
done
timeout -k 10 120 python -u tools/attn_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.json
