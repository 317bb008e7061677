# CLIP bf16 visual tower with the fused residual LayerNorms: CLIP GPU tests, C3 bf16 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_clip.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in 0 1; do
  VIT_FUSED_RESID=$v timeout -k 10 300 python -u tools/bench_clip.py --dtype bf16 > $O/c3b_${v}_${i}.json 2>/dev/null || exit 1
  echo "fused=$v#$i $(python3 -c "import json; d=json.load(open('$O/c3b_${v}_${i}.json')); print(d['value'], d['ms_per_step'])")"
done
done
