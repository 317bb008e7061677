# fused residual LayerNorms in fp32 compute: full GPU suite (f32 golden tests must stay at their
# tolerances), C3 fp32 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in 0 1; do
  VIT_FUSED_RESID_F32=$v timeout -k 10 300 python -u tools/bench_clip.py > $O/c3_${v}_${i}.json 2>/dev/null || exit 1
  echo "fused_f32=$v#$i $(python3 -c "import json; d=json.load(open('$O/c3_${v}_${i}.json')); print(d['value'], d['ms_per_step'], d['final_loss'])")"
done
done
