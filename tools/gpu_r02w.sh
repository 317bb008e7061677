# f32 MFMA attention forward: kernel tests, full GPU suite, C3 fp32 A/B against the scalar kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sdpa" -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in 1 0; do
  VIT_ATTN_F32_GENERIC=$v timeout -k 10 300 python -u tools/bench_clip.py > $O/c3_${v}_${i}.json 2>/dev/null || exit 1
  echo "generic=$v#$i $(python3 -c "import json; d=json.load(open('$O/c3_${v}_${i}.json')); print(d['value'], d['ms_per_step'])")"
done
done
