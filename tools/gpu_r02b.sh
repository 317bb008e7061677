# round-2 GPU pass B: kernel / CLIP / parity tests after the f32 MFMA GEMM, DoRA dropout and
# AdamW changes; C3 step in both dtypes.  Outputs under gpurun_out/r02b/.
set -o pipefail
O=gpurun_out/r02b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python tools/bench_clip.py --dtype f32 --steps 5 --warmup 2 > $O/clip_f32.json 2>&1 || { tail $O/clip_f32.json; exit 1; }
timeout -k 10 200 python tools/bench_clip.py --dtype bf16 --steps 10 --warmup 3 > $O/clip_bf16.json 2>&1 || exit 1
grep metric $O/clip_f32.json $O/clip_bf16.json
