# round-2 GPU pass C: fp8 attention tests + the kernels/model tests it touches
set -o pipefail
O=gpurun_out/r02c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8_attention.py tests/test_gpu_kernels.py tests/test_clip.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $O/pytest.log | grep -E "fp8|FAILED|Error" | head -40; tail -2 $O/pytest.log
exit $rc
