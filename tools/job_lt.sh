# hipBLASLt plain GEMMs: parity test, then the full GPU suite, then an in-step A/B of the library classes
set -o pipefail
mkdir -p gpurun_out/lt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s -k "blaslt" --timeout 200 --timeout-method thread > gpurun_out/lt/pytest_lt.log 2>&1 || { tail -40 gpurun_out/lt/pytest_lt.log; exit 1; }
grep "bitwise" gpurun_out/lt/pytest_lt.log; tail -1 gpurun_out/lt/pytest_lt.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lt/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/lt/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/lt/pytest_gpu.log
bash tools/ab_env.sh gpurun_out/lt/ab 2 "VIT_GEMM_LIB=0" "-" "VIT_GEMM_LIB=3"
