#!/bin/bash
# GPU job: g4 kernel tests, then the step-shape GEMM bench (tools/bench_g4.py).
set -o pipefail
mkdir -p gpurun_out/g4
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
  -k "g4" > gpurun_out/g4/pytest_g4.log 2>&1 || { tail -30 gpurun_out/g4/pytest_g4.log; exit 1; }
tail -3 gpurun_out/g4/pytest_g4.log
timeout -k 10 300 python -u tools/bench_g4.py --walks ${BENCH_ARGS} > gpurun_out/g4/bench_g4.jsonl 2> gpurun_out/g4/bench_g4.err \
  || { tail -20 gpurun_out/g4/bench_g4.err; exit 1; }
cat gpurun_out/g4/bench_g4.jsonl
