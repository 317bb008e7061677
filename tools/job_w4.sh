# round 5 GPU job: the GPU suite, the weight-gradient kernels, a short bench (each step under its own limit)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r5_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5_pytest_gpu.log
timeout -k 10 300 python -u tools/bench_wgrad.py > gpurun_out/r5_bench_wgrad.jsonl 2>&1 || { tail -20 gpurun_out/r5_bench_wgrad.jsonl; exit 1; }
cat gpurun_out/r5_bench_wgrad.jsonl
timeout -k 10 300 python -u bench.py --no-c3 --no-cpu --steps 20 --warmup 10 > gpurun_out/r5_bench_a.json 2>&1 || { tail -20 gpurun_out/r5_bench_a.json; exit 1; }
tail -1 gpurun_out/r5_bench_a.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:700])"
