# Same-box A/B of two builds of the library: tools/ab_lib.sh <base .so> [rounds] [pytest -k filter]
# (correctness of the new build first, then kernel table and alternating bench runs)
set -o pipefail
BASE=$1; ROUNDS=${2:-2}; K=${3:-}
NEW=vit-project_amd/vit_amd/lib/libvit_hip.so
mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
  tail -1 gpurun_out/ab/pytest.log
fi
for lib in $BASE $NEW; do
  VIT_HIP_LIB=$lib timeout -k 10 200 python tools/bench_kernels.py > gpurun_out/ab/kern_$(basename $lib).jsonl 2>&1 || exit 1
done
for i in $(seq 1 $ROUNDS); do
  for lib in $BASE $NEW; do
    VIT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 40 --warmup 10 > gpurun_out/ab/bench_$(basename $lib)_$i.json || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab/bench_$(basename $lib)_$i.json "$(basename $lib)#$i"
  done
done
