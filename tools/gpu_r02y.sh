# attention: accumulator-initialised backward + tree max/sum forward vs HEAD (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02y
mkdir -p $O
B=vit-project_amd/vit_amd/lib/libvit_hip_base.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sdpa" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in $B vit-project_amd/vit_amd/lib/libvit_hip.so; do
  VIT_HIP_LIB=$lib timeout -k 10 120 python -u tools/bench_attn.py > $O/attn_$(basename $lib).json 2>/dev/null || exit 1
  echo "$(basename $lib) $(cat $O/attn_$(basename $lib).json)"
done
timeout -k 10 120 python -u tools/attn_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.json
for i in 1 2; do
  for lib in $B vit-project_amd/vit_amd/lib/libvit_hip.so; do
    VIT_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu --steps 40 --warmup 10 > $O/bench_$(basename $lib)_$i.json || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_$(basename $lib)_$i.json "$(basename $lib)#$i"
  done
done
