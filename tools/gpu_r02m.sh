# first-wave desync of the 256x256 GEMM: standalone kernel table + step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02m
mkdir -p $O
for d in 0 12000 24000 40000; do
  VIT_GEMM_DESYNC=$d timeout -k 10 200 python tools/bench_kernels.py > $O/kern_$d.jsonl 2>&1 || { tail -3 $O/kern_$d.jsonl; exit 1; }
  echo "desync=$d $(python3 -c "
import json,sys
for l in open('$O/kern_$d.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l)
    n=d.get('name','')
    if n.startswith('fwd_') or 'gelubwd' in n: print(n, d.get('ms'), end='; ')
")"
done
for i in 1 2; do
for d in 0 24000; do
  VIT_GEMM_DESYNC=$d timeout -k 10 200 python -u bench.py --no-cpu --steps 40 --warmup 10 > $O/bench_$d_$i.json || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/bench_$d_$i.json "desync=$d#$i"
done
done
