# CLIP C3 fp32 step kernel trace (config C3 at the reference's precision)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02v
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_clip.py --steps 4 --warmup 2 > $O/c3.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
cat $O/c3.json
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open([__import__('glob').glob('gpurun_out/r02v/prof/*kernel_stats.csv')][0][0])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['TotalDurationNs'])/tot*100:5.1f}% n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.1f}us {r['Name'][:100]}")
PY
