# attention phase stamps at the step shape
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 120 python -u tools/attn_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.json
timeout -k 10 120 python -u tools/bench_attn.py > $O/bench_attn.json 2>&1 || { tail $O/bench_attn.json; exit 1; }
cat $O/bench_attn.json
