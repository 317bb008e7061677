set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 120 python -u tools/attn_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.json
