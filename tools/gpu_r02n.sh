# fused residual-add LayerNorm: full GPU suite, then step A/B against the EPI_RESID epilogues
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_bench.sh VIT_FUSED_RESID "0 1" 2
