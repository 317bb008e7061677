set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_bench.sh VIT_FWD_HALF_DELTA "8 12 16" 3 || exit 1
bash tools/ab_bench.sh VIT_FWD_STAGGER "0 1 3" 2
