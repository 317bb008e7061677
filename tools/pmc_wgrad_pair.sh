# HBM traffic of the step's MLP weight-gradient pair (grouped launch + its slab-sum launch): separate
# FETCH_SIZE and WRITE_SIZE passes, summed per call by tools/pmc_traffic.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_pair
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r -- python3 tools/kernel_probe.py wgrad_pair 5 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r -- python3 tools/kernel_probe.py wgrad_pair 5 > /dev/null 2>&1 || exit 1
python3 tools/pmc_traffic.py $O pp_kernel2,colreduce_batch --out $O/traffic.json
