# HBM traffic of the roofline kernel (fc1 forward, bias+GELU epilogue): separate FETCH_SIZE and
# WRITE_SIZE passes (MI355X_MICROARCH.md HBM section), summarised by tools/pmc_traffic.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_fc1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r -- python3 tools/kernel_probe.py fwd_fc1_gelu 5 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r -- python3 tools/kernel_probe.py fwd_fc1_gelu 5 > /dev/null 2>&1 || exit 1
python3 tools/pmc_traffic.py $O gemm_kernel --out $O/traffic.json > /dev/null
