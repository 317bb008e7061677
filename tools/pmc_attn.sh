# rocprofv3 counter passes (one per block budget) over the attention kernels; outputs under gpurun_out/pmc_attn
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_attn
for w in sdpa_fwd sdpa_bwd; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/$w/fetch -o r -- python3 tools/kernel_probe.py $w 5 > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/$w/write -o r -- python3 tools/kernel_probe.py $w 5 > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/$w/sq -o r --output-format csv -- python3 tools/kernel_probe.py $w 5 > /dev/null 2>&1 || exit 1
done
