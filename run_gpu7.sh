set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for k in wgrad_fc1 fwd_fc1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_$k -o p1 --output-format csv -- python3 $R/tools/kernel_probe.py $k 3 > $R/gpurun_out/pmc_$k.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_$k -o p2 --output-format csv -- python3 $R/tools/kernel_probe.py $k 3 >> $R/gpurun_out/pmc_$k.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc_$k -o p3 --output-format csv -- python3 $R/tools/kernel_probe.py $k 3 >> $R/gpurun_out/pmc_$k.log 2>&1 || exit 1
done
echo ok
