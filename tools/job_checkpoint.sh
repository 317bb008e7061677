# closing checkpoint: GPU suite, smoke, step trace, counter passes on the current kernel sources, then the
# bench (which reads the fresh counter files, copied into this tree's profiles/r05 first)
set -o pipefail
bash tools/gpu_job.sh r5f tests smoke prof pmc && bash tools/pmc_wgrad_pair.sh && \
  cp gpurun_out/r5f/pmc_step_classes.json profiles/r05/pmc_step_classes_r05f.json && \
  cp gpurun_out/pmc_pair/traffic.json profiles/r05/pmc_traffic_wgrad_pair.json && \
  bash tools/gpu_job.sh r5f bench
