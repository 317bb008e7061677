set -o pipefail
bash tools/gpu_job.sh r5c tests smoke bench prof pmc && bash tools/pmc_wgrad_pair.sh && cat gpurun_out/pmc_pair/traffic.json
