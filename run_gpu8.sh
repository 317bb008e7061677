set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python tools/bench_kernels.py --sweep 1,2,5 --reps 10 > gpurun_out/sweep8.log 2>&1
echo "sweep rc=$?"; grep SUMMARY gpurun_out/sweep8.log; grep -v amdgpu gpurun_out/sweep8.log | awk -F'max_rel_vs_v0' '{print $2}' | sort | tail -3
