#!/bin/bash
# Closing measurements of a round, one call: full GPU suite + smoke, the default bench line, the step's
# kernel trace (summary, classes, phases), the step counter passes and the MLP weight-gradient pair's
# HBM bytes (both stamped with the weight-gradient kernel sources' hash).  Output under gpurun_out/final/.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/final
rm -rf $O; mkdir -p $O
bash tools/job_fulltest.sh || exit 1
cp gpurun_out/pytest_gpu_full.log gpurun_out/smoke.log $O/
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-c3 > $O/bench_underprof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_kernels.py "$T" 40 > $O/rocprof_step_summary.txt || exit 1
python3 tools/step_classes.py "$T" 3 --json $O/step_classes.json > /dev/null || exit 1
python3 tools/step_phases.py "$T" 3 --json $O/step_phases.json > /dev/null || exit 1
cp "$(find $O/prof -name "*kernel_stats.csv" | head -1)" $O/rocprof_kernel_stats.csv
P=$O/pmc
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$P/sq" -o r \
  -- python3 tools/step_probe.py 2 1 > "$P.sq.log" 2>&1 || { tail -5 "$P.sq.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o r \
  -- python3 tools/step_probe.py 2 1 > "$P.fetch.log" 2>&1 || { tail -5 "$P.fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o r \
  -- python3 tools/step_probe.py 2 1 > "$P.write.log" 2>&1 || { tail -5 "$P.write.log"; exit 1; }
python3 tools/pmc_step_classes.py "$P" --json $O/pmc_step_classes.json > /dev/null || exit 1
bash tools/pmc_wgrad_pair.sh || exit 1
cp gpurun_out/pmc_pair/traffic.json $O/pmc_traffic_wgrad_pair.json
rm -rf $O/prof $P
ls $O
