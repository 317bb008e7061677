#!/bin/bash
# One GPU job, steps chosen on the command line; every step has its own time limit and the job
# stops at the first failure (no GPU step runs after a fault, abort or timeout).
#   bash tools/gpu_job.sh <out dir under gpurun_out> <step> [<step> ...]
# steps:
#   tests       pytest -m gpu (full GPU suite)         tests:<k>  only tests matching -k <k>
#   smoke       __graft_entry__.smoke()
#   bench       default bench line (bench.py, N=1)     bench:<args> with extra bench.py arguments
#   prof        rocprofv3 kernel trace of the bench step + step summaries (trace_overlap, step_classes)
#   pmc         counter passes over tools/step_probe.py: SQ/GRBM (with kernel trace), FETCH_SIZE,
#               WRITE_SIZE -> pmc_step_classes.json (MFMA busy, HBM GB/s per kernel)
#   kernels     tools/bench_kernels.py (standalone kernel table)
#   c3          tools/bench_clip.py (config C3 leg alone)
#   wgrad       tools/bench_wgrad.py (weight-gradient kernels / pairs per variant)
#   w4b         tools/lab/w4b_lab.py (the two-workgroup-per-CU w4 loop vs the library forward / dgrad)
#   w4r         tools/lab/w4r_lab.py (register-staged w4 weight gradient vs the LDS-DMA one)
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== $step $(date +%T)"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
        > "$O/pytest.log" 2>&1 || fail tests "$O/pytest.log"
      tail -2 "$O/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail smoke "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python -u bench.py $arg > "$O/bench.json" 2> "$O/bench.err" || fail bench "$O/bench.err"
      cat "$O/bench.json" ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 3 --no-cpu --no-c3 > "$O/bench_prof.json" 2> "$O/prof.err" || fail prof "$O/prof.err"
      T=$(ls "$O"/prof/*kernel_trace.csv | head -1)
      python3 tools/trace_overlap.py "$T" 3 > "$O/step_summary.txt"
      python3 tools/step_classes.py "$T" 3 --json "$O/step_classes.json" > "$O/step_classes.txt"
      python3 tools/step_phases.py "$T" 3 --json "$O/step_phases.json" > /dev/null
      head -16 "$O/step_summary.txt"; cat "$O/step_classes.txt" ;;
    pmc)
      P="$O/pmc"
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$P/sq" -o r \
        -- python3 tools/step_probe.py 2 1 > "$P.sq.log" 2>&1 || fail pmc-sq "$P.sq.log"
      timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o r \
        -- python3 tools/step_probe.py 2 1 > "$P.fetch.log" 2>&1 || fail pmc-fetch "$P.fetch.log"
      timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o r \
        -- python3 tools/step_probe.py 2 1 > "$P.write.log" 2>&1 || fail pmc-write "$P.write.log"
      python3 tools/pmc_step_classes.py "$P" --json "$O/pmc_step_classes.json" ;;
    kernels)
      timeout -k 10 300 python tools/bench_kernels.py $arg > "$O/kernels.jsonl" 2>&1 || fail kernels "$O/kernels.jsonl"
      tail -30 "$O/kernels.jsonl" ;;
    wgrad)
      timeout -k 10 300 python -u tools/bench_wgrad.py $arg > "$O/wgrad.jsonl" 2>&1 || fail wgrad "$O/wgrad.jsonl"
      cat "$O/wgrad.jsonl" ;;
    w4b)
      timeout -k 10 300 python -u tools/lab/w4b_lab.py $arg > "$O/w4b.jsonl" 2>&1 || fail w4b "$O/w4b.jsonl"
      cat "$O/w4b.jsonl" ;;
    w4r)
      timeout -k 10 300 python -u tools/lab/w4r_lab.py $arg > "$O/w4r.jsonl" 2>&1 || fail w4r "$O/w4r.jsonl"
      cat "$O/w4r.jsonl" ;;
    c3)
      timeout -k 10 400 python -u tools/bench_clip.py $arg > "$O/c3.json" 2> "$O/c3.err" || fail c3 "$O/c3.err"
      cat "$O/c3.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
