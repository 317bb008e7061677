#!/bin/bash
# HBM bytes per launch, g4 vs hipBLASLt at the step's plain-GEMM shapes (tools/pmc_g4_lib.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/pmc_g4lib
rm -rf $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o r -- python3 tools/pmc_g4_lib.py run > /dev/null 2> $O.fetch.err || { tail -5 $O.fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o r -- python3 tools/pmc_g4_lib.py run > /dev/null 2> $O.write.err || { tail -5 $O.write.err; exit 1; }
python3 tools/pmc_g4_lib.py sum $O
