#!/bin/bash
# Round 6 closing measurement: FETCH_SIZE traffic per config, PMC passes, the default bench line
# (+ --detail), and rocprofv3 --kernel-trace --stats over the same command (tools/gpu.sh round);
# then smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh round || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round_smoke.txt 2>&1; rc=$?
cat gpurun_out/round_smoke.txt; exit $rc
