#!/bin/bash
# Round 6, batch 3: the decode two-row pass A/B (tools/r6_dpair.sh), then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r6_dpair.sh || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_gpu_suite.txt 2>&1
rc=$?; tail -5 gpurun_out/r6_gpu_suite.txt; exit $rc
