#!/bin/bash
# Round 6: the whole GPU suite, one process, per-test time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_suite.txt 2>&1
rc=$?; tail -5 gpurun_out/r6_suite.txt; exit $rc
