#!/bin/bash
# Round 6: the grouped / layer / stream GPU tests after the last source clean-up.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_kstream.py tests/test_gpu_gemm_grouped.py \
  tests/test_gpu_ilc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_check.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_check.txt; exit $rc
