#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_paths.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fp8_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/fp8_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert|^E " gpurun_out/fp8_pytest.log | head -30; exit $rc; }
