#!/usr/bin/env bash
# Full GPU parity suite + smoke, each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
