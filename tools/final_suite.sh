#!/bin/bash
# the round-end checks the driver runs: GPU suite and smoke, each under its own limit
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
