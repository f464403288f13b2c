#!/bin/bash
# sharded C ABI: GPU tests, then the N > 1 bench rehearsal (native assemble inside the graph)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 120 --timeout-method thread \
  -k "assemble or sharded" > gpurun_out/shard_test.log 2>&1 || { tail -40 gpurun_out/shard_test.log; exit 1; }
grep -E "passed|failed" gpurun_out/shard_test.log | tail -3
bash tools/dist_rehearsal.sh > gpurun_out/dist_rehearsal.log 2>&1 || { tail -30 gpurun_out/dist_rehearsal.log; exit 2; }
grep -o '"metric[^}]*' gpurun_out/dist_rehearsal.log | cut -c1-200
