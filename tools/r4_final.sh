#!/bin/bash
# Round-4 closing call: the stream-K layer sweep (ab10), the layer PMC (ab11), the whole GPU suite,
# then the round-end measurements (tools/gpu.sh round).  Each step under its own limit; a fault
# or time limit ends the script.
bash tools/r4_ab10.sh || exit $?
timeout -k 10 420 bash tools/r4_ab11.sh > gpurun_out/ab11.txt 2>&1; rc=$?; echo "ab11 rc=$rc"; tail -3 gpurun_out/ab11.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_steps.sh tests 400 'python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread' \
  round 900 'bash tools/gpu.sh round'
