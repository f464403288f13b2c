#!/bin/bash
# Round-4 closing call (second): the whole GPU suite, the round-end measurements
# (tools/gpu.sh round) and the layer sweep.
bash tools/gpu_steps.sh tests 400 'python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread' \
  round 900 'bash tools/gpu.sh round' \
  layer 300 'python -u tools/layer_time.py 1,2,4,5,8,16,32,64,128,256,512 && python -u tools/layer_time.py 1,2,8,16,128 --grouped-only --act fp8'
