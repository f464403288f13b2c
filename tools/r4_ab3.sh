#!/bin/bash
# Round-4 batch 3: the GPU suite (up to 10 failures listed), decode stamps, the default bench line.
bash tools/gpu_steps.sh \
tests 800 'python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread' \
stamps 120 'python -u tools/decode_stamps.py q6_k_28672x8192_m1 q6_k_8192x28672_m1 q4_k_4096x11008_m1' \
bench 300 'python -u bench.py --steps 20 --warmup 5'
