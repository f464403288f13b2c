#!/bin/bash
# LayerMix fusion: parity tests, then the layer sweep fused vs unfused
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k layer_mix tests/test_gpu_fp8.py > gpurun_out/layer_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --layer-only --steps 200 --warmup 10 > gpurun_out/layer_sweep.json 2> gpurun_out/layer_sweep.err
