#!/bin/bash
# Round-4 batch 9: stream-K by default for the grouped GEMM's 16-token tiles, LayerMix grouped from
# 5 tokens: the grouped tests, the layer at 5..16 (default) and 24..64 default vs stream-K forced.
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_gemm_grouped.py tests/test_gpu_routes.py tests/test_gpu_bench_strong.py -q --timeout 120 --timeout-method thread' \
layer 500 "python -u tools/layer_time.py 5,8,12,16,24,32,48,64 --grouped-only && python -u tools/layer_time.py 24,32,48,64 --grouped-only --tune GQ_SGEMM_STREAMK=1 && python -u tools/layer_time.py 8,16 --grouped-only --act fp8 && python -u tools/layer_time.py 8,16 --grouped-only --act fp8 --gemm-min 100"
