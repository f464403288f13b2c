#!/bin/bash
# Round-4 batch 10: stream-K for every grouped plan: the grouped tests and the layer 5..512.
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_gemm_grouped.py tests/test_gpu_routes.py -q --timeout 120 --timeout-method thread' \
layer 500 "python -u tools/layer_time.py 5,8,16,24,32,48,64,96,128,192,256,512 --grouped-only && python -u tools/layer_time.py 24,32,64,128 --grouped-only --tune GQ_SGEMM_STREAMK=0"
