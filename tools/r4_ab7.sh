#!/bin/bash
# Round-4 batch 7: resident GEMM (forced, several rounds) vs the default at 64/128 tokens; the
# layer at 8..48 tokens grouped vs per call; the routing tests.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 200 'python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_rgemm.py -q --timeout 120 --timeout-method thread' \
rg64 300 "python -u $RC --steps-only --configs q4_k_11008x4096_m64,q4_k_22016x4096_m64,q4_k_4096x11008_m64,q8_0_11008x4096_m64,q6_k_11008x4096_m64,q4_k_11008x4096_m128,q4_k_22016x4096_m128,q6_k_4096x11008_m128,q4_k_11008x4096_m48 --rounds 2 --variants rg=GQ_RGEMM:1+GQ_SKINNY:0,def=GQ_SGEMM:-1" \
layer 300 'python -u tools/layer_time.py 8,16,24,32,48 --grouped-only && python -u tools/layer_time.py 24,32,48,64 --grouped-only --tune GQ_RGEMM=1'
