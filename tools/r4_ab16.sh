#!/bin/bash
# Round-4 batch 16: Q4_K 16-token tiles on per-wave weight rings (GQ_SGEMM_WRING): same-bits tests,
# the layer, single-matrix streaming steps.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_gemm_grouped.py -q -k "schedule" --timeout 120 --timeout-method thread' \
layer 400 "python -u tools/layer_time.py 5,8,16 --grouped-only && python -u tools/layer_time.py 5,8,16 --grouped-only --tune GQ_SGEMM_WRING=1" \
steps 300 "python -u $RC --steps-only --rounds 3 --variants full=GQ_RGEMM:0+GQ_SKINNY:0+GQ_SGEMM:1,wring=GQ_RGEMM:0+GQ_SKINNY:0+GQ_SGEMM:1+GQ_SGEMM_WRING:1,def=GQ_SGEMM:-1 --configs q4_k_11008x4096_m16,q4_k_4096x11008_m16,q4_k_4096x4096_m16,q4_k_22016x4096_m16"
