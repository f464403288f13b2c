#!/bin/bash
# Round-4 batch 12: XCD-aware workgroup order for the resident / streaming GEMMs (GQ_RGEMM_XCD,
# GQ_SGEMM_XCD: 0 blockIdx, 1 a tile's splits on one XCD, 2 a split's row tiles): same-bits test,
# step times, and FETCH_SIZE per launch under each order.
RC=tools/rgemm_check.py
V="x0=GQ_RGEMM_XCD:0+GQ_SGEMM_XCD:0,x1=GQ_RGEMM_XCD:1+GQ_SGEMM_XCD:1,x2=GQ_RGEMM_XCD:2+GQ_SGEMM_XCD:2"
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_rgemm.py -q -k xcd --timeout 120 --timeout-method thread' \
steps 400 "python -u $RC --steps-only --rounds 3 --variants $V --configs q4_k_11008x4096_m16,q4_k_4096x4096_m16,q4_k_22016x4096_m16,q4_k_4096x11008_m16,q8_0_11008x4096_m16,q6_k_11008x4096_m16,q4_k_11008x4096_m64,q8_0_4096x4096_m128,q4_k_4096x4096_m128,q4_k_11008x4096_m128,q4_k_4096x11008_m128,q6_k_28672x8192_m128,q6_k_8192x28672_m128" \
traffic 400 "GQ_RGEMM_XCD=1 GQ_SGEMM_XCD=1 python3 tools/pmc_traffic.py q4_k_11008x4096_m16 q8_0_4096x4096_m128 q4_k_4096x11008_m128 && GQ_RGEMM_XCD=2 GQ_SGEMM_XCD=2 python3 tools/pmc_traffic.py q4_k_11008x4096_m16 q8_0_4096x4096_m128 q4_k_4096x11008_m128"
