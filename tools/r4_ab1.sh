#!/bin/bash
# Round-4 A/B batch 1: rgemm v2 / sgemm / grouped GEMM tests, spol variants, small-N routes,
# decode prologue refill, layer sweep (outputs: gpurun_out/<step>.txt).
RC=tools/rgemm_check.py
exec_steps() { bash tools/gpu_steps.sh "$@"; }
exec_steps \
t_rg 500 'python -u -m pytest tests/test_gpu_rgemm.py tests/test_gpu_gemm_grouped.py tests/test_gpu_cus.py -x -q --timeout 120 --timeout-method thread' \
rg_v2 200 "python -u $RC --configs q8_0_4096x4096_m128,q4_k_4096x4096_m128,q6_k_4096x4096_m128 --rounds 2 --variants p0=GQ_RGEMM:1+GQ_RGEMM_SPOL:0,nt=GQ_RGEMM:1+GQ_RGEMM_SPOL:2,sc1=GQ_RGEMM:1+GQ_RGEMM_SPOL:16,old=GQ_RGEMM:0" \
rg_small 150 "python -u $RC --steps-only --configs q4_k_4096x4096_m16,q8_0_4096x4096_m16,q6_k_4096x4096_m16,q4_k_4096x4096_m8,q6_k_4096x4096_m8 --rounds 2 --variants rg=GQ_RGEMM:1+GQ_SKINNY:0,old=GQ_RGEMM:0" \
sg_small 150 "python -u $RC --configs q4_k_11008x4096_m16,q4_k_4096x11008_m16,q8_0_11008x4096_m16,q6_k_11008x4096_m16,q6_k_4096x11008_m16 --rounds 2 --variants old=GQ_RGEMM:0,sg=GQ_RGEMM:0+GQ_SGEMM:1+GQ_SKINNY:0" \
sg_v1 200 "python -u $RC --configs q6_k_28672x8192_m128,q6_k_8192x28672_m128,q4_k_11008x4096_m128,q4_k_4096x11008_m128,q8_0_11008x4096_m128 --rounds 1 --variants old=GQ_RGEMM:0,sg=GQ_RGEMM:0+GQ_SGEMM:1" \
dec_early 150 "python -u $RC --steps-only --configs q6_k_28672x8192_m1,q6_k_8192x28672_m1,q8_0_4096x4096_m1,q4_k_4096x11008_m1,q6_k_28672x8192_m2 --rounds 2 --variants e0=GQ_DECODE_EARLY:0,e1=GQ_DECODE_EARLY:1,e2=GQ_DECODE_EARLY:2" \
layer 300 'python -u bench.py --layer-only --steps 80'
