#!/bin/bash
# Round-4 batch 6: the resident GEMM past one round of the chip at 8-32 tokens (forced) vs the
# default routes; the eager host cost.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
rg2 300 "python -u $RC --steps-only --configs q4_k_22016x4096_m16,q4_k_14336x4096_m16,q4_k_11008x4096_m32,q4_k_22016x4096_m8,q6_k_4096x11008_m16,q6_k_11008x4096_m16,q8_0_11008x4096_m16,q4_k_4096x14336_m16,q6_k_4096x4096_m4,q4_k_4096x4096_m4 --rounds 2 --variants rg=GQ_RGEMM:1+GQ_SKINNY:0,def=GQ_RGEMM:-1" \
eager 120 'python -u tools/eager_probe.py'
