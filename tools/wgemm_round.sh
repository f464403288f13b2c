#!/bin/bash
# One GPU round for the weight-register GEMM: quick parity, then timings of variants
# (VARIANTS / CONFIGS: names in tools/wgemm_check.py; ABLS: diagnostic builds, make wabl WABL=n)
set -e
timeout -k 10 200 python -u tools/wgemm_check.py --quick --no-time
V=${VARIANTS:-old,w_rg2_nb8,w_rg2_nb4,w_rg1_nb8,w_rg2_nb8_s1}
timeout -k 10 400 python -u tools/wgemm_check.py --only-time --variants $V --configs ${CONFIGS:-q8_0_4096x4096_m128,q4_k_4096x4096_m128,q4_k_11008x4096_m128,q4_k_4096x11008_m128,q6_k_28672x8192_m128,q6_k_8192x28672_m128}
for a in ${ABLS:-}; do
  timeout -k 10 120 python -u tools/wgemm_check.py --only-time --configs q8_0_4096x4096_m128,q6_k_28672x8192_m128 --variants w_rg2_nb8,w_rg1_nb8 --lib gguf-triton-kernel_amd/lib/libgguf_mmq_wabl$a.so
done
