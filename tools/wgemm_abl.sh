#!/bin/bash
# Ablation timings of the weight-register GEMM (diagnostic builds: make -C gguf-triton-kernel_amd wabl WABL=n)
# Run on the GPU box: bash tools/wgemm_abl.sh [abl numbers...] > gpurun_out/wabl.log
set -e
C=${CONFIGS:-q8_0_4096x4096_m128,q4_k_11008x4096_m128,q6_k_28672x8192_m128}
L=gguf-triton-kernel_amd/lib
timeout -k 10 240 python -u tools/wgemm_check.py --only-time --configs $C --variants ${VARIANTS:-old,w_rg2_nb8}
for a in "$@"; do
  timeout -k 10 120 python -u tools/wgemm_check.py --only-time --configs $C --variants w_rg2_nb8 --lib $L/libgguf_mmq_wabl$a.so
done
