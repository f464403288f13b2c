#!/bin/bash
# Round-4 A/B batch 2: the GPU suite, the sgemm ring depth (NS 6 vs 4 build), sgemm vs the other
# GEMM routes across token counts, the layer sweep (outputs: gpurun_out/<step>.txt).
RC=tools/rgemm_check.py
L=gguf-triton-kernel_amd/lib
bash tools/gpu_steps.sh \
tests 700 'python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
ns 200 "python -u $RC --configs q4_k_11008x4096_m16,q6_k_11008x4096_m16,q4_k_11008x4096_m32,q6_k_28672x8192_m128,q4_k_11008x4096_m128 --rounds 2 --variants sg=GQ_RGEMM:0+GQ_SGEMM:1+GQ_SKINNY:0 --libs ns6=$L/libgguf_mmq.so,ns4=$L/libgguf_mmq_ns4.so" \
sg_n 300 "python -u $RC --configs q6_k_28672x8192_m32,q6_k_28672x8192_m64,q6_k_28672x8192_m256,q6_k_28672x8192_m512,q4_k_11008x4096_m32,q4_k_11008x4096_m64,q4_k_11008x4096_m256,q8_0_11008x4096_m64,q8_0_11008x4096_m256,q6_k_8192x28672_m64 --rounds 1 --variants old=GQ_RGEMM:0,sg=GQ_RGEMM:0+GQ_SGEMM:1" \
layer 300 'python -u bench.py --layer-only --steps 80' \
stamps 120 'python -u tools/decode_stamps.py q6_k_28672x8192_m1 q6_k_8192x28672_m1 q4_k_4096x11008_m1' \
f8 200 'python -u tools/layer_time.py 1,2 --grouped-only --act fp8 --tune GQ_DECODE_F8_ITC=1 && python -u tools/layer_time.py 1,2 --grouped-only --act fp8 --tune GQ_DECODE_F8_ITC=0'
