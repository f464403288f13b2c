#!/bin/bash
# Round-4 batch 14: a super-block's two half stages issued together (GQ_SGEMM_PAIR 1: rings of
# 4+ slots, 2: 3+) in the streaming GEMMs: same-bits tests, the layer, the DMA-only ablation, and
# single streaming-GEMM steps.
L=gguf-triton-kernel_amd/lib
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_gemm_grouped.py -q --timeout 120 --timeout-method thread' \
layer 500 "python -u tools/layer_time.py 8,16,32,64,128 --grouped-only && python -u tools/layer_time.py 8,16,32,64,128 --grouped-only --tune GQ_SGEMM_PAIR=1 && python -u tools/layer_time.py 8,16,32,64,128 --grouped-only --tune GQ_SGEMM_PAIR=2 && python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl4.so && python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl4.so --tune GQ_SGEMM_PAIR=2" \
steps 300 "python -u $RC --steps-only --rounds 3 --variants p0=GQ_SGEMM_PAIR:0,p1=GQ_SGEMM_PAIR:1,p2=GQ_SGEMM_PAIR:2 --configs q4_k_4096x11008_m128,q4_k_11008x4096_m128,q6_k_28672x8192_m128,q4_k_11008x4096_m32"
