#!/bin/bash
# Round-4 batch 15: Q4_K whole-super-block stages in the streaming GEMM (GQ_SGEMM_FULL, 16/32-token
# tiles): same-bits tests, the layer, the DMA-only ablation, single-matrix steps.
L=gguf-triton-kernel_amd/lib
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
t 300 'python -u -m pytest tests/test_gpu_gemm_grouped.py -q -k "schedule or bit_identical or parity" --timeout 120 --timeout-method thread' \
layer 500 "python -u tools/layer_time.py 8,16,24,32 --grouped-only && python -u tools/layer_time.py 8,16,24,32 --grouped-only --tune GQ_SGEMM_FULL=1 && python -u tools/layer_time.py 16 --grouped-only --lib $L/libgguf_mmq_rabl4.so && python -u tools/layer_time.py 16 --grouped-only --lib $L/libgguf_mmq_rabl4.so --tune GQ_SGEMM_FULL=1" \
steps 300 "python -u $RC --steps-only --rounds 3 --variants half=GQ_RGEMM:0+GQ_SKINNY:0+GQ_SGEMM:1,full=GQ_RGEMM:0+GQ_SKINNY:0+GQ_SGEMM:1+GQ_SGEMM_FULL:1,def=GQ_SGEMM:-1 --configs q4_k_11008x4096_m16,q4_k_4096x11008_m16,q4_k_11008x4096_m32,q4_k_4096x4096_m16"
