#!/bin/bash
# Round-4 batch 13: the 7B layer at 16 / 32 / 128 tokens with ablation builds of mmq_rgemm.hip
# (never the product): 4 = no multiply, 1 = no weight DMA, 5 = neither (x~ stages, barriers,
# epilogue only) -- which part of the grouped streaming GEMM sets its time.
L=gguf-triton-kernel_amd/lib
bash tools/gpu_steps.sh \
layer 500 "python -u tools/layer_time.py 16,32,128 --grouped-only && python -u tools/layer_time.py 16,32,128 --grouped-only --lib $L/libgguf_mmq_rabl4.so && python -u tools/layer_time.py 16,32,128 --grouped-only --lib $L/libgguf_mmq_rabl1.so && python -u tools/layer_time.py 16,32,128 --grouped-only --lib $L/libgguf_mmq_rabl5.so"
