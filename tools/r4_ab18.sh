#!/bin/bash
# Round-4 batch 18: is the grouped GEMM's weight stream bound by its access pattern?  Ablation
# builds (never the product): 4 = no multiply; 20 = no multiply, each weight stage read as one
# contiguous run of the tile's rows (same bytes, wrong values); 5 = neither weights nor multiply.
L=gguf-triton-kernel_amd/lib
bash tools/gpu_steps.sh \
layer 500 "python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl4.so && python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl20.so && python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl5.so && python -u tools/layer_time.py 16,128 --grouped-only"
