#!/bin/bash
# Round-4 batch 19: how long must the weight runs be?  No-multiply ablations of the grouped
# GEMM (never the product): 4 = the product's pattern (one super-block per row per stage), 20 = one
# contiguous run per stage, 20rL = runs of L bytes from consecutive rows (L = 288, 1152, 2304).
L=gguf-triton-kernel_amd/lib
bash tools/gpu_steps.sh \
layer 600 "for v in 4 20r288 20r1152 20r2304 20; do python -u tools/layer_time.py 16,128 --grouped-only --lib $L/libgguf_mmq_rabl\$v.so || exit \$?; done"
