#!/bin/bash
# Round-4 batch 17: the streaming GEMM's weight DMAs non-temporal (GQ_SGEMM_NT, as the decode
# kernel's): the layer and single streaming steps.
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
layer 400 "python -u tools/layer_time.py 8,16,32,128 --grouped-only && python -u tools/layer_time.py 8,16,32,128 --grouped-only --tune GQ_SGEMM_NT=1" \
steps 300 "python -u $RC --steps-only --rounds 3 --variants def=GQ_SGEMM_NT:0,nt=GQ_SGEMM_NT:1 --configs q4_k_11008x4096_m128,q4_k_4096x11008_m128,q6_k_28672x8192_m128,q6_k_8192x28672_m128"
