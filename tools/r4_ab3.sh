#!/bin/bash
# Round-4 batch 3: the GPU suite (up to 10 failures listed), decode stamps (default and x-first
# prologue builds), decode x-first A/B, the default bench line.
L=gguf-triton-kernel_amd/lib
bash tools/gpu_steps.sh \
tests 800 'python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread' \
stamps 120 'python -u tools/decode_stamps.py q6_k_28672x8192_m1 q6_k_8192x28672_m1 q4_k_4096x11008_m1 && GQ_STAMPS_SO=xfirst_stamps python -u tools/decode_stamps.py q6_k_28672x8192_m1 q6_k_8192x28672_m1 q4_k_4096x11008_m1' \
xfirst 150 "python -u tools/rgemm_check.py --steps-only --configs q6_k_28672x8192_m1,q6_k_8192x28672_m1,q8_0_4096x4096_m1,q4_k_4096x11008_m1,q4_k_4096x4096_m1,q6_k_28672x8192_m2 --rounds 2 --variants d=GQ_DECODE_EARLY:0 --libs main=$L/libgguf_mmq.so,xfirst=$L/libgguf_mmq_xfirst.so,scalarq=$L/libgguf_mmq_scalarq.so" \
rg_q4 150 "python -u tools/rgemm_check.py --steps-only --configs q4_k_11008x4096_m16,q4_k_4096x11008_m16,q4_k_11008x4096_m8,q4_k_14336x4096_m16 --rounds 2 --variants rg=GQ_RGEMM:1+GQ_SKINNY:0,sk=GQ_RGEMM:0" \
layer 200 'python -u tools/layer_time.py 16,128,256,512 --grouped-only && python -u tools/layer_time.py 256,512 --grouped-only --tune GQ_BLAS_MIN_TOKENS=256' \
bench 300 'python -u bench.py --steps 20 --warmup 5'
