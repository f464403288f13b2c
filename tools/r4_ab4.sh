#!/bin/bash
# Round-4 batch 4: stream-K sgemm / grouped GEMM -- GPU tests of the GEMM paths, timings vs the
# whole-tile split plan (GQ_SGEMM_SPLITS pinned to what it would choose is not expressible, so
# the A/B is stream-K (auto) vs the previous measurements), the layer sweep; decode x-first at
# 2/4 tokens.
L=gguf-triton-kernel_amd/lib
RC=tools/rgemm_check.py
bash tools/gpu_steps.sh \
tests 600 'python -u -m pytest tests/test_gpu_gemm_grouped.py tests/test_gpu_rgemm.py tests/test_gpu_paths.py tests/test_gpu_skinny.py -q --maxfail=10 --timeout 120 --timeout-method thread' \
sk 200 "python -u $RC --configs q6_k_28672x8192_m128,q6_k_8192x28672_m128,q4_k_11008x4096_m128,q8_0_11008x4096_m128,q6_k_28672x8192_m32,q6_k_11008x4096_m16 --rounds 2 --variants sk=GQ_RGEMM:0,sp2=GQ_RGEMM:0+GQ_SGEMM:1+GQ_SGEMM_SPLITS:2" \
layer 200 'python -u tools/layer_time.py 16,32,64,128,192 --grouped-only' \
xf2 200 "python -u $RC --steps-only --configs q4_k_4096x4096_m2,q4_k_4096x4096_m4,q4_k_11008x4096_m2,q4_k_11008x4096_m4,q6_k_4096x11008_m2,q6_k_8192x28672_m2,q8_0_4096x4096_m3 --rounds 2 --variants d=GQ_DECODE_EARLY:0 --libs main=$L/libgguf_mmq.so,xfirst=$L/libgguf_mmq_xfirst.so" \
xfl 200 "python -u tools/layer_time.py 1,2,3,4 --grouped-only && python -u tools/layer_time.py 1,2,3,4 --grouped-only --lib $L/libgguf_mmq_xfirst.so"
