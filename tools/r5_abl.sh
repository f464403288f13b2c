#!/bin/bash
# Round 5: where the resident GEMM's time goes on the M=128 shapes (ablation builds, make rabl),
# the streaming form at several split counts, and the vendor library's fp16 GEMM for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=${CFGS:-"q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q4_k_11008x4096_m16"}
L=gguf-triton-kernel_amd/lib
for lib in libgguf_mmq libgguf_mmq_rabl1 libgguf_mmq_rabl2 libgguf_mmq_rabl4 libgguf_mmq_rabl8 libgguf_mmq_rabl12 libgguf_mmq_rabl3 libgguf_mmq_rabl15; do
  args=""
  for c in $CFGS; do args="$args $c"; done
  echo "== $lib (MMQ, prepared)"
  timeout -k 10 120 python3 tools/gemm_tune.py --lib=$L/$lib.so $args || exit $?
  echo "== $lib (step)"
  timeout -k 10 120 python3 tools/gemm_tune.py --step --lib=$L/$lib.so $args || exit $?
done
echo "== streaming GEMM on the headline"
timeout -k 10 200 python3 tools/gemm_tune.py --step q8_0_4096x4096_m128 q8_0_4096x4096_m128:GQ_RGEMM=0,GQ_SGEMM=1,GQ_SGEMM_SPLITS=16 \
  q8_0_4096x4096_m128:GQ_RGEMM=0,GQ_SGEMM=1,GQ_SGEMM_SPLITS=8 q8_0_4096x4096_m128:GQ_RGEMM=0,GQ_SGEMM=1,GQ_SGEMM_SPLITS=4 \
  q8_0_4096x4096_m128:GQ_RGEMM=0,GQ_SGEMM=1,GQ_SGEMM_SPLITS=2 || exit $?
echo "== vendor fp16 GEMM"
timeout -k 10 200 python3 tools/ref_gemm.py
