#!/bin/bash
# Round 5: resident GEMM with per-wave weight images (no weight barriers) vs the previous build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=${CFGS:-"q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q8_0_4096x4096_m16 q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_4096x4096_m64 q8_0_11008x4096_m16"}
for r in 1 2; do
  for lib in gguf-triton-kernel_amd/lib/ab/libgguf_mmq_old.so gguf-triton-kernel_amd/lib/libgguf_mmq.so; do
    echo "== round $r $lib"
    timeout -k 10 300 python3 tools/gemm_tune.py --step --lib=$lib $CFGS || exit $?
  done
done
