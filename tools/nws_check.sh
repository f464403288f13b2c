#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CF="q4_k_4096x4096_m16 q4_k_4096x4096_m8 q4_k_4096x4096_m32 q8_0_4096x4096_m16 q4_k_11008x4096_m16 q6_k_28672x8192_m16 q6_k_28672x8192_m32"
for lib in gguf-triton-kernel_amd/lib/libgguf_mmq.so gguf-triton-kernel_amd/lib/libgguf_mmq_nws3.so gguf-triton-kernel_amd/lib/libgguf_mmq_nws4.so; do
  echo "== $lib"
  timeout -k 10 200 python tools/gemm_tune.py --lib=$lib $CF 2>&1 | grep kernel_us || exit 1
done
