#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CF="q4_k_4096x4096_m1 q8_0_4096x4096_m1 q4_k_11008x4096_m1 q4_k_4096x4096_m2 q4_k_4096x4096_m4 q6_k_28672x8192_m1"
for lib in libgguf_mmq.so libgguf_mmq_ni3.so libgguf_mmq_ni4.so; do
  echo "== $lib"; AB_R=3 AB_LIB=gguf-triton-kernel_amd/lib/$lib bash tools/ab.sh --step $CF || exit 1
done
