#!/bin/bash
# Round 5: diagnostic-library A/B (graph-timed gq_mmq steps): the product library against the
# builds named in LIBS (gguf-triton-kernel_amd/lib/libgguf_mmq_<name>.so), R interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C=${CFGS:-"q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q4_k_11008x4096_m16"}
for r in $(seq ${R:-3}); do
  timeout -k 10 200 python3 tools/gemm_tune.py --step $C || exit $?
  for l in $LIBS; do
    timeout -k 10 200 python3 tools/gemm_tune.py --step --lib=gguf-triton-kernel_amd/lib/libgguf_mmq_$l.so $C | sed "s/^/$l:/" || exit $?
  done
done 2>&1 | grep kernel_us | awk '{print $1, $3}' | sort | awk '{k=$1; v[k]=v[k]" "$2} END {for (k in v) print k, v[k]}' | sort
