#!/bin/bash
# Round 5: K-chunked stream A/B against a diagnostic build (LIB=gguf-triton-kernel_amd/lib/libgguf_mmq_<name>.so):
# tests of the stream, prepared-call kernel time (graph-timed), the grouped 7B layer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=gguf-triton-kernel_amd/lib/libgguf_mmq_${KLIB:?name of the diagnostic build}.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kstream.py tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
C=${KCFGS:-"q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_22016x4096_m16 q6_k_4096x4096_m16 q8_0_11008x4096_m16 q4_k_22016x4096_m32 q6_k_4096x11008_m16"}
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/gemm_tune.py $C || exit $?
  timeout -k 10 200 python3 tools/gemm_tune.py --lib=$L $C | sed "s/^/alt:/" || exit $?
done 2>&1 | grep kernel_us | awk '{print $1, $3}' | sort | awk '{k=$1; v[k]=v[k]" "$2} END {for (k in v) print k, v[k]}' | sort
timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only || exit $?
timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only --lib $L || exit $?
