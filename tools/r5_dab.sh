#!/bin/bash
# Round 5: decode A/B against a diagnostic build (LIBS: names of gguf-triton-kernel_amd/lib/libgguf_mmq_<name>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grouped.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
C=${DCFGS:-"q6_k_8192x28672_m1 q6_k_28672x8192_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1 q4_k_4096x11008_m1 q8_0_4096x4096_m1 q6_k_28672x8192_m2"}
CFGS="$C" R=3 bash tools/r5_libab.sh || exit $?
timeout -k 10 300 python3 tools/layer_time.py 1,2 --grouped-only || exit $?
for l in $LIBS; do timeout -k 10 300 python3 tools/layer_time.py 1,2 --grouped-only --lib gguf-triton-kernel_amd/lib/libgguf_mmq_$l.so || exit $?; done
