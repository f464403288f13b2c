#!/bin/bash
# Round 5: the review's "done when" figures in one call -- graph-timed single calls (step = gq_mmq
# with in-kernel quantization) and the 7B Q4_K_M layer (q8_1 and fp8) at the named token counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "== step"
timeout -k 10 300 python3 tools/gemm_tune.py --step q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 \
  q6_k_28672x8192_m128 q4_k_11008x4096_m16 q6_k_8192x28672_m1 q6_k_28672x8192_m1 || exit $?
echo "== layer q8_1"
timeout -k 10 300 python3 tools/layer_time.py 1,2,8,16,64 --grouped-only || exit $?
echo "== layer fp8"
timeout -k 10 300 python3 tools/layer_time.py 1,2 --grouped-only --act fp8 || exit $?
