#!/bin/bash
# Round 5: the K-chunked streaming MMQ (GQ_KSTREAM=1) against the default routes, step us
# (gq_mmq incl. the in-kernel quantization) and MMQ us (prepared x~), 5..32 tokens.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=${CFGS:-"q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_22016x4096_m16 q4_k_12288x4096_m16 q6_k_4096x4096_m16 q8_0_11008x4096_m16 q4_k_22016x4096_m32 q4_k_22016x4096_m8"}
A=""
for c in $CFGS; do A="$A $c $c:GQ_KSTREAM=1"; done
echo "== step"
timeout -k 10 300 python3 tools/gemm_tune.py --step $A || exit $?
echo "== MMQ (prepared)"
timeout -k 10 300 python3 tools/gemm_tune.py $A || exit $?
