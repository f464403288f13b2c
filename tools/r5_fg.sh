#!/bin/bash
# Round 5: the full-K tile GEMM (GQ_FGEMM=1) against the default routes, per tile shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=${CFGS:-"q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128 q8_0_11008x4096_m128 q4_k_4096x4096_m64 q4_k_4096x4096_m32 q8_0_4096x4096_m32"}
for mode in "" "--step"; do
  A=""
  for c in $CFGS; do
    A="$A $c $c:GQ_FGEMM=1 $c:GQ_FGEMM=1,GQ_FGEMM_RW=2,GQ_FGEMM_NB=2 $c:GQ_FGEMM=1,GQ_FGEMM_RW=4,GQ_FGEMM_NB=2 $c:GQ_FGEMM=1,GQ_FGEMM_RW=4,GQ_FGEMM_NB=4 $c:GQ_FGEMM=1,GQ_FGEMM_RW=8,GQ_FGEMM_NB=4"
  done
  echo "== mode ${mode:-mmq}"
  timeout -k 10 400 python3 tools/gemm_tune.py $mode $A || exit $?
done
