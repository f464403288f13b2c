#!/bin/bash
# Round 5: where the K-chunked streaming MMQ's time goes (ablation builds, make kabl KABL=n;
# never the product): 1 no multiply, 2 no reduce, 4 no weight DMA; MMQ us (prepared x~).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CFGS=${CFGS:-"q4_k_22016x4096_m16:GQ_KSTREAM=1 q4_k_4096x4096_m16:GQ_KSTREAM=1 q6_k_12288x4096_m16:GQ_KSTREAM=1 q8_0_11008x4096_m16:GQ_KSTREAM=1"}
L=gguf-triton-kernel_amd/lib
for lib in libgguf_mmq ${KABLS:-libgguf_mmq_kabl2 libgguf_mmq_kabl4 libgguf_mmq_kabl6}; do
  echo "== $lib"
  timeout -k 10 120 python3 tools/gemm_tune.py --lib=$L/$lib.so $CFGS || exit $?
done
