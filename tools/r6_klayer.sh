#!/bin/bash
# Round 6: balance of the grouped K-chunked stream on the 7B layer (kstamps build) at 16 / 24 / 32
# tokens, and the single-matrix per-format cost at 16 / 32 tokens (prepared, product build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/kstream_layer_stamps.py 16 24 32 > gpurun_out/r6_klayer.txt 2>&1
rc=$?; cat gpurun_out/r6_klayer.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/gemm_tune.py q4_k_4096x4096_m16 q6_k_4096x4096_m16 q8_0_4096x4096_m16 \
  q4_k_4096x4096_m32 q6_k_4096x4096_m32 q8_0_4096x4096_m32 q6_k_4096x11008_m32:GQ_KSTREAM=1 \
  q4_k_4096x11008_m32:GQ_KSTREAM=1 2>&1 | grep kernel_us | tee gpurun_out/r6_kfmt.txt
