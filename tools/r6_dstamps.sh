#!/bin/bash
# Round 6: per-wave phase stamps of the decode kernel (diagnostic build lib/libgguf_mmq_stamps.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/decode_stamps.py q6_k_8192x28672_m1 q6_k_28672x8192_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1 > gpurun_out/r6_dstamps.txt 2>&1
rc=$?; cat gpurun_out/r6_dstamps.txt; exit $rc
