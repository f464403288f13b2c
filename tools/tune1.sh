#!/usr/bin/env bash
# GPU session: parity tests (stop on failure), then the GEMM tuning / ablation sweep.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -3
T="timeout -k 10 400 python tools/gemm_tune.py --abl"
$T ${TUNE_SPECS:-q6_k_28672x8192_m128 q6_k_28672x8192_m128:GQ_GEMM_SPLITS=1 q6_k_28672x8192_m128:GQ_GEMM_RG=1 \
   q6_k_28672x8192_m128:GQ_ABLATE=1 q6_k_28672x8192_m128:GQ_ABLATE=2 q6_k_28672x8192_m128:GQ_ABLATE=4 \
   q6_k_28672x8192_m128:GQ_ABLATE=6 q6_k_28672x8192_m128:GQ_ABLATE=14 \
   q4_k_11008x4096_m128 q4_k_11008x4096_m128:GQ_GEMM_RG=1 q4_k_11008x4096_m128:GQ_ABLATE=1 q4_k_11008x4096_m128:GQ_ABLATE=6 \
   q4_k_4096x4096_m128 q4_k_4096x4096_m128:GQ_GEMM_RG=1 \
   q8_0_4096x4096_m128 q8_0_4096x4096_m128:GQ_GEMM_RG=1 q8_0_4096x4096_m128:GQ_GEMM_RG=2 q8_0_4096x4096_m128:GQ_ABLATE=1 q8_0_4096x4096_m128:GQ_ABLATE=6 \
   q4_k_4096x4096_m16 q4_k_11008x4096_m16} 2>&1 | grep -v amdgpu.ids
