#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_tune.py --abl ${SPECS:-q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q4_k_11008x4096_m16 q6_k_28672x8192_m128:GQ_ABLATE=6 q6_k_28672x8192_m128:GQ_ABLATE=1 q8_0_4096x4096_m128:GQ_ABLATE=15} 2>&1 | grep -v amdgpu
