#!/usr/bin/env bash
# GPU session: parity tests (stop on failure), then decode-step timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gemm_tune.py --step ${SPECS:-q6_k_28672x8192_m1 q4_k_11008x4096_m1 q8_0_4096x4096_m1 q4_k_4096x4096_m1 q6_k_8192x28672_m1 q4_k_4096x11008_m1 q4_k_4096x4096_m4 q6_k_28672x8192_m8} > gpurun_out/tune.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/tune.log; exit $rc
