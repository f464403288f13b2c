#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 300 --timeout-method thread -k "huge" > gpurun_out/pf16b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pf16b_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/pf16b_pytest.log | head -20; exit $rc; }
GQ_GEMM_PARTIAL=f16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_fp8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pf16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pf16_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/pf16_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/gemm_tune.py --step q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f32 q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f16 q4_k_4096x4096_m128:GQ_GEMM_PARTIAL=f32 q4_k_4096x4096_m128:GQ_GEMM_PARTIAL=f16 && python tools/gemm_tune.py q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f32 q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f16 q4_k_11008x4096_m128:GQ_GEMM_PARTIAL=f32 q4_k_11008x4096_m128:GQ_GEMM_PARTIAL=f16 > gpurun_out/pf16_step.txt 2>&1
rc=$?; cat gpurun_out/pf16_step.txt; exit $rc
