#!/usr/bin/env bash
# fp16 split-K partials: parity of the GEMM tests under GQ_GEMM_PARTIAL=f16, then times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GQ_GEMM_PARTIAL=f16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -x -q --timeout 300 --timeout-method thread -k "golden or ragged or long_rows or baseline or 256_row or prepared or chunked" > gpurun_out/pf16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pf16_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/pf16_pytest.log | head -20; exit $rc; }
A=""
for cfg in q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64 q4_k_4096x11008_m128; do
  for p in f32 f16; do A="$A $cfg:GQ_GEMM_PARTIAL=$p"; done
done
for nb in 4 8; do for s in 4 8 16; do A="$A q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f16,GQ_GEMM_SPLITS=$s,GQ_GEMM_NB=$nb"; done; done
timeout -k 10 300 python tools/gemm_tune.py $A > gpurun_out/pf16_tune.txt 2>&1
rc=$?; cat gpurun_out/pf16_tune.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gemm_tune.py --step q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f32 q8_0_4096x4096_m128:GQ_GEMM_PARTIAL=f16 > gpurun_out/pf16_step.txt 2>&1
rc=$?; cat gpurun_out/pf16_step.txt; exit $rc
