#!/usr/bin/env bash
# int8-MFMA Q8_0 GEMM: parity tests, then kernel time vs the fp16 form (tools/gemm_tune.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 120 --timeout-method thread -k "int8 or prepared" > gpurun_out/i8_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/i8_pytest.log; [ $rc -eq 0 ] || exit $rc
A=""
for cfg in q8_0_4096x4096_m128 q8_0_4096x4096_m16 q8_0_4096x4096_m64 q8_0_11008x4096_m128 q8_0_4096x4096_m256; do
  for i8 in 0 1; do A="$A $cfg:GQ_GEMM_I8=$i8"; done
done
for s in 2 4 8 16; do A="$A q8_0_4096x4096_m128:GQ_GEMM_I8=1,GQ_GEMM_SPLITS=$s"; done
timeout -k 10 300 python tools/gemm_tune.py $A > gpurun_out/i8_tune.txt 2>&1
rc=$?; cat gpurun_out/i8_tune.txt; exit $rc
