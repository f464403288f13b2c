#!/usr/bin/env bash
# GEMM variant check: parity of the ragged/golden GEMM tests under GQ_GEMM_LOADERS=${L:-4},
# then kernel times with and without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GQ_GEMM_LOADERS=${L:-4} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "golden or ragged or long_rows or baseline or 256_row" > gpurun_out/loader_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/loader_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/loader_pytest.log | head -20; exit $rc; }
A=""
for cfg in q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64; do
  for l in 0 4; do A="$A $cfg:GQ_GEMM_LOADERS=$l"; done
done
for s in 1 2 4; do for l in 0 4; do A="$A q8_0_4096x4096_m128:GQ_GEMM_LOADERS=$l,GQ_GEMM_SPLITS=$s"; done; done
timeout -k 10 300 python tools/gemm_tune.py $A > gpurun_out/loader_tune.txt 2>&1
rc=$?; cat gpurun_out/loader_tune.txt; exit $rc
