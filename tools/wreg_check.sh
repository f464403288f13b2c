#!/bin/bash
# GEMM weight-path variants: register weights (GQ_GEMM_WREG=1) and split loaders with a 3-stage
# weight ring (GQ_GEMM_LSPLIT=2): parity of each, then interleaved A/B against the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in GQ_GEMM_WREG=1 GQ_GEMM_LSPLIT=2; do
  env $v timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_paths.py -k "not full_size" > gpurun_out/wreg_tests.log 2>&1 || { echo $v; tail -30 gpurun_out/wreg_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/wreg_tests.log)"
done
S=""
for c in ${CFGS:-q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64 q6_k_8192x28672_m128 q4_k_4096x11008_m128}; do
  S="$S $c $c:GQ_GEMM_WREG=1 $c:GQ_GEMM_LSPLIT=2"
done
AB_R=3 bash tools/ab.sh $S > gpurun_out/wreg_ab.txt 2>&1; cat gpurun_out/wreg_ab.txt
