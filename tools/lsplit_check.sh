#!/bin/bash
# split loaders: parity under GQ_GEMM_LSPLIT=1 and 2, then interleaved A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 1 2; do
  GQ_GEMM_LSPLIT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_paths.py > gpurun_out/lsplit_tests_$v.log 2>&1 || { tail -30 gpurun_out/lsplit_tests_$v.log; exit 1; }
  tail -1 gpurun_out/lsplit_tests_$v.log
done
S=""
for c in q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64 q6_k_8192x28672_m128; do
  S="$S $c $c:GQ_GEMM_LSPLIT=1 $c:GQ_GEMM_LSPLIT=2"
done
AB_R=3 bash tools/ab.sh $S > gpurun_out/lsplit_ab.txt 2>&1; cat gpurun_out/lsplit_ab.txt
