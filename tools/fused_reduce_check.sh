#!/bin/bash
# fused split-K reduce: parity test, step A/B against the separate reduce launch, GPU suite
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread \
  -k fused_split_k > gpurun_out/fused_test.log 2>&1 || { tail -30 gpurun_out/fused_test.log; exit 1; }
tail -2 gpurun_out/fused_test.log
CFGS="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64"
for env in GQ_GEMM_FUSED_REDUCE=0 GQ_GEMM_FUSED_REDUCE=1 GQ_GEMM_FUSED_REDUCE=0 GQ_GEMM_FUSED_REDUCE=1; do
  args=""; for c in $CFGS; do args="$args $c:$env"; done
  timeout -k 10 120 python -u tools/gemm_tune.py --step $args 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/fused_ab.txt || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
