#!/bin/bash
# cold (weights rotated over 1 GiB, as bench.py) vs warm (2 copies: MALL-resident) weights
set -o pipefail
mkdir -p gpurun_out
CFGS="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_4096x4096_m16 q4_k_4096x4096_m1 q8_0_4096x4096_m1 q6_k_28672x8192_m1 q6_k_28672x8192_m128"
for i in 1 2; do
  timeout -k 10 150 python -u tools/gemm_tune.py --step $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/cold /' | tee -a gpurun_out/rotate_ab.txt || exit 1
  GQ_TUNE_ROTATE=1 timeout -k 10 150 python -u tools/gemm_tune.py --step $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/warm /' | tee -a gpurun_out/rotate_ab.txt || exit 1
done
