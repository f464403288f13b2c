#!/bin/bash
# GEMM first-sub-stage wait by DMA stream (stamps + ablation build): full, no activation DMA, no weight DMA
set -o pipefail
mkdir -p gpurun_out
CFGS="q8_0_4096x4096_m128 q4_k_4096x4096_m16"
for a in 0 4 2 6; do
  echo "== GQ_ABLATE=$a" | tee -a gpurun_out/first_wait.txt
  GQ_ABLATE=$a timeout -k 10 120 python -u tools/gemm_stamps.py $CFGS 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/first_wait.txt || exit 1
done
