#!/bin/bash
# Q8_0 one-sub-stage weight stages (GQ_GEMM_Q8_FINE=1) with 7 / 9 weight slots (6 / 8 sub-stages of weights in flight) vs the shipping super-block stages
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for n in 7 9; do
  L=gguf-triton-kernel_amd/lib/libgguf_mmq_fine$n.so
  timeout -k 10 300 python -u tools/lib_parity.py $L tests/test_gpu_paths.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -m gpu -k "q8_0 and (gemm or golden or fused_split_k)" > gpurun_out/fine${n}_test.log 2>&1 || { tail -30 gpurun_out/fine${n}_test.log; exit 1; }
  tail -1 gpurun_out/fine${n}_test.log
done
CFGS="q8_0_4096x4096_m128 q8_0_4096x4096_m64 q8_0_11008x4096_m128 q8_0_4096x4096_m256 q8_0_14336x4096_m128"
for i in 1 2; do
  timeout -k 10 150 python -u tools/gemm_tune.py --step $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/base  /' | tee -a gpurun_out/fine_nws_ab.txt || exit 1
  for n in 7 9; do
    timeout -k 10 150 python -u tools/gemm_tune.py --step --lib=gguf-triton-kernel_amd/lib/libgguf_mmq_fine$n.so $CFGS 2>&1 | grep -v amdgpu.ids | sed "s/^/fine$n /" | tee -a gpurun_out/fine_nws_ab.txt || exit 1
  done
done
