#!/bin/bash
# serialized GEMM prologue (GQ_GEMM_PSER=1: W(0) lands before the activation DMAs issue) vs both together
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=gguf-triton-kernel_amd/lib/libgguf_mmq_pser.so
timeout -k 10 300 python -u tools/lib_parity.py $L tests/test_gpu_paths.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "fused_split_k or gemm or golden" > gpurun_out/pser_test.log 2>&1 || { tail -30 gpurun_out/pser_test.log; exit 1; }
tail -1 gpurun_out/pser_test.log
CFGS="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128 q6_k_28672x8192_m128 q8_0_4096x4096_m64 q4_k_4096x4096_m16 q6_k_4096x4096_m32 q8_0_11008x4096_m128 q4_k_28672x8192_m128"
for i in 1 2; do
  timeout -k 10 150 python -u tools/gemm_tune.py --step $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/base /' | tee -a gpurun_out/pser_ab.txt || exit 1
  timeout -k 10 150 python -u tools/gemm_tune.py --step --lib=$L $CFGS 2>&1 | grep -v amdgpu.ids | sed "s/^/pser /" | tee -a gpurun_out/pser_ab.txt || exit 1
done
