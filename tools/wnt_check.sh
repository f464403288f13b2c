#!/bin/bash
# nt cache policy on the GEMM's weight DMA (GQ_GEMM_WNT=1 build) vs default policy; weights rotated over >= 1 GiB (cold, as bench.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
L=gguf-triton-kernel_amd/lib/libgguf_mmq_wnt.so
timeout -k 10 300 python -u tools/lib_parity.py $L tests/test_gpu_paths.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "fused_split_k or gemm or golden" > gpurun_out/wnt_test.log 2>&1 || { tail -30 gpurun_out/wnt_test.log; exit 1; }
tail -1 gpurun_out/wnt_test.log
CFGS="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128 q6_k_28672x8192_m128 q8_0_4096x4096_m64 q4_k_4096x4096_m16 q6_k_4096x4096_m32"
for i in 1 2; do
  timeout -k 10 150 python -u tools/gemm_tune.py --step $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/base /' | tee -a gpurun_out/wnt_ab.txt || exit 1
  timeout -k 10 150 python -u tools/gemm_tune.py --step --lib=$L $CFGS 2>&1 | grep -v amdgpu.ids | sed 's/^/wnt  /' | tee -a gpurun_out/wnt_ab.txt || exit 1
done
