#!/bin/bash
# GEMM loop variants: parity under GQ_GEMM_PIPE=1, then interleaved A/B and the ablations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GQ_GEMM_PIPE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_paths.py > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
S=""
for c in q8_0_4096x4096_m128 q4_k_4096x4096_m128 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m16 q8_0_4096x4096_m64; do
  S="$S $c $c:GQ_GEMM_PIPE=1"
done
AB_R=3 bash tools/ab.sh $S > gpurun_out/pipe_ab.txt 2>&1; cat gpurun_out/pipe_ab.txt
[ -n "$ABL" ] && { AB_R=2 AB_LIB=gguf-triton-kernel_amd/lib/libgguf_mmq_abl.so bash tools/ab.sh $ABL > gpurun_out/abl.txt 2>&1; cat gpurun_out/abl.txt; }
true
