#!/bin/bash
# Round 6: the split-K reduce as split_reduce_kernel (16-byte units, vector exponent loads, every
# split in flight; default) vs gemm_reduce_f16_kernel (lib/libgguf_mmq_rablred1.so,
# -DGQ_REDUCE_V2=0): parity tests, then an interleaved step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_rgemm.py tests/test_gpu_ilc.py tests/test_gpu_streams.py \
  tests/test_gpu_parity.py tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_red_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_red_tests.txt; [ $rc -eq 0 ] || exit $rc
C="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q8_0_4096x4096_m64 q4_k_4096x4096_m16 q8_0_4096x4096_m16 q4_k_11008x4096_m128 q6_k_28672x8192_m128 q4_k_4096x11008_m128"
RL=gguf-triton-kernel_amd/lib/libgguf_mmq_rablred1.so
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py --step $C | sed "s/^/v2 /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --step --lib=$RL $C | sed "s/^/v1 /" || exit $?
done 2>&1 | tee gpurun_out/r6_red_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_red_ab.txt
