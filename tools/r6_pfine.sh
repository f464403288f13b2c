#!/bin/bash
# Round 6: the K-chunked stream's issue priority in four levels (rank 0-3 -> 0, 4-5 -> 1, 6 -> 2, last -> 3;
# lib/libgguf_mmq_pfine.so) against three (0-3 -> 0, 4-6 -> 1, last -> 2; the product): tests, bits, A/B.
#
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kstream.py tests/test_gpu_gemm_grouped.py tests/test_gpu_grouped.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_pfine_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_pfine_tests.txt; [ $rc -eq 0 ] || exit $rc
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_pfine.so
BC="q4_k_4096x4096_m32 q4_k_11008x4096_m17 q4_k_4096x11008_m28 q6_k_4096x4096_m32 q8_0_4096x2816_m21 q4_k_4096x4096_m16 q4_k_4096x11008_m12 layer_m32 layer_m24 layer_m16 layer_m7"
timeout -k 10 300 python3 tools/lib_bits.py --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_pfine_bits1.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_pfine_bits2.txt 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
diff gpurun_out/r6_pfine_bits1.txt gpurun_out/r6_pfine_bits2.txt && echo "bits identical" || { echo "bits differ"; exit 1; }
C="q4_k_4096x4096_m32 q4_k_4096x4096_m16 q4_k_11008x4096_m24 q4_k_22016x4096_m32 q4_k_22016x4096_m16 q6_k_4096x4096_m32 q8_0_4096x4096_m32"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$VL $C | sed "s/^/fine /" || exit $?
done 2>&1 | tee gpurun_out/r6_pfine_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_pfine_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only --lib $VL | sed "s/^/fine /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_pfine_layer.txt
