#!/bin/bash
# (measured, not taken: profiles/r06/kstream_tsb_nb1_ab.txt; the variant macro is gone)
# Round 6: the K-chunked stream at 5..16 tokens with one Q4_K super-block per task
# (lib/libgguf_mmq_t1nb1.so: -DGQ_KSTREAM_NB1_TSB=1) against two (the product): bits, then
# interleaved per-matrix (prepared) and 7B-layer A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kstream.py tests/test_gpu_gemm_grouped.py tests/test_gpu_grouped.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_t1nb1_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_t1nb1_tests.txt; [ $rc -eq 0 ] || exit $rc
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_t1nb1.so
BC="q4_k_4096x4096_m16 q4_k_11008x4096_m8 q4_k_4096x11008_m12 q4_k_4096x4096_m5"
timeout -k 10 300 python3 tools/lib_bits.py --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_t1nb1_bits2.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_t1nb1_bits1.txt 2>&1
rc=$?; cat gpurun_out/r6_t1nb1_bits2.txt gpurun_out/r6_t1nb1_bits1.txt; [ $rc -eq 0 ] || exit $rc
diff gpurun_out/r6_t1nb1_bits2.txt gpurun_out/r6_t1nb1_bits1.txt || { echo "TSB bits differ"; exit 1; }
C="q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_22016x4096_m8 q4_k_22016x4096_m16 q4_k_4096x4096_m8"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/tsb2 /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$VL $C | sed "s/^/tsb1 /" || exit $?
done 2>&1 | tee gpurun_out/r6_t1nb1_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_t1nb1_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16 --grouped-only | sed "s/^/tsb2 /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16 --grouped-only --lib $VL | sed "s/^/tsb1 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_t1nb1_layer.txt
