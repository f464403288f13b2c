#!/bin/bash
# Round 6: the K-chunked stream at 3..4 q8_1 tokens (lib/libgguf_mmq_nmin3.so: -DGQ_KSTREAM_NMIN=3;
# LayerMix with the grouped decode only up to 2 tokens: --decode-max 2) against the grouped decode
# at 3..4 (the product): bits of the stream's form, the 7B layer and prepared single matrices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_nmin3.so
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL q4_k_4096x4096_m3 q6_k_4096x11008_m4 q8_0_4096x4096_m4 > gpurun_out/r6_nmin3_bits.txt 2>&1
rc=$?; cat gpurun_out/r6_nmin3_bits.txt; [ $rc -eq 0 ] || exit $rc
C="q4_k_4096x4096_m3 q4_k_4096x4096_m4 q4_k_11008x4096_m4 q4_k_22016x4096_m4 q6_k_4096x4096_m4 q8_0_4096x4096_m4"
for r in 1 2; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$VL $C | sed "s/^/nmin3 /" || exit $?
done 2>&1 | tee gpurun_out/r6_nmin3_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_nmin3_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 2,3,4,5 --grouped-only | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 2,3,4,5 --grouped-only --lib $VL --decode-max 2 | sed "s/^/nmin3 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_nmin3_layer.txt
