#!/bin/bash
# (adopted: one super-block per task at 17..32 tokens is the product since this A/B; profiles/r06/kstream_tsb_ab.txt)
# Round 6: the K-chunked stream at 17..32 tokens with one Q4_K super-block per task (no register
# spill: 253 VGPRs, 0 scratch; lib/libgguf_mmq_tsb1.so) against two (the product: 256 VGPRs +
# 84 bytes of scratch): parity of the variant (lib_check), then interleaved A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_tsb1.so
# (the task size does not change a wave's summation order: the same bits)
BC="q4_k_4096x4096_m32 q4_k_11008x4096_m24 q4_k_4096x4096_m17 q4_k_4096x11008_m20 q6_k_4096x4096_m32"
timeout -k 10 300 python3 tools/lib_bits.py --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_tsb_bits2.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_tsb_bits1.txt 2>&1
rc=$?; cat gpurun_out/r6_tsb_bits2.txt gpurun_out/r6_tsb_bits1.txt; [ $rc -eq 0 ] || exit $rc
diff gpurun_out/r6_tsb_bits2.txt gpurun_out/r6_tsb_bits1.txt || { echo "TSB bits differ"; exit 1; }
C="q4_k_4096x4096_m32 q4_k_22016x4096_m32 q4_k_11008x4096_m24 q4_k_4096x4096_m20"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/tsb2 /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$VL $C | sed "s/^/tsb1 /" || exit $?
done 2>&1 | tee gpurun_out/r6_tsb_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_tsb_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 17,24,32 --grouped-only | sed "s/^/tsb2 /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 17,24,32 --grouped-only --lib $VL | sed "s/^/tsb1 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_tsb_layer.txt
