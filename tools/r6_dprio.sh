#!/bin/bash
# Round 6: issue priority in the decode kernel (A/B builds): dprio1 = waves 4-7 lead for the first
# half of their tasks, waves 0-3 for the rest; dprio3 = waves 4-7 at priority 1 throughout;
# against none (the product).  Stamps by wave index first (product and dprio1 stamps builds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="q6_k_8192x28672_m1 q6_k_28672x8192_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1"
timeout -k 10 300 python3 tools/decode_stamps.py $S > gpurun_out/r6_dstamps2.txt 2>&1 &&
GQ_STAMPS_SO=stampsp1 timeout -k 10 300 python3 tools/decode_stamps.py $S > gpurun_out/r6_dstamps2_p1.txt 2>&1
rc=$?; grep -E "waves=|by wave" gpurun_out/r6_dstamps2.txt gpurun_out/r6_dstamps2_p1.txt; [ $rc -eq 0 ] || exit $rc
L=gguf-triton-kernel_amd/lib
BC="q4_k_4096x4096_m1 q6_k_28672x8192_m1 q8_0_4096x4096_m2 q4_k_11008x4096_m4 layer_m1 layer_m2"
timeout -k 10 300 python3 tools/lib_bits.py $BC > gpurun_out/r6_dprio_bits0.txt 2>&1 || exit $?
for v in 1 3; do
  timeout -k 10 300 python3 tools/lib_bits.py --lib=$L/libgguf_mmq_dprio$v.so $BC > gpurun_out/r6_dprio_bits$v.txt 2>&1 || exit $?
  diff gpurun_out/r6_dprio_bits0.txt gpurun_out/r6_dprio_bits$v.txt || { echo "dprio$v bits differ"; exit 1; }
done
echo "bits identical"
C="q8_0_4096x4096_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1 q4_k_4096x11008_m1 q6_k_28672x8192_m1 q6_k_8192x28672_m1"
for r in 1 2; do
  for v in 0 1 3; do
    if [ $v = 0 ]; then a=""; else a="--lib=$L/libgguf_mmq_dprio$v.so"; fi
    timeout -k 10 300 python3 tools/gemm_tune.py --step $a $C | sed "s/^/dprio$v /" || exit $?
  done
done 2>&1 | tee gpurun_out/r6_dprio_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_dprio_ab.txt
for r in 1 2; do
  for v in 0 1 3; do
    if [ $v = 0 ]; then a=""; else a="--lib $L/libgguf_mmq_dprio$v.so"; fi
    timeout -k 10 300 python3 tools/layer_time.py 1,2,4 --grouped-only $a | sed "s/^/dprio$v /" || exit $?
  done
done 2>&1 | grep points | tee gpurun_out/r6_dprio_layer.txt
