#!/bin/bash
# Round 6: decode with waves 4-7 at issue priority 1 until the activation barrier (they are the ones
# it waits for), none after (lib/libgguf_mmq_dprio4.so, -DGQ_DECODE_PRIO=4) against none (the
# product): stamps of both (prologue / barrier), bits, step and 7B-layer A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="q6_k_8192x28672_m1 q6_k_28672x8192_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1"
timeout -k 10 300 python3 tools/decode_stamps.py $S > gpurun_out/r6_dstamps3.txt 2>&1 &&
GQ_STAMPS_SO=stampsp4 timeout -k 10 300 python3 tools/decode_stamps.py $S > gpurun_out/r6_dstamps3_p4.txt 2>&1
rc=$?; grep -E "waves=|prologue:|by wave" gpurun_out/r6_dstamps3.txt gpurun_out/r6_dstamps3_p4.txt; [ $rc -eq 0 ] || exit $rc
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_dprio4.so
BC="q4_k_4096x4096_m1 q6_k_28672x8192_m1 q8_0_4096x4096_m2 q4_k_11008x4096_m4 layer_m1 layer_m2"
timeout -k 10 300 python3 tools/lib_bits.py $BC > gpurun_out/r6_dprio4_bits0.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL $BC > gpurun_out/r6_dprio4_bits4.txt 2>&1 || exit $?
diff gpurun_out/r6_dprio4_bits0.txt gpurun_out/r6_dprio4_bits4.txt && echo "bits identical" || { echo "bits differ"; exit 1; }
C="q8_0_4096x4096_m1 q4_k_4096x4096_m1 q4_k_11008x4096_m1 q4_k_4096x11008_m1 q6_k_28672x8192_m1 q6_k_8192x28672_m1"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py --step $C | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --step --lib=$VL $C | sed "s/^/p4 /" || exit $?
done 2>&1 | tee gpurun_out/r6_dprio4_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_dprio4_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 1,2,4 --grouped-only | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 1,2,4 --grouped-only --lib $VL | sed "s/^/p4 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_dprio4_layer.txt
