#!/bin/bash
# Round 6: issue priority in the K-chunked stream (A/B builds): prio1 = waves 4-7 at s_setprio 1
# (static), prio2 = by hand-off position (yield after arriving, the last arriver leads), against
# none (the product): bits, then interleaved single-matrix and 7B-layer A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gguf-triton-kernel_amd/lib
BC="q4_k_4096x4096_m32 q4_k_11008x4096_m17 q6_k_4096x4096_m32 q4_k_4096x4096_m16 q4_k_4096x11008_m12 layer_m32 layer_m16"
timeout -k 10 300 python3 tools/lib_bits.py --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_prio_bits0.txt 2>&1 || exit $?
for v in 1 2; do
  timeout -k 10 300 python3 tools/lib_bits.py --lib=$L/libgguf_mmq_prio$v.so --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_prio_bits$v.txt 2>&1 || exit $?
  diff gpurun_out/r6_prio_bits0.txt gpurun_out/r6_prio_bits$v.txt || { echo "prio$v bits differ"; exit 1; }
done
echo "bits identical"
C="q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_22016x4096_m16 q4_k_4096x4096_m32 q4_k_22016x4096_m32 q6_k_4096x4096_m32"
for r in 1 2; do
  for v in 0 1 2; do
    if [ $v = 0 ]; then a=""; else a="--lib=$L/libgguf_mmq_prio$v.so"; fi
    timeout -k 10 300 python3 tools/gemm_tune.py $a $C | sed "s/^/prio$v /" || exit $?
  done
done 2>&1 | tee gpurun_out/r6_prio_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_prio_ab.txt
for r in 1 2; do
  for v in 0 1 2; do
    if [ $v = 0 ]; then a=""; else a="--lib $L/libgguf_mmq_prio$v.so"; fi
    timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only $a | sed "s/^/prio$v /" || exit $?
  done
done 2>&1 | grep points | tee gpurun_out/r6_prio_layer.txt
