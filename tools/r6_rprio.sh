#!/bin/bash
# Round 6: issue priority in the resident / streaming GEMMs (A/B builds): rprio1 = waves 4-7 lead
# until the resident GEMM's second half multiply, waves 0-3 after; rprio3 = waves 4-7 at priority 1
# throughout (both GEMMs); against none (the product): bits, step A/B, the layer at 64-512 tokens.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=gguf-triton-kernel_amd/lib
BC="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m64 q4_k_11008x4096_m128 layer_m128"
timeout -k 10 300 python3 tools/lib_bits.py $BC > gpurun_out/r6_rprio_bits0.txt 2>&1 || exit $?
for v in 1 3; do
  timeout -k 10 300 python3 tools/lib_bits.py --lib=$L/libgguf_mmq_rprio$v.so $BC > gpurun_out/r6_rprio_bits$v.txt 2>&1 || exit $?
  diff gpurun_out/r6_rprio_bits0.txt gpurun_out/r6_rprio_bits$v.txt || { echo "rprio$v bits differ"; exit 1; }
done
echo "bits identical"
C="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q8_0_4096x4096_m64 q4_k_11008x4096_m128 q6_k_28672x8192_m128"
for r in 1 2; do
  for v in 0 1 3; do
    if [ $v = 0 ]; then a=""; else a="--lib=$L/libgguf_mmq_rprio$v.so"; fi
    timeout -k 10 300 python3 tools/gemm_tune.py --step $a $C | sed "s/^/rprio$v /" || exit $?
  done
done 2>&1 | tee gpurun_out/r6_rprio_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_rprio_ab.txt
for r in 1 2; do
  for v in 0 1 3; do
    if [ $v = 0 ]; then a=""; else a="--lib $L/libgguf_mmq_rprio$v.so"; fi
    timeout -k 10 300 python3 tools/layer_time.py 64,128,512 --grouped-only $a | sed "s/^/rprio$v /" || exit $?
  done
done 2>&1 | grep points | tee gpurun_out/r6_rprio_layer.txt
