#!/bin/bash
# Round 6: the K-chunked stream's cross-wave hand-off with two scratch buffers (a wave may run a
# hand-off further ahead of the summing wave; lib/libgguf_mmq_dbuf.so, -DGQ_KSTREAM_DBUF=1)
# against one (the product): the layer's per-workgroup stamps first (product logic), then bits,
# then interleaved single-matrix and 7B-layer A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/kstream_layer_stamps.py 16 32 > gpurun_out/r6_klayer2.txt 2>&1
rc=$?; cat gpurun_out/r6_klayer2.txt; [ $rc -eq 0 ] || exit $rc
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_dbuf.so
BC="q4_k_4096x4096_m16 q4_k_11008x4096_m8 q4_k_4096x11008_m12 q6_k_4096x4096_m32 q4_k_4096x4096_m24 q8_0_4096x2816_m5 layer_m16 layer_m32 layer_m7"
timeout -k 10 300 python3 tools/lib_bits.py --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_dbuf_bits1.txt 2>&1 &&
timeout -k 10 300 python3 tools/lib_bits.py --lib=$VL --tune=GQ_KSTREAM=1 $BC > gpurun_out/r6_dbuf_bits2.txt 2>&1
rc=$?; cat gpurun_out/r6_dbuf_bits1.txt gpurun_out/r6_dbuf_bits2.txt; [ $rc -eq 0 ] || exit $rc
diff gpurun_out/r6_dbuf_bits1.txt gpurun_out/r6_dbuf_bits2.txt || { echo "DBUF bits differ"; exit 1; }
timeout -k 10 60 python3 -c "
import sys; sys.path[:0] = ['.', 'gguf-triton-kernel_amd']
import kernels._lib as kl; kl.LIB_PATH = '$VL'
import ctypes; f = kl.lib().gq_debug_sync_timeouts; f.restype = ctypes.c_uint; print('dbuf lib sync timeouts (fresh process):', f())"
C="q4_k_4096x4096_m16 q4_k_11008x4096_m16 q4_k_22016x4096_m16 q4_k_4096x4096_m32 q4_k_22016x4096_m32 q6_k_4096x4096_m32"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/one /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$VL $C | sed "s/^/two /" || exit $?
done 2>&1 | tee gpurun_out/r6_dbuf_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_dbuf_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only | sed "s/^/one /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 5,8,16,24,32 --grouped-only --lib $VL | sed "s/^/two /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_dbuf_layer.txt
