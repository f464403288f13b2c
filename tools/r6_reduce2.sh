#!/bin/bash
# Round 6: the K-chunked stream's K-range reduce with 8 ranges in flight (kstream_reduce_kernel;
# default) against one range per iteration (lib/libgguf_mmq_red1.so: -DGQ_KRED_V2=0): GPU tests
# of the grouped / K-chunked paths, then interleaved step and 7B-layer A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_grouped.py tests/test_gpu_kstream.py tests/test_gpu_grouped.py \
  tests/test_gpu_ilc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_red2_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_red2_tests.txt; [ $rc -eq 0 ] || exit $rc
RL=gguf-triton-kernel_amd/lib/libgguf_mmq_red1.so
C="q4_k_4096x11008_m16 q6_k_4096x11008_m16 q4_k_4096x28672_m16"
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py $C | sed "s/^/v2 /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --lib=$RL $C | sed "s/^/v1 /" || exit $?
done 2>&1 | tee gpurun_out/r6_red2_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_red2_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 8,16,24,40,64,128 --grouped-only | sed "s/^/v2 /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 8,16,24,40,64,128 --grouped-only --lib $RL | sed "s/^/v1 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_red2_layer.txt
