#!/bin/bash
# Round 6: in-launch combine with the XCD-contiguous 1-D order, and the grouped stream-K combine:
# GPU tests, then the interleaved A/B (GQ_RGEMM_ILC=0 = two launches) on the resident, streaming
# and grouped (7B layer) shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ilc.py tests/test_gpu_gemm_grouped.py tests/test_gpu_streams.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_ilc2_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r6_ilc2_tests.txt; [ $rc -eq 0 ] || exit $rc
C="q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q8_0_4096x4096_m64 q6_k_28672x8192_m128 q6_k_8192x28672_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128"
S=""
for c in $C; do S="$S $c $c:GQ_RGEMM_ILC=0"; done
for r in 1 2; do
  timeout -k 10 400 python3 tools/gemm_tune.py --step $S | sed "s/^/step /" || exit $?
done 2>&1 | tee gpurun_out/r6_ilc2_ab_raw.txt | grep kernel_us | awk '{print $1, $2, $3}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_ilc2_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 40,64,128,256,512 --grouped-only || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 40,64,128,256,512 --grouped-only --tune GQ_RGEMM_ILC=0 || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_ilc2_layer.txt
