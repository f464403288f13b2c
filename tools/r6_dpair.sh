#!/bin/bash
# (the two-row pass was measured neutral-to-slower and removed after this A/B: profiles/r06/decode_rowpair_ab.txt;
#  the dpair0 target went with it)
# Round 6: decode with two-row passes (default) vs without (lib/libgguf_mmq_dpair0.so): the decode
# parity tests, then interleaved step A/B at one token and the 7B layer at 1-2 tokens.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grouped.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r6_dpair_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_dpair_tests.txt; [ $rc -eq 0 ] || exit $rc
C="q4_k_4096x4096_m1 q8_0_4096x4096_m1 q4_k_11008x4096_m1 q4_k_4096x11008_m1 q6_k_4096x4096_m1 q4_k_4096x4096_m2 q6_k_28672x8192_m1"
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/gemm_tune.py --step $C | sed "s/^/pair /" || exit $?
  timeout -k 10 200 python3 tools/gemm_tune.py --step --lib=gguf-triton-kernel_amd/lib/libgguf_mmq_dpair0.so $C | sed "s/^/nopair /" || exit $?
done 2>&1 | tee gpurun_out/r6_dpair_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_dpair_ab.txt
for r in 1 2; do
  timeout -k 10 200 python3 tools/layer_time.py 1,2 --grouped-only | sed "s/^/pair /" || exit $?
  timeout -k 10 200 python3 tools/layer_time.py 1,2 --grouped-only --lib gguf-triton-kernel_amd/lib/libgguf_mmq_dpair0.so | sed "s/^/nopair /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_dpair_layer.txt
