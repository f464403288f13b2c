#!/bin/bash
# (measured and removed: profiles/r06/kstream_nb4_ab.txt -- this script needs the round-6 commit 37193c3 tree)
# Round 6: the K-chunked stream at 33..64 tokens (four 16-token tiles, one super-block per wave,
# K ranges of 8 super-blocks; GQ_KSTREAM=1) -- parity first, then A/B against the default routes
# (resident / streaming GEMM) per matrix and on the 7B layer; then the NB=2 task-size A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kstream.py tests/test_gpu_gemm_grouped.py tests/test_gpu_grouped.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_nb4_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_nb4_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for n in 40 64; do
    C=""
    for s in q4_k_4096x4096 q4_k_11008x4096 q4_k_4096x11008 q6_k_4096x4096 q6_k_4096x11008 q8_0_4096x4096; do
      C="$C ${s}_m$n ${s}_m$n:GQ_KSTREAM=1"
    done
    timeout -k 10 300 python3 tools/gemm_tune.py $C || exit $?
  done
done 2>&1 | tee gpurun_out/r6_nb4_raw.txt | grep kernel_us | awk '{print $1, $3}' | sort | \
  awk '{v[$1]=v[$1]" "$2} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_nb4_ab.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 33,40,48,64 --grouped-only || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 33,40,48,64 --grouped-only --tune GQ_KSTREAM=1 || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_nb4_layer.txt
bash tools/r6_tsb.sh
