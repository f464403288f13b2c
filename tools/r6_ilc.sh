#!/bin/bash
# Round 6: the resident GEMM's in-launch split-K combine -- GPU tests, then an interleaved A/B of
# the step (gq_mmq) and the prepared kernel against the two-launch form (GQ_RGEMM_ILC=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_ilc.py tests/test_gpu_rgemm.py tests/test_gpu_streams.py} \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/r6_ilc_tests.txt 2>&1
  rc=$?; tail -5 gpurun_out/r6_ilc_tests.txt; [ $rc -eq 0 ] || exit $rc
fi
C=${CFGS:-"q8_0_4096x4096_m128 q4_k_4096x4096_m128 q6_k_4096x4096_m128 q8_0_4096x4096_m64 q4_k_4096x4096_m16 q8_0_4096x4096_m16"}
S=""
for c in $C; do S="$S $c $c:GQ_RGEMM_ILC=0"; done
for r in $(seq ${R:-3}); do
  timeout -k 10 300 python3 tools/gemm_tune.py --step $S | sed "s/^/step /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py $S | sed "s/^/kern /" || exit $?
done 2>&1 | tee gpurun_out/r6_ilc_ab_raw.txt | grep kernel_us | awk '{print $1, $2, $3}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_ilc_ab.txt
