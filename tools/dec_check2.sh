#!/usr/bin/env bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dec_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/dec_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAIL" gpurun_out/dec_pytest.log | head; exit $rc; }
A=""
for c in q4_k_4096x4096_m1 q8_0_4096x4096_m1 q4_k_11008x4096_m1 q6_k_28672x8192_m1 q4_k_4096x4096_m2 q4_k_4096x4096_m4 q6_k_8192x28672_m1; do A="$A $c $c:GQ_DECODE_WIDE_ROWS=1"; done
timeout -k 10 300 python tools/gemm_tune.py --step $A 2>&1 | grep kernel_us
