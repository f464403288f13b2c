#!/bin/bash
# Round 6: the streaming GEMM's split-major 1-D order (default) vs the 3-D grid
# (lib/libgguf_mmq_rablzord0.so, -DGQ_SGEMM_ZORDER=0): parity tests, interleaved step A/B, and a
# FETCH_SIZE pass of each build on the four 128-token streaming shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rgemm.py tests/test_gpu_ilc.py tests/test_gpu_streams.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6_zord_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r6_zord_tests.txt; [ $rc -eq 0 ] || exit $rc
C="q6_k_28672x8192_m128 q6_k_8192x28672_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128 q8_0_11008x4096_m128 q6_k_28672x8192_m64"
ZL=gguf-triton-kernel_amd/lib/libgguf_mmq_rablzord0.so
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/gemm_tune.py --step $C | sed "s/^/zord /" || exit $?
  timeout -k 10 300 python3 tools/gemm_tune.py --step --lib=$ZL $C | sed "s/^/grid3d /" || exit $?
done 2>&1 | tee gpurun_out/r6_zord_raw.txt | grep kernel_us | awk '{print $1, $2, $4}' | sort | \
  awk '{k=$1" "$2; v[k]=v[k]" "$3} END {for (k in v) print k, v[k]}' | sort | tee gpurun_out/r6_zord_ab.txt
T="q6_k_28672x8192_m128 q6_k_8192x28672_m128 q4_k_11008x4096_m128 q4_k_4096x11008_m128"
PMC_LIB=gguf-triton-kernel_amd/lib/libgguf_mmq.so timeout -k 10 600 python3 tools/pmc_traffic.py $T > gpurun_out/r6_zord_traffic.txt 2>&1 || exit $?
PMC_LIB=$ZL timeout -k 10 600 python3 tools/pmc_traffic.py $T >> gpurun_out/r6_zord_traffic.txt 2>&1 || exit $?
python3 -c "
import json
for l in open('gpurun_out/r6_zord_traffic.txt'):
    if l.startswith('{'):
        d = json.loads(l); print(d['config'], d.get('lib'), round(d['traffic_over_alg'], 3), d['kernel'])"
