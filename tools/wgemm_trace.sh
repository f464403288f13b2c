#!/bin/bash
# Kernel trace of the 4096^2 x 128 GEMMs (old LDS-DMA kernel vs weight-register kernel):
# per-kernel durations, to split GEMM / split-K reduce / gaps.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace_q8
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_q8 -o run -- python3 -u tools/wgemm_check.py --only-time --variants ${VARIANTS:-old,w_rg1_nb8_wd3} --configs ${CONFIGS:-q8_0_4096x4096_m128,q4_k_4096x4096_m128}
