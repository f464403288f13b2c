#!/usr/bin/env bash
# bench.py's N > 1 path on a 1-GPU gpurun box: world 1 through the same code (BENCH_FORCE_DIST=1:
# RCCL process group, every all_gather captured into the HIP graphs; speedup_vs_1gpu ~ 1).
# The 2-rank launcher and line are covered on the CPU by tests/test_dist_gloo.py (gloo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_FORCE_DIST=1 timeout -k 10 400 python -u bench.py --steps ${STEPS:-50} --warmup 5 \
  > gpurun_out/dist1_rccl.json 2> gpurun_out/dist1_rccl.err
rc=$?; cat gpurun_out/dist1_rccl.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/dist1_rccl.err; exit $rc; }
