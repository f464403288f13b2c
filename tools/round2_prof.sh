#!/usr/bin/env bash
# Round-end evidence: rocprofv3 kernel-trace stats of the default bench, PMC passes on the
# headline GEMM, the Q6_K 70B GEMM and decode.  Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/r02prof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o bench -- \
    python3 $R/bench.py --steps 30 --warmup 5 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 5; }
python3 $R/tools/kstats.py $OUT/bench/bench_kernel_stats.csv > $OUT/kernel_stats_summary.txt
cat $OUT/kernel_stats_summary.txt | head -30
cd $R && bash tools/pmc.sh q8_0_4096x4096_m128 q6_k_28672x8192_m128 q4_k_4096x4096_m128 q6_k_28672x8192_m1 > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 6; }
cp gpurun_out/pmc/summary.txt $OUT/pmc_summary.txt
echo ALL_DONE
