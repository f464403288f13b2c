#!/bin/bash
# Copy a closing run's results (tools/r6_final.sh, merged into gpurun_out/) into the tracked
# profiles: profiles/r06/final/ and the per-config FETCH records profiles/pmc_<config>.json.
cd "$(dirname "$0")/.."
set -e
D=profiles/r06/final
mkdir -p $D
cp gpurun_out/round_bench.json gpurun_out/round_detail.json gpurun_out/round_traffic.log gpurun_out/round_smoke.txt $D/
cp gpurun_out/round_prof/kstats.txt $D/kstats.txt
cp gpurun_out/round_prof/run_kernel_stats.csv $D/run_kernel_stats.csv 2>/dev/null || \
  cp "$(ls gpurun_out/round_prof/*kernel_stats.csv | head -1)" $D/run_kernel_stats.csv
cp gpurun_out/pmc/summary.txt $D/pmc_summary.txt
for f in gpurun_out/pmc_traffic/pmc_*.json; do cp "$f" profiles/; done
ls -la $D
