#!/bin/bash
# End-of-session evidence: smoke, default bench line, rocprof kernel stats + PMC passes
set -o pipefail
mkdir -p gpurun_out/final
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail -20 gpurun_out/final/bench_default.err; exit 2; }
tail -c 1500 gpurun_out/final/bench_default.json
timeout -k 10 900 bash tools/round2_prof.sh > gpurun_out/final/prof.log 2>&1 || { tail -20 gpurun_out/final/prof.log; exit 3; }
tail -5 gpurun_out/final/prof.log
