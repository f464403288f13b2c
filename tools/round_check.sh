#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, PMC HBM traffic per config, bench (+ sweep) that
# reads that traffic, rocprofv3 kernel-trace summary.  Each GPU step has its own time limit;
# a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 3; }
cat "$OUT/smoke.log"
timeout -k 10 600 python tools/pmc_traffic.py ${PMC_CONFIGS:-} > "$OUT/pmc_traffic.log" 2>&1 || { tail -5 "$OUT/pmc_traffic.log"; exit 4; }
timeout -k 10 900 python bench.py --steps ${STEPS:-100} --warmup 10 --sweep > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 5; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu --sweep > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { tail -20 "$OUT/prof.err"; exit 6; }
echo ALL_DONE
