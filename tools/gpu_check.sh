#!/usr/bin/env bash
# One GPU-box session: parity tests, smoke, bench (+ sweep), rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-100}

timeout -k 10 900 python -m pytest tests -m gpu -q -rf > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest -m gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 3; }
cat "$OUT/smoke.log"

timeout -k 10 900 python bench.py --steps "$STEPS" --warmup 10 ${BENCH_ARGS:---sweep} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"

if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
      python3 "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu ${PROF_ARGS:---sweep} > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed"; tail -20 "$OUT/prof.err"; exit 5; }
  find "$OUT/prof" -name "*stats*" | head
fi
echo ALL_DONE
