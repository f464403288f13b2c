#!/usr/bin/env bash
# rocprof kernel stats per ablation mask (pure kernel durations, no launch gaps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/ablprof; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for a in ${MASKS:-0 15 6 1}; do
  GQ_ABLATE=$a timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/m$a" -o run -- \
      python3 "$ROOT/tools/ablate.py" ${1:-q8_0_4096x4096_m128} ${LIB:-} > "$OUT/m$a.txt" 2>&1 || { echo "mask $a failed"; tail -5 "$OUT/m$a.txt"; exit 1; }
  echo "== mask $a"; grep ablate= "$OUT/m$a.txt"
  python3 - "$OUT/m$a" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gq::" in r["Name"]:
            n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            print(f"   {n:40s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f}")
PY
done
