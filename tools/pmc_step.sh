#!/usr/bin/env bash
# PMC counters of the drop-in step (gemm_tune.py --step SPEC), one rocprofv3 pass per group.
# Usage: bash tools/pmc_step.sh SPEC [GROUP...]   (groups: comma-separated counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcs; mkdir -p "$OUT"
SPEC=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  d="$OUT/step/p$i"; mkdir -p "$d"
  timeout -k 10 120 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d "$d" -o run -- \
      python3 "$ROOT/tools/gemm_tune.py" --step $SPEC > "$d/out.txt" 2> "$d/err.txt"
  rc=$?; echo "pass $i ($grp): rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$d/err.txt"; exit $rc; }
  i=$((i+1))
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
