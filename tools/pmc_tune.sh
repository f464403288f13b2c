#!/usr/bin/env bash
# PMC passes over gemm_tune.py specs (one rocprofv3 run per counter group, --kernel-trace only).
# Usage: bash tools/pmc_tune.sh SPEC...   -> gpurun_out/pmct/<n>/p<i>/ + summary
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmct
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
PASSES=${PASSES:-"SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,GRBM_GUI_ACTIVE|SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_LDS|SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_VALU_MFMA_BUSY_CYCLES|FETCH_SIZE|SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_MFMA|TA_TA_BUSY_sum,TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum"}
n=0
for spec in "$@"; do
  IFS='|' read -ra PS <<< "$PASSES"
  i=0
  for p in "${PS[@]}"; do
    ctrs=${p//,/ }
    d="$OUT/$n/p$i"
    mkdir -p "$d"
    echo "$spec" > "$OUT/$n/spec.txt"
    timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$d" -o run -- \
        python3 "$ROOT/tools/gemm_tune.py" "$spec" > "$d/out.txt" 2> "$d/err.txt"
    rc=$?
    echo "$spec pass $i ($ctrs): rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$d/err.txt"; if [ $rc -ge 124 ]; then exit $rc; fi; fi
    i=$((i+1))
  done
  n=$((n+1))
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
