#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per counter group; --kernel-trace only beside --pmc) for
# the configs given as arguments (bench.py config names).  Output: gpurun_out/pmc/<cfg>/<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
PASSES=${PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES|TA_TA_BUSY_sum,TA_BUSY_avr,TCP_TCC_READ_REQ_sum,TCC_HIT_sum,TCC_MISS_sum|SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU|SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_ANY,SQ_WAIT_ANY"}
for cfg in "$@"; do
  IFS='|' read -ra PS <<< "$PASSES"
  i=0
  for p in "${PS[@]}"; do
    ctrs=${p//,/ }
    d="$OUT/$cfg/p$i"
    mkdir -p "$d"
    timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$d" -o run -- \
        python3 "$ROOT/bench.py" --config "$cfg" --steps 10 --warmup 2 --no-cpu --quick > "$d/bench.json" 2> "$d/err.txt"
    rc=$?
    echo "$cfg pass $i ($ctrs): rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$d/err.txt"; if [ $rc -ge 124 ]; then exit $rc; fi; fi
    i=$((i+1))
  done
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
