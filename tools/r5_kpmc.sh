#!/bin/bash
# Round 5: PMC passes (one rocprofv3 run per counter group, --kernel-trace beside --pmc only) of
# tools/gemm_tune.py SPEC (default: the K-chunked streaming MMQ on Q4_K 22016x4096 x16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
SPEC=${SPEC:-q4_k_22016x4096_m16:GQ_KSTREAM=1}
OUT=$ROOT/gpurun_out/kpmc; mkdir -p "$OUT"
PASSES=${PASSES:-"SQ_WAVES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES|SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_MFMA|SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_ANY,SQ_WAIT_ANY|SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_ANY|TA_TA_BUSY_sum,TA_BUSY_avr,TCP_TCC_READ_REQ_sum"}
cd /tmp && export TMPDIR=/tmp
IFS='|' read -ra PS <<< "$PASSES"
i=0
for p in "${PS[@]}"; do
  d="$OUT/k/p$i"; mkdir -p "$d"
  timeout -s KILL 120 rocprofv3 --pmc ${p//,/ } --kernel-trace --output-format csv -d "$d" -o run -- \
    python3 "$ROOT/tools/gemm_tune.py" $SPEC > "$d/out.txt" 2> "$d/err.txt"
  rc=$?; echo "pass $i ($p): rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$d/err.txt"; exit $rc; }
  i=$((i+1))
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
