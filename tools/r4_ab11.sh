#!/bin/bash
# Round-4 batch 11: where the grouped streaming GEMM's time goes in the 7B layer at 16 / 32 tokens:
# rocprofv3 kernel stats, then one PMC pass per counter group (--kernel-trace beside --pmc only).
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/lpmc; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/tools/layer_time.py" 16,32 --grouped-only > "$OUT/prof.txt" 2>&1 || exit $?
python3 "$ROOT/tools/kstats.py" "$OUT/prof/run_kernel_stats.csv" > "$OUT/kstats.txt"
i=0
for p in "SQ_WAVES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES" "SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_MFMA" \
         "SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_ANY,SQ_WAIT_ANY" "FETCH_SIZE" "TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum"; do
  d="$OUT/layer/p$i"; mkdir -p "$d"
  timeout -s KILL 120 rocprofv3 --pmc ${p//,/ } --kernel-trace --output-format csv -d "$d" -o run -- \
    python3 "$ROOT/tools/layer_time.py" 16,32 --grouped-only > "$d/out.txt" 2>&1
  rc=$?; echo "pass $i ($p): rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$d/out.txt"; exit $rc; }
  i=$((i+1))
done
python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
cat "$OUT/kstats.txt" | head -30
