#!/usr/bin/env bash
# The GPU-box recipes, one entry point (run through gpurun from the repo root):
#
#   bash tools/gpu.sh tests                 pytest -m gpu (one process, per-test timeout)
#   bash tools/gpu.sh bench [ARGS...]       bench.py (default: the driver's N=1 line)
#   bash tools/gpu.sh prof NAME -- CMD...   rocprofv3 --kernel-trace --stats of CMD -> gpurun_out/NAME
#   bash tools/gpu.sh pmc CFG...            PMC passes (one rocprofv3 run per counter group, --kernel-trace
#                                           beside --pmc only) of bench.py --config CFG -> gpurun_out/pmc
#   bash tools/gpu.sh traffic CFG...        HBM bytes per launch from FETCH_SIZE (tools/pmc_traffic.py)
#   bash tools/gpu.sh ab ARGS...            tools/ab.py: graph-timed A/B of tuning variants / builds
#   bash tools/gpu.sh ab SPEC...            interleaved A/B of tools/gemm_tune.py specs (AB_R rounds)
#   bash tools/gpu.sh dist                  bench.py's N > 1 path at world 1 over RCCL (BENCH_FORCE_DIST)
#   bash tools/gpu.sh round                 round-end measurements: FETCH_SIZE traffic per config (read by
#                                           bench.py into roofline.traffic), the PMC passes of the shipping
#                                           kernels, the default bench line, and rocprofv3 stats of that command
#
# Every GPU step runs under its own timeout; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
cmd=${1:-tests}; shift || true
case "$cmd" in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" ;;
bench)
  timeout -k 10 900 python -u bench.py "$@" ;;
prof)
  name=$1; shift; [ "${1:-}" = "--" ] && shift
  out=$ROOT/gpurun_out/$name; mkdir -p "$out"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- "$@" > "$out/stdout.txt" 2> "$out/stderr.txt"
  rc=$?; [ $rc -eq 0 ] || { tail -20 "$out/stderr.txt"; exit $rc; }
  python3 "$ROOT/tools/kstats.py" "$out/run_kernel_stats.csv" | tee "$out/kstats.txt" ;;
pmc)
  OUT=$ROOT/gpurun_out/pmc; mkdir -p "$OUT"
  PASSES=${PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES|TA_TA_BUSY_sum,TA_BUSY_avr,TCP_TCC_READ_REQ_sum,TCC_HIT_sum,TCC_MISS_sum|SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_INSTS_SALU|SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_ANY,SQ_WAIT_ANY"}
  cd /tmp && export TMPDIR=/tmp
  for cfg in "$@"; do
    IFS='|' read -ra PS <<< "$PASSES"
    i=0
    for p in "${PS[@]}"; do
      d="$OUT/$cfg/p$i"; mkdir -p "$d"
      timeout -s KILL 120 rocprofv3 --pmc ${p//,/ } --kernel-trace --output-format csv -d "$d" -o run -- \
        python3 "$ROOT/bench.py" --config "$cfg" --steps 10 --warmup 2 --no-cpu --quick > "$d/bench.json" 2> "$d/err.txt"
      rc=$?; echo "$cfg pass $i ($p): rc=$rc"
      [ $rc -eq 0 ] || { tail -5 "$d/err.txt"; exit $rc; }
      i=$((i+1))
    done
  done
  python3 "$ROOT/tools/pmc_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt" ;;
traffic)
  timeout -k 10 900 python3 tools/pmc_traffic.py "$@" ;;
ab)
  A=""
  for r in $(seq ${AB_R:-3}); do for s in "$@"; do A="$A $s"; done; done
  timeout -k 10 500 python tools/gemm_tune.py ${AB_LIB:+--lib=$AB_LIB} $A 2>&1 | grep kernel_us | python3 -c "
import sys, collections
d = collections.OrderedDict()
for l in sys.stdin:
    k, v = l.split()[0], float(l.split('kernel_us=')[1].split()[0])
    d.setdefault(k, []).append(v)
for k, v in d.items(): print(f'{k:60s} min={min(v):7.2f} med={sorted(v)[len(v)//2]:7.2f} all={v}')
" ;;
dist)
  BENCH_FORCE_DIST=1 timeout -k 10 400 python -u bench.py --steps ${STEPS:-50} --warmup 5 ;;
round)
  TCFGS=${TCFGS:-"q8_0_4096x4096_m128 q8_0_4096x4096_m1 q4_k_4096x4096_m1 q4_k_4096x4096_m16 q4_k_4096x4096_m128 q4_k_11008x4096_m1 q4_k_11008x4096_m16 q4_k_11008x4096_m128 q4_k_4096x11008_m1 q4_k_4096x11008_m128 q6_k_28672x8192_m1 q6_k_28672x8192_m128 q6_k_8192x28672_m1 q6_k_8192x28672_m128"}
  PCFGS=${PCFGS:-"q8_0_4096x4096_m128 q4_k_4096x11008_m128 q6_k_28672x8192_m128 q4_k_11008x4096_m16"}
  timeout -k 10 600 python3 tools/pmc_traffic.py $TCFGS > gpurun_out/round_traffic.log 2>&1 &&
  PASSES="FETCH_SIZE|SQ_VALU_MFMA_BUSY_CYCLES,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE|TA_BUSY_avr,TCC_HIT_sum,TCC_MISS_sum|SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VALU,SQ_INSTS_MFMA" \
    bash tools/gpu.sh pmc $PCFGS > gpurun_out/round_pmc.log 2>&1 &&
  timeout -k 10 600 python3 -u bench.py --detail gpurun_out/round_detail.json > gpurun_out/round_bench.json 2> gpurun_out/round_bench.err &&
  mkdir -p gpurun_out/round_prof && cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/round_prof" -o run -- \
    python3 "$ROOT/bench.py" > "$ROOT/gpurun_out/round_prof/bench.json" 2> "$ROOT/gpurun_out/round_prof/bench.err" &&
  python3 "$ROOT/tools/kstats.py" "$ROOT/gpurun_out/round_prof/run_kernel_stats.csv" > "$ROOT/gpurun_out/round_prof/kstats.txt" &&
  # the per-dispatch CSVs are summarized above (summary.txt, pmc_*.json, kstats.txt): drop them so
  # gpurun_out stays under the copy-back limit
  find "$ROOT/gpurun_out" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete ;;
*)
  echo "unknown recipe: $cmd" >&2; exit 2 ;;
esac
