#!/bin/bash
# Round 6: VALU / MFMA / LDS counters of the K-chunked stream on prepared calls (the raw call's
# count includes every workgroup's in-kernel quantization of its x chunk): per config one
# rocprofv3 --pmc pass (its own run) over tools/gemm_tune.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for cfg in q4_k_11008x4096_m16 q4_k_22016x4096_m32 q6_k_4096x4096_m32 q4_k_11008x4096_m8; do
  OUT=$ROOT/gpurun_out/r6_kpmc/$cfg; mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace \
    --output-format csv -d "$OUT" -o run -- python3 "$ROOT/tools/gemm_tune.py" $cfg > "$OUT/tune.txt" 2> "$OUT/err.txt" \
    || { tail -5 "$OUT/err.txt"; exit 1; }
  python3 - "$OUT" "$cfg" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "").replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if "kstream_kernel" in k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(sys.argv[2], k, {n: round(x) for n, x in m.items()}, "dispatches", len(next(iter(c.values()))),
          "VALU/MFMA %.1f" % (m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]), flush=True)
PY
  find "$OUT" -name "*counter_collection.csv" -delete
done 2>&1 | tee "$ROOT/gpurun_out/r6_kpmc/summary.txt"
