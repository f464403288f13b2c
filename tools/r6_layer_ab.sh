#!/bin/bash
# Round 6: the 7B layer M-sweep of the round-4 tree (ab_r4/: commit 354c853 built in-tree, its own
# bench.py) against this tree, interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for t in ab_r4 .; do
    echo "== round $r tree $t"
    timeout -k 10 400 python3 $t/bench.py --layer-only --steps 20 --warmup 5 > gpurun_out/r6_layer_${r}_$(basename $(realpath $t)).json 2> gpurun_out/r6_layer_err.txt || { tail -5 gpurun_out/r6_layer_err.txt; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6_layer_*_*.json")):
    d = json.load(open(f))
    for blk, (fused, grouped) in zip(d, [(True, "auto"), (True, False), (False, "auto"), (False, False)]):
        pts = blk["points"]
        print(f.split("/")[-1], "fused" if fused else "unfused", "grouped" if grouped else "per-call",
              " ".join(f"{p['M_tok']}:{p['us_per_step']}" for p in pts))
PY
