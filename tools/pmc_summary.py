"""Aggregate rocprofv3 --pmc CSVs under a directory: mean counter value per (config, kernel)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
res = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "p*", "**", "*counter_collection.csv"), recursive=True):
    cfg = os.path.relpath(f, root).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))
        if "gq::" not in k:
            continue
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("gq::", "")
        res[(cfg, short)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (cfg, k), ctrs in sorted(res.items()):
    print(f"{cfg:24s} {k}")
    for c, v in sorted(ctrs.items()):
        print(f"    {c:28s} mean={sum(v) / len(v):14.1f}  n={len(v)}")
