"""Print rocprofv3 kernel_stats.csv rows (gq kernels first): calls, avg/min/max us."""
import csv
import glob
import sys

for f in sys.argv[1:] or glob.glob("gpurun_out/prof/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: ("gq::" not in r["Name"], r["Name"]))
    for r in rows:
        n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{n[:60]:60s} calls={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.2f} "
              f"min={float(r['MinNs'])/1e3:8.2f} max={float(r['MaxNs'])/1e3:8.2f} us")
