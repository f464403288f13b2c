"""Print a compact table of a bench.json line (+ sweep) and a rocprof kernel_stats csv."""
import csv
import json
import sys

b = json.load(open(sys.argv[1]))


def show(name, d, tf):
    r = d["roofline"]
    print(f"{name:24.24s} step_us={d['ms_per_step'] * 1000:8.2f} TF={tf:8.2f} wGB/s={d['weight_GBps']:8.1f} "
          f"kern_us={r['kernel_us']:8.2f} frac={r['frac']:.3f} {r['bound']}")


show(b["config"]["workload"], b, b["value"])
for s in b.get("sweep", []):
    show(s["config"], s, s["tflops"])
if b.get("cpu_baseline"):
    print("cpu_baseline TFLOP/s", b["cpu_baseline"]["value"])
if len(sys.argv) > 2:
    for r in csv.DictReader(open(sys.argv[2])):
        n = r["Name"]
        if "gq::" in n:
            n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            print(f"{n:40s} calls={r['Calls']:>5} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
                  f"min_us={float(r['MinNs']) / 1e3:8.2f}")
