#!/usr/bin/env python3
"""Q4_K_M Llama-7B layer (bench.bench_layer) at decode sizes, grouped vs one launch per set."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
Ns = tuple(int(n) for n in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(","))
for grouped in (True, False):  # (True: grouped at 1..4 tokens)
    r = bench.bench_layer(Ns, ("q8_1",), 50, 5, dev, fuse=True, grouped=grouped)
    print(json.dumps({"grouped": grouped, "weight_bytes": r["weight_bytes"],
                      "points": [(p["M_tok"], p["us_per_step"], p["weight_GBps"]) for p in r["points"]]}), flush=True)
