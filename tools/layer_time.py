#!/usr/bin/env python3
"""Q4_K_M Llama-7B layer (bench.bench_layer) at decode sizes, grouped vs one launch per set.
python tools/layer_time.py [Ns] [--lib other-build.so] [--grouped-only] [--tune KEY=V,...] [--act fp8]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
args = [a for a in sys.argv[1:]]
lib = args[args.index("--lib") + 1] if "--lib" in args else None
if lib:
    import kernels._lib as kl
    kl.LIB_PATH = os.path.abspath(lib)
if "--tune" in args:  # library tuning overrides (gq_debug_set_tuning)
    import kernels._lib as kl
    for kv in filter(None, args[args.index("--tune") + 1].split(",")):
        k, v = kv.split("=")
        kl.set_tuning(k, int(v))
if "--decode-max" in args:  # q8_1: the grouped decode up to D tokens, prepared + grouped GEMM / stream from D + 1
    import kernels.layer_mix as lm
    D = int(args[args.index("--decode-max") + 1])
    lm.GROUPED_MAX_TOKENS[True] = D
    lm.GEMM_GROUPED_MIN_TOKENS[True] = D + 1
    lm.PREPARED_MIN_TOKENS["q8_1"] = D + 1
act = args[args.index("--act") + 1] if "--act" in args else "q8_1"
gmin = int(args[args.index("--gemm-min") + 1]) if "--gemm-min" in args else None  # LayerMix gemm_grouped_min
pos = [a for i, a in enumerate(args)
       if not a.startswith("--") and (i == 0 or args[i - 1] not in ("--lib", "--tune", "--act", "--gemm-min", "--decode-max"))]
Ns = tuple(int(n) for n in (pos[0] if pos else "1,2,3,4").split(","))
for grouped in ((True,) if "--grouped-only" in args else (True, False)):  # (True: grouped at 1..4 tokens)
    r = bench.bench_layer(Ns, (act,), 50, 5, dev, fuse=True, grouped=grouped, gemm_grouped_min=gmin)
    print(json.dumps({"grouped": grouped, "act": act, "tune": args[args.index("--tune") + 1] if "--tune" in args else "", "gemm_min": gmin, "lib": os.path.basename(lib or "libgguf_mmq.so"), "weight_bytes": r["weight_bytes"],
                      "points": [(p["M_tok"], p["us_per_step"], p["weight_GBps"]) for p in r["points"]]}), flush=True)
