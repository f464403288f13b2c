#!/usr/bin/env python3
"""Token sweep of the drop-in step (gq_mmq: activation quantization + MMQ) on the BASELINE
shapes: us per step (graph of 50 calls over >= 1 GiB of weight copies, best of 3) and the
weight-stream rate.  python tools/msweep.py [--shapes q4_k:4096:4096,...] [--tokens 1,2,...]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="q4_k:4096:4096,q4_k:11008:4096,q8_0:4096:4096,q6_k:28672:8192")
    ap.add_argument("--tokens", default="1,2,4,5,8,12,16,17,24,32,48,64")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--tune", default="", help="KEY=V,... library tuning overrides (gq_debug_set_tuning)")
    ap.add_argument("--lib", default=None, help="another build of libgguf_mmq.so (diagnostic variants)")
    ap.add_argument("--act", default="q8_1", help="activation format: q8_1 or fp8")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    import kernels._lib as kl
    if a.lib:
        kl.LIB_PATH = os.path.abspath(a.lib)
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        kl.set_tuning(k, int(v))
    for shp in a.shapes.split(","):
        fmt, M, K = shp.split(":")
        M, K = int(M), int(K)
        row = {"shape": shp, "act": a.act, "tune": a.tune, "lib": os.path.basename(kl.LIB_PATH), "us": {}, "hbm_frac": {}}
        for N in (int(t) for t in a.tokens.split(",")):
            r = bench.Runner(fmt, M, K, N, dev, a.steps, act=a.act)
            g = r.capture(r.step, [i % r.ncopies for i in range(a.steps)])
            g.replay()
            t = min(bench.timed_replay(g, dev) for _ in range(3)) / a.steps
            _, alg, _ = bench.model(fmt, M, K, N)
            row["us"][N] = round(t * 1e6, 2)
            row["hbm_frac"][N] = round(alg / t / 8e12, 3)
            del r, g
            torch.cuda.empty_cache()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
