#!/usr/bin/env python3
"""Resident-split GEMM (mmq_rgemm.hip) A/B: graph-timed us per MMQ call over >= 1 GiB of weight
copies, prepared activations (the MMQ alone) and the whole step (gq_mmq: quantization included),
against the library's other GEMM routes (GQ_RGEMM=0).

  python tools/rgemm_check.py [--configs a,b] [--rounds R]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import wgemm_check as W  # noqa: E402

CONFIGS = dict(W.CONFIGS)
CONFIGS.update({"q6_k_4096x4096_m128": ("q6_k", 4096, 4096, 128), "q8_0_4096x4096_m32": ("q8_0", 4096, 4096, 32),
                "q4_k_4096x4096_m32": ("q4_k", 4096, 4096, 32), "q8_0_2048x4096_m128": ("q8_0", 2048, 4096, 128),
                "q8_0_8192x4096_m128": ("q8_0", 8192, 4096, 128), "q4_k_4096x4096_m96": ("q4_k", 4096, 4096, 96),
                "q8_0_11008x4096_m128": ("q8_0", 11008, 4096, 128), "q6_k_11008x4096_m128": ("q6_k", 11008, 4096, 128)})


def parse_cfg(name):
    """A CONFIGS name, or any "<fmt>_<M>x<K>_m<N>" (e.g. q6_k_28672x8192_m2)."""
    if name in CONFIGS:
        return CONFIGS[name]
    fmt, mk, n = name.rsplit("_", 2)
    M, K = (int(v) for v in mk.split("x"))
    return fmt, M, K, int(n[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="q8_0_4096x4096_m128,q4_k_4096x4096_m128,q6_k_4096x4096_m128,"
                                          "q8_0_4096x4096_m64,q4_k_4096x4096_m64,q8_0_4096x4096_m32")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="rgemm=GQ_RGEMM:1,old=GQ_RGEMM:0")
    ap.add_argument("--libs", default=None,
                    help="name=path,... : time each build (ablations) under the first --variants entry "
                         "(default GQ_RGEMM=1)")
    ap.add_argument("--steps-only", action="store_true", help="time the step (gq_mmq) only")
    a = ap.parse_args()
    if a.libs:  # one process per build would cost minutes: load each .so under its own handle
        import kernels._lib as kl
        v0 = a.variants.split(",")[0].split("=", 1)[1]
        lcfg = {k: int(x) for k, x in (p.split(":") for p in v0.split("+"))}
        for name in a.configs.split(","):
            fmt, M, K, N = parse_cfg(name)
            row = {"config": name}
            for spec in a.libs.split(","):
                lname, path = spec.split("=")
                kl._lib, kl._mmq_ex, kl.LIB_PATH = None, None, path
                kl._call_ws.clear()
                for prep in ((False,) if a.steps_only else (True, False)):
                    us = min(W.time_cfg(fmt, M, K, N, torch.device("cuda:0"), lcfg, prepared=prep)
                             for _ in range(a.rounds))
                    row[lname + ("_mmq" if prep else "_step")] = round(us, 2)
            print(json.dumps(row), flush=True)
        return
    dev = torch.device("cuda:0")
    variants = []
    for v in a.variants.split(","):
        name, kv = v.split("=")
        cfg = {k: int(x) for k, x in (p.split(":") for p in kv.split("+"))}
        variants.append((name, cfg))
    for name in a.configs.split(","):
        fmt, M, K, N = parse_cfg(name)
        flops = 2.0 * M * N * K
        row = {"config": name}
        for r in range(a.rounds):
            for vname, cfg in variants:
                for prep in ((False,) if a.steps_only else (True, False)):
                    us = W.time_cfg(fmt, M, K, N, dev, cfg, prepared=prep)
                    key = vname + ("_mmq" if prep else "_step")
                    row[key] = min(row.get(key, 1e9), round(us, 2))
        for k in list(row):
            if k.endswith("_step") or k.endswith("_mmq"):
                row[k + "_tf"] = round(flops / row[k] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
