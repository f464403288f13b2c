#!/usr/bin/env python3
"""Weight-register GEMM (mmq_wgemm.hip): parity against the oracle, then graph-timed A/B
against the LDS-DMA GEMM (mmq_gemm.hip) and per-(RG, NB, splits) timings.

  python tools/wgemm_check.py [--quick] [--only-time] [--configs a,b]

Prints one JSON object per line (kind = parity | time)."""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gguf-triton-kernel_amd"), os.path.join(ROOT, "oracle"), ROOT):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import kernels._lib as kl  # noqa: E402

TIGHT = 4e-3


def parity(dev, quick):
    import oracle as O
    from utils.synth import random_activations, random_blocks
    shapes = [(130, 33, 256), (200, 64, 512), (257, 100, 768), (300, 128, 1024), (64, 200, 512), (1000, 48, 2048),
              (520, 256, 1024)]
    cfgs = [dict(GQ_WGEMM=1), dict(GQ_WGEMM=1, GQ_WGEMM_RG=1)] + ([] if quick else [dict(GQ_WGEMM=1, GQ_WGEMM_NB=2),
                                                   dict(GQ_WGEMM=1, GQ_WGEMM_NB=4, GQ_WGEMM_SPLITS=3),
                                                   dict(GQ_WGEMM=1, GQ_WGEMM_SPLITS=1),
                                                   dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=8, GQ_WGEMM_SPLITS=2)])
    ok = True
    for fmt in ("q8_0", "q4_k", "q6_k"):
        for (M, N, K) in shapes:
            qA = random_blocks(fmt, M, K, seed=M + N)
            B = random_activations(N, K, seed=K + N)
            ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
            A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
            B_t = torch.from_numpy(B).to(dev)
            for cfg in cfgs:
                with kl.tuning(**cfg):
                    C = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
                    torch.cuda.synchronize()
                got = C.cpu().numpy()
                err = float(O.max_rel_err(got, ideal))
                good = bool(np.isfinite(got.astype(np.float32)).all() and err <= TIGHT)
                ok &= good
                print(json.dumps({"kind": "parity", "fmt": fmt, "M": M, "N": N, "K": K, "cfg": cfg, "err": err,
                                  "ok": good}), flush=True)
    return ok


BLOCK = {"q8_0": (32, 34), "q4_k": (256, 144), "q6_k": (256, 210)}


def rand_blocks(fmt, M, K, dev, seed):
    qk, nbytes = BLOCK[fmt]
    nb = M * (K // qk)
    g = torch.Generator(device=dev).manual_seed(seed)
    raw = torch.randint(0, 256, (nb, nbytes), dtype=torch.uint8, device=dev, generator=g)
    sc = ((torch.rand(nb, device=dev, generator=g) + 0.5) * 2.0 ** -7).to(torch.float16).view(torch.uint8)
    if fmt == "q8_0":
        raw[:, 0:2] = sc.view(nb, 2)
    elif fmt == "q4_k":
        raw[:, 0:2] = sc.view(nb, 2)
        raw[:, 2:4] = sc.view(nb, 2)
    else:
        raw[:, 208:210] = sc.view(nb, 2)
    return raw.view(-1).view(torch.int8)


def time_cfg(fmt, M, K, N, dev, cfg, steps=40, prepared=True):
    """us per MMQ call (activations prepared once; graph of `steps` calls over >= 1 GiB of
    weight copies), best of 3 replays."""
    wb = M * (K // BLOCK[fmt][0]) * BLOCK[fmt][1]
    ncopies = max(2, math.ceil((1 << 30) / wb))
    base = rand_blocks(fmt, M, K, dev, 1)
    Ws = [base] + [base.clone() for _ in range(ncopies - 1)]
    B = torch.randn(N, K, device=dev).to(torch.float16)
    C = torch.empty(N, M, dtype=torch.float16, device=dev)
    t = kl.TYPES[fmt]
    with kl.tuning(**cfg):
        need = kl.workspace_size(t, M, N, K)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        L = kl.lib()

        def call(i):
            stream = torch.cuda.current_stream().cuda_stream
            if prepared:
                rc = L.gq_mmq_prepared(t, Ws[i % ncopies].data_ptr(), ws.data_ptr(), need, C.data_ptr(), M, N, K, M, stream)
            else:
                rc = L.gq_mmq(t, Ws[i % ncopies].data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, M, ws.data_ptr(), need,
                              stream)
            assert rc == 0, L.gq_last_error()

        kl.act_prepare(B, N, K, ws)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            call(0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(steps):
                call(i)
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / steps)
    del Ws, g
    torch.cuda.empty_cache()
    return best


CONFIGS = {
    "q8_0_4096x4096_m128": ("q8_0", 4096, 4096, 128),
    "q4_k_4096x4096_m128": ("q4_k", 4096, 4096, 128),
    "q4_k_11008x4096_m128": ("q4_k", 11008, 4096, 128),
    "q4_k_4096x11008_m128": ("q4_k", 4096, 11008, 128),
    "q6_k_28672x8192_m128": ("q6_k", 28672, 8192, 128),
    "q6_k_8192x28672_m128": ("q6_k", 8192, 28672, 128),
    "q4_k_4096x4096_m64": ("q4_k", 4096, 4096, 64),
    "q4_k_4096x4096_m256": ("q4_k", 4096, 4096, 256),
    "q4_k_4096x4096_m40": ("q4_k", 4096, 4096, 40),
    "q8_0_4096x4096_m64": ("q8_0", 4096, 4096, 64),
    "q8_0_4096x4096_m256": ("q8_0", 4096, 4096, 256),
    "q8_0_4096x4096_m512": ("q8_0", 4096, 4096, 512),
    "q4_k_11008x4096_m512": ("q4_k", 11008, 4096, 512),
}


VARIANTS = {
    "old": dict(GQ_WGEMM=0),
    "w_rg2_nb8": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=8),
    "w_rg2_nb4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=4),
    "w_rg1_nb8": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=8),
    "w_rg1_nb4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=4),
    "w_rg2_nb8_s1": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=8, GQ_WGEMM_SPLITS=1),
    "w_rg2_nb4_s4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=4, GQ_WGEMM_SPLITS=4),
    "w_rg2_nb4_s8": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=4, GQ_WGEMM_SPLITS=8),
    "w_rg1_nb8_s4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=8, GQ_WGEMM_SPLITS=4),
    "w_rg1_nb8_wd3": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=8, GQ_WGEMM_WD=3),
    "w_rg1_nb8_wd4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=8, GQ_WGEMM_WD=4),
    "w_rg2_nb8_wd3": dict(GQ_WGEMM=1, GQ_WGEMM_RG=2, GQ_WGEMM_NB=8, GQ_WGEMM_WD=3),
    "w_rg1_nb4_wd4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=4, GQ_WGEMM_WD=4),
    "w_rg1_nb2_wd4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_NB=2, GQ_WGEMM_WD=4),
    "w_rg1_wd4": dict(GQ_WGEMM=1, GQ_WGEMM_RG=1, GQ_WGEMM_WD=4),
}


def timing(dev, names, quick, vnames=None):
    vnames = vnames or ["old", "w_rg2_nb8", "w_rg2_nb4", "w_rg1_nb8"]
    if quick:
        vnames = vnames[:2]
    variants = [(v, VARIANTS[v]) for v in vnames]
    for name in names:
        fmt, M, K, N = CONFIGS[name]
        flops = 2.0 * M * N * K
        row = {"kind": "time", "config": name, "lib": os.path.basename(kl.LIB_PATH)}
        for vname, cfg in variants:
            us = time_cfg(fmt, M, K, N, dev, cfg)
            row[vname] = round(us, 2)
            row[vname + "_tf"] = round(flops / us / 1e6, 1)
        print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only-time", action="store_true")
    ap.add_argument("--no-time", action="store_true")
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--lib", default=None, help="another build of libgguf_mmq.so (diagnostic variants)")
    ap.add_argument("--variants", default=None, help="comma list of timing variants (names in VARIANTS)")
    a = ap.parse_args()
    if a.lib:
        kl.LIB_PATH = a.lib
    dev = torch.device("cuda:0")
    t0 = time.time()
    ok = True
    if not a.only_time:
        ok = parity(dev, a.quick)
        print(json.dumps({"kind": "parity_summary", "ok": ok, "s": round(time.time() - t0, 1)}), flush=True)
        if not ok:
            sys.exit(1)
    if not a.no_time:
        timing(dev, a.configs.split(","), a.quick, a.variants.split(",") if a.variants else None)


if __name__ == "__main__":
    main()
