#!/usr/bin/env python3
"""bench.py -- GGUF MMQ throughput on MI355X (BASELINE.json metric:
"effective fp16 TFLOPS + quant-weight GB/s per GGUF type, M=1 and M=128").

Default workload = BASELINE.json configs[1]: Q8_0 weights N_out=4096 x K=4096, M_tok=128
fp16 activations on one MI355X.  One "step" = one drop-in call: q8_1 quantization of the
activations + the MMQ over one weight matrix (gq_mmq).  Inputs are resident in HBM before
timing; the steps cycle through >= 1 GiB of distinct weight copies so the 256 MB
Infinity Cache cannot serve them.  K steps are captured into one hipGraph and replayed;
time = HIP events around the replay, bracketed by barrier + synchronize.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--sweep] [--no-cpu]

N > 1 (torch.distributed.run, one rank per GPU, RCCL): weak scaling of the row-sharded
layer -- every rank owns an N_out-row shard of an (N * N_out)-row weight matrix, runs the
step on it and all-gathers the fp16 output shards over xGMI (RCCL all_gather, overlapped
with the next step's compute).  value = all ranks' FLOPs / max-over-ranks time.

Extra JSON fields: roofline (dominant kernel = the MMQ launch, timed alone with HIP events
in its own graph), cpu_baseline (oracle/ C restatement of kernels/cpu_impls, one thread,
bounded row sample, rank 0 at N=1 only), sweep (other BASELINE configs with --sweep).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gguf-triton-kernel_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TF = 2500.0  # dense fp16/bf16 MFMA spec
ROTATE_BYTES = 1 << 30     # >= 4x the 256 MiB Infinity Cache

# name -> (fmt, N_out (weight rows), K, M_tok)
CONFIGS = {
    "q8_0_4096x4096_m128": ("q8_0", 4096, 4096, 128),   # BASELINE configs[1] -- the headline
    "q8_0_4096x4096_m1": ("q8_0", 4096, 4096, 1),
    "q4_k_4096x4096_m1": ("q4_k", 4096, 4096, 1),
    "q4_k_4096x4096_m16": ("q4_k", 4096, 4096, 16),
    "q4_k_4096x4096_m128": ("q4_k", 4096, 4096, 128),
    "q4_k_11008x4096_m1": ("q4_k", 11008, 4096, 1),
    "q4_k_11008x4096_m16": ("q4_k", 11008, 4096, 16),
    "q4_k_11008x4096_m128": ("q4_k", 11008, 4096, 128),
    "q6_k_28672x8192_m1": ("q6_k", 28672, 8192, 1),
    "q6_k_28672x8192_m128": ("q6_k", 28672, 8192, 128),
}
DEFAULT = "q8_0_4096x4096_m128"
BLOCK = {"q8_0": (32, 34), "q4_k": (256, 144), "q6_k": (256, 210)}
GTYPE = {"q8_0": 0, "q4_k": 1, "q6_k": 2}


def device_random_blocks(fmt: str, M: int, K: int, dev, seed: int) -> torch.Tensor:
    """Random packed blocks made on the device; fp16 scale fields = U(0.5,1.5)*2^-7."""
    qk, nbytes = BLOCK[fmt]
    nb = M * (K // qk)
    g = torch.Generator(device=dev).manual_seed(seed)
    raw = torch.randint(0, 256, (nb, nbytes), dtype=torch.uint8, device=dev, generator=g)

    def scales():
        return ((torch.rand(nb, device=dev, generator=g) + 0.5) * 2.0 ** -7).to(torch.float16).view(torch.uint8)

    if fmt == "q8_0":
        raw[:, 0:2] = scales().view(nb, 2)
    elif fmt == "q4_k":
        raw[:, 0:2] = scales().view(nb, 2)
        raw[:, 2:4] = scales().view(nb, 2)
    else:
        raw[:, 208:210] = scales().view(nb, 2)
    return raw.view(-1).view(torch.int8)


def model(fmt, M, K, N):
    qk, nbytes = BLOCK[fmt]
    wbytes = M * (K // qk) * nbytes
    alg_bytes = wbytes + 2 * N * K + 2 * N * M
    flops = 2.0 * N * M * K
    return wbytes, alg_bytes, flops


class Runner:
    """Holds resident buffers for one config and the captured graphs."""

    def __init__(self, fmt, M, K, N, dev, steps, seed=0):
        import kernels._lib as kl
        self.kl, self.L = kl, kl.lib()
        self.fmt, self.M, self.K, self.N, self.dev = fmt, M, K, N, dev
        self.gtype = GTYPE[fmt]
        wbytes, _, _ = model(fmt, M, K, N)
        self.ncopies = max(2, math.ceil(ROTATE_BYTES / wbytes))
        base = device_random_blocks(fmt, M, K, dev, seed)
        self.weights = [base] + [base.clone() for _ in range(self.ncopies - 1)]
        g = torch.Generator(device=dev).manual_seed(seed + 1)
        self.B = torch.randn(N, K, device=dev, generator=g).to(torch.float16)
        self.C = [torch.empty(N, M, dtype=torch.float16, device=dev) for _ in range(2)]
        self.ws_bytes = kl.workspace_size(self.gtype, M, N, K)
        self.ws = torch.empty(max(self.ws_bytes, 1), dtype=torch.uint8, device=dev)
        self.stream_ptr = None

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def step(self, i, c=None):
        A = self.weights[i % self.ncopies]
        C = self.C[i & 1] if c is None else c
        rc = self.L.gq_mmq(self.gtype, A.data_ptr(), self.B.data_ptr(), C.data_ptr(), self.M, self.N, self.K,
                           self.K, self.M, self.ws.data_ptr(), self.ws_bytes, self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def prepare(self):
        rc = self.L.gq_act_prepare(self.B.data_ptr(), self.N, self.K, self.K, self.ws.data_ptr(), self.ws_bytes,
                                   self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def kernel(self, i):
        A = self.weights[i % self.ncopies]
        rc = self.L.gq_mmq_prepared(self.gtype, A.data_ptr(), self.ws.data_ptr(), self.ws_bytes,
                                    self.C[i & 1].data_ptr(), self.M, self.N, self.K, self.M, self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def capture(self, fn, n):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            fn(0)  # warm the launch path outside capture
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with torch.cuda.graph(g):
            for i in range(n):
                fn(i)
        return g


def timed_replay(graph, dev, dist_on=False) -> float:
    """Seconds for one replay, max over ranks."""
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) / 1e3
    if dist_on:
        torch.distributed.barrier()
        tt = torch.tensor([t], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        t = float(tt.item())
    return t


def roofline(fmt, M, K, N, t_kernel, traffic=None):
    _, alg_bytes, flops = model(fmt, M, K, N)
    t_hbm = alg_bytes / (HBM_PEAK_GBS * 1e9)
    t_mfma = flops / (MFMA_F16_PEAK_TF * 1e12)
    if t_hbm >= t_mfma:
        ach = alg_bytes / t_kernel / 1e9
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes, "kernel_us": round(t_kernel * 1e6, 3)}
    ach = flops / t_kernel / 1e12
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_F16_PEAK_TF, "unit": "TFLOP/s",
            "frac": round(ach / MFMA_F16_PEAK_TF, 4), "traffic": traffic,
            "alg_flops_per_launch": flops, "kernel_us": round(t_kernel * 1e6, 3)}


def load_traffic(name):
    """HBM bytes per launch from a committed PMC pass (profiles/pmc_<config>.json), or None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def cpu_baseline(fmt, M, K, N, target_s=12.0):
    """oracle/ C restatement of kernels/cpu_impls (the reference's arithmetic), one thread,
    on the first R weight rows x all N tokens; R sized for ~target_s of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from utils.synth import random_activations, random_blocks
    qk, nbytes = BLOCK[fmt]
    B = random_activations(N, K, seed=1)
    Bq = O.quantize_q8_1(B)
    rows = 1
    while True:
        A = random_blocks(fmt, rows, K, seed=2)
        t0 = time.perf_counter()
        O.mmq(fmt, A, Bq, rows, N, K, O.EXACT)
        dt = time.perf_counter() - t0
        if dt > 0.5 or rows >= M:
            break
        rows = min(M, rows * 4)
    if dt < target_s and rows < M:
        rows = min(M, max(rows, int(rows * target_s / max(dt, 1e-6))))
        A = random_blocks(fmt, rows, K, seed=2)
        t0 = time.perf_counter()
        O.mmq(fmt, A, Bq, rows, N, K, O.EXACT)
        dt = time.perf_counter() - t0
    tflops = 2.0 * rows * N * K / dt / 1e12
    return {"value": tflops, "unit": "TFLOP/s", "cores": 1, "kind": "port",
            "sample": f"{fmt} rows 0..{rows - 1} of N_out={M} x all {N} tokens, K={K}: oracle/mmq_oracle.c "
                      f"mode EXACT (kernels/cpu_impls arithmetic, fp16 running sum), 1 thread, {dt:.2f} s; "
                      f"extrapolated full step {dt * M / rows:.1f} s",
            "seconds": round(dt, 3), "rows": rows}


def bench_config(name, steps, warmup, dev, dist_on, world, rank):
    fmt, M, K, N = CONFIGS[name]
    r = Runner(fmt, M, K, N, dev, steps, seed=rank)
    # full step graph (act quant + mmq); warmup graph separately sized
    gw = r.capture(r.step, max(1, warmup))
    gw.replay()
    torch.cuda.synchronize(dev)
    if dist_on and world > 1:
        t, t_compute = bench_dist(r, steps, dev, world)
    else:
        g = r.capture(r.step, steps)
        g.replay()  # first replay pays lazy init
        t = min(timed_replay(g, dev, dist_on) for _ in range(3))
        t_compute = t
    # dominant kernel: decode (N <= 4) -- the step IS one launch (fused quantizer + weight
    # stream), so its time is the step's; GEMM -- the MMQ call alone (gemm_kernel [+ split-K
    # reduce]) with the activations prepared once, K launches in a graph
    if N <= 4:
        t_k = (t_compute if dist_on and world > 1 else t) / steps
        kname = "stream_decode_kernel (fused q8_1 + decode)"
    else:
        r.prepare()
        gk = r.capture(r.kernel, steps)
        gk.replay()
        t_k = min(timed_replay(gk, dev, dist_on) for _ in range(3)) / steps
        kname = "gemm_kernel (+ gemm_reduce_kernel when split-K)"
    wbytes, alg_bytes, flops = model(fmt, M, K, N)
    per_step = t / steps
    out = {
        "config": name, "fmt": fmt, "N_out": M, "K": K, "M_tok": N,
        "ms_per_step": per_step * 1e3,
        "tflops": world * flops / per_step / 1e12,
        "weight_GBps": world * wbytes / per_step / 1e9,
        "compute_only_tflops": world * flops / (t_compute / steps) / 1e12,
        "roofline": dict(roofline(fmt, M, K, N, t_k, load_traffic(name)), kernel=kname),
        "weight_copies": r.ncopies,
    }
    del r
    torch.cuda.empty_cache()
    return out


def bench_layer(N, steps, warmup, dev):
    """BASELINE configs[4]: the seven projections of a Llama-7B block under GGUF Q4_K_M (layer 0:
    attn_v and ffn_down in Q6_K, the rest Q4_K), shared inputs quantized once per group
    (kernels.layer_mix.LayerMix).  Weights rotate over >= 1 GiB of copies."""
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    types = q4_k_m_layer_types(0, 32)
    one = {n: device_random_blocks(types[n], M, K, dev, seed=i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    layer_bytes = sum(t.numel() for t in one.values())
    ncopies = max(2, math.ceil(ROTATE_BYTES / layer_bytes))
    layers = [LayerMix({n: GGUFLinear(types[n], one[n] if c == 0 else one[n].clone(), *LLAMA_LAYER_SHAPES[n])
                        for n in LLAMA_LAYER_SHAPES}) for c in range(ncopies)]
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(N, 4096, device=dev, generator=g).to(torch.float16)
    h = torch.randn(N, 11008, device=dev, generator=g).to(torch.float16)
    outs = {n: torch.empty(N, M, dtype=torch.float16, device=dev) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    flops = sum(2.0 * N * M * K for M, K in LLAMA_LAYER_SHAPES.values())
    for i in range(max(1, warmup)):  # also creates any library handles outside capture
        layers[i % ncopies].forward(x, h, outs)
    torch.cuda.synchronize(dev)
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        layers[0].forward(x, h, outs)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    with torch.cuda.graph(gr):
        for i in range(steps):
            layers[i % ncopies].forward(x, h, outs)
    gr.replay()
    t = min(timed_replay(gr, dev) for _ in range(3)) / steps
    return {"config": f"q4_k_m_llama7b_layer_m{N}", "fmt": "q4_k+q6_k", "M_tok": N, "ms_per_step": t * 1e3,
            "tflops": flops / t / 1e12, "weight_GBps": layer_bytes / t / 1e9, "weight_bytes": layer_bytes,
            "types": types, "weight_copies": ncopies}


def bench_msweep(steps, warmup, dev, fmt="q4_k", M=4096, K=4096):
    """configs[4]'s M sweep: tokens 1..512 on one Q4_K 4096x4096 matrix (the step: gq_mmq)."""
    res = []
    for N in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
        r = Runner(fmt, M, K, N, dev, steps)
        gw = r.capture(r.step, max(1, warmup))
        gw.replay()
        gs = r.capture(r.step, steps)
        gs.replay()
        t = min(timed_replay(gs, dev) for _ in range(3)) / steps
        wbytes, alg_bytes, flops = model(fmt, M, K, N)
        res.append({"M_tok": N, "us_per_step": round(t * 1e6, 2), "tflops": round(flops / t / 1e12, 3),
                    "weight_GBps": round(wbytes / t / 1e9, 1), "alg_GBps": round(alg_bytes / t / 1e9, 1)})
        del r, gw, gs
        torch.cuda.empty_cache()
    return {"config": f"{fmt}_{M}x{K}_msweep", "points": res}


def bench_dist(r, steps, dev, world):
    """Each step: MMQ on the local row shard, then all_gather of the (N, N_out) fp16 shards
    into (world, N, N_out) on a side stream (RCCL), overlapped with the next step."""
    import torch.distributed as dist
    gathered = [torch.empty(world, r.N, r.M, dtype=torch.float16, device=dev) for _ in range(2)]
    gstep = [r.capture(lambda i, j=j: r.step(j), 1) for j in range(2)]

    def run(n):
        works = []
        for i in range(n):
            gstep[i & 1].replay()
            works.append(dist.all_gather_into_tensor(gathered[i & 1].view(world * r.N, r.M), r.C[i & 1],
                                                     async_op=True))
            if len(works) > 1:
                works.pop(0).wait()
        for w in works:
            w.wait()

    run(4)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize(dev)
    t = time.perf_counter() - t0
    # compute only
    g = r.capture(r.step, steps)
    g.replay()
    tc = timed_replay(g, dev, True)
    tt = torch.tensor([t], device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dist.barrier()
    return float(tt.item()), tc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=DEFAULT, choices=sorted(CONFIGS))
    ap.add_argument("--sweep", action="store_true", help="also measure the other BASELINE configs")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1
    if dist_on:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    head = bench_config(args.config, args.steps, args.warmup, dev, dist_on, world, rank)
    sweep = []
    if args.sweep:
        for name in CONFIGS:
            if name != args.config:
                sweep.append(bench_config(name, max(20, args.steps // 4), args.warmup, dev, dist_on, world, rank))
        if not dist_on:
            for n in (1, 128):
                sweep.append(bench_layer(n, max(20, args.steps // 4), args.warmup, dev))
            sweep.append(bench_msweep(max(20, args.steps // 4), args.warmup, dev))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        fmt, M, K, N = CONFIGS[args.config]
        cpu = cpu_baseline(fmt, M, K, N)

    if rank == 0:
        fmt, M, K, N = CONFIGS[args.config]
        line = {
            "metric": "effective fp16 TFLOPS (+ quant-weight GB/s) per GGUF type",
            "value": round(head["tflops"], 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["ms_per_step"], 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16" if N > 4 else "i8",
            "arith": "q8_1 activations x dequantized GGUF weights on fp16 MFMA, fp32 accumulate" if N > 4 else
                     "q8_1 int8 activations x GGUF int codes on v_dot4_i32_i8, fp32 block scaling",
            "data": "synthetic (random packed blocks, N(0,1) fp16 activations)",
            "config": {"workload": args.config, "gguf_type": fmt, "N_out": M, "K": K, "M_tok": N,
                       "global_N_out": M * world, "parallelism": f"rowshard{world}" if world > 1 else "single",
                       "weight_copies_rotated": head["weight_copies"]},
            "weight_GBps": round(head["weight_GBps"], 1),
            "compute_only_tflops": round(head["compute_only_tflops"], 3),
            "roofline": head["roofline"],
            "cpu_baseline": cpu,
        }
        if sweep:
            line["sweep"] = [{k: (round(v, 4) if isinstance(v, float) else v) for k, v in s.items()} for s in sweep]
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
