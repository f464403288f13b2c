#!/usr/bin/env python3
"""bench.py -- GGUF MMQ throughput on MI355X (BASELINE.json metric:
"effective fp16 TFLOPS + quant-weight GB/s per GGUF type, M=1 and M=128").

Default workload = BASELINE.json configs[1]: Q8_0 weights N_out=4096 x K=4096, M_tok=128
fp16 activations on one MI355X.  One "step" = one drop-in call: q8_1 quantization of the
activations + the MMQ over one weight matrix (gq_mmq).  Inputs are resident in HBM before
timing; the steps cycle through >= 1 GiB of distinct weight copies so the 256 MB
Infinity Cache cannot serve them.  K steps are captured into one hipGraph and replayed;
time = HIP events around the replay, bracketed by barrier + synchronize.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--strong] [--quick] [--no-cpu]

N > 1 (torch.distributed.run, one rank per GPU, RCCL): the row-sharded matmul of
dist/row_shard.py (RowShardedMMQ: local MMQ on the rank's rows, RCCL all_gather of the fp16
output slabs over xGMI, overlapped with the next step's compute, assembled to (N, M)).
  default   weak scaling: every rank owns an N_out-row shard of an (N * N_out)-row matrix;
            value = all ranks' FLOPs / max-over-ranks time.  The line also carries
            "strong": the Q6_K Llama-70B matrices (BASELINE configs[3]) at fixed global size,
            split over the N ranks, compute-only and end-to-end.
  --strong  the headline itself is the strong-scaling Q6_K 28672x8192 (M_tok 128) run.

Extra JSON fields: roofline (dominant kernel = the MMQ launch, timed alone with HIP events
in its own graph), cpu_baseline (oracle/ C restatement of kernels/cpu_impls, rank 0 at N=1
only: all host cores (row slices), plus the 1-thread literal port and the product's own
vectorised CPU MMQ in cpu_baseline_variants), sweep (every GGUF type at M=1 and M=128 on the
BASELINE shapes incl. the down projections, the Q4_K_M layer and the token sweep; --quick
skips it).
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
    "q4_k_4096x11008_m1": ("q4_k", 4096, 11008, 1),     # Llama-7B ffn_down
    "q4_k_4096x11008_m128": ("q4_k", 4096, 11008, 128),
    "q6_k_28672x8192_m1": ("q6_k", 28672, 8192, 1),     # Llama-70B ffn_gate/up
    "q6_k_28672x8192_m128": ("q6_k", 28672, 8192, 128),
    "q6_k_8192x28672_m1": ("q6_k", 8192, 28672, 1),     # Llama-70B ffn_down
    "q6_k_8192x28672_m128": ("q6_k", 8192, 28672, 128),
}
STRONG = ("q6_k_28672x8192_m1", "q6_k_28672x8192_m128")  # BASELINE configs[3]: row-sharded over the ranks
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

    def __init__(self, fmt, M, K, N, dev, steps, seed=0, act="q8_1"):
        import kernels._lib as kl
        self.kl, self.L = kl, kl.lib()
        self.fmt, self.M, self.K, self.N, self.dev = fmt, M, K, N, dev
        self.act = kl.ACTS[act]
        self.gtype = GTYPE[fmt]
        wbytes, _, _ = model(fmt, M, K, N)
        self.ncopies = max(2, math.ceil(ROTATE_BYTES / wbytes))
        base = device_random_blocks(fmt, M, K, dev, seed)
        self.weights = [base] + [base.clone() for _ in range(self.ncopies - 1)]
        g = torch.Generator(device=dev).manual_seed(seed + 1)
        self.B = torch.randn(N, K, device=dev, generator=g).to(torch.float16)
        self.C = [torch.empty(N, M, dtype=torch.float16, device=dev) for _ in range(2)]
        self.ws_bytes = kl.workspace_size(self.gtype, M, N, K, act)
        self.ws = torch.empty(max(self.ws_bytes, 1), dtype=torch.uint8, device=dev)
        self.stream_ptr = None

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def step(self, i, c=None):
        A = self.weights[i % self.ncopies]
        C = self.C[i & 1] if c is None else c
        rc = self.L.gq_mmq_ex(self.gtype, self.act, A.data_ptr(), self.B.data_ptr(), C.data_ptr(), self.M, self.N,
                              self.K, self.K, self.M, self.ws.data_ptr(), self.ws_bytes, self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def prepare(self):
        rc = self.L.gq_act_prepare_ex(self.act, self.B.data_ptr(), self.N, self.K, self.K, self.ws.data_ptr(),
                                      self.ws_bytes, self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def kernel(self, i):
        A = self.weights[i % self.ncopies]
        rc = self.L.gq_mmq_prepared_ex(self.gtype, self.act, A.data_ptr(), self.ws.data_ptr(), self.ws_bytes,
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


def host_cores() -> int:
    """Host threads for the CPU baseline: the process's affinity set, capped at 16 (the GPU
    box gives one GPU's job a 16-core share; OMP_NUM_THREADS says the same there)."""
    n = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(n, cap, 16))


# The reference's own CPU path (kernels/cpu_impls, Python loops) measured in the survey
# container: ms per (weight row x token) at K = 4096.
REF_CPU_MS_PER_ROW_TOKEN = {"q8_0": 4.29, "q4_k": 7.63, "q6_k": 18.52}


def _timed_rows(run, M, target_s):
    """Grow a row count until run(rows) takes ~target_s (or all M rows); -> (rows, seconds)."""
    rows = 1
    while True:
        t0 = time.perf_counter()
        run(rows)
        dt = time.perf_counter() - t0
        if dt > 0.25 * target_s or rows >= M:
            break
        rows = min(M, rows * 4)
    if dt < target_s and rows < M:
        rows = min(M, max(rows, int(rows * target_s / max(dt, 1e-6))))
        t0 = time.perf_counter()
        run(rows)
        dt = time.perf_counter() - t0
    return rows, dt


def cpu_baseline(fmt, M, K, N, target_s=6.0):
    """The reference's CPU arithmetic on the host cores, on a bounded row sample of the
    workload (all N tokens, the first R weight rows; R sized for ~target_s per leg):
      main     oracle/mmq_oracle.c EXACT (restatement of kernels/cpu_impls), row slices
               over host_cores() threads (ctypes drops the GIL; outputs independent);
      variants the same oracle on 1 thread (the reference's literal loop order), and the
               product's vectorised C++ CPU MMQ (kernels.cpu_impls drop-in, libgguf_quant)
               on all cores -- bit-identical outputs, different speed."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from kernels.cpu_impls._cpu import cpu_mmq
    from utils.synth import random_activations, random_blocks
    cores = host_cores()
    B = random_activations(N, K, seed=1)
    Bq = O.quantize_q8_1(B)
    qk, nbytes = BLOCK[fmt]
    row_bytes = (K // qk) * nbytes
    A_all = random_blocks(fmt, min(M, 4096), K, seed=2)

    def rows_of(r):
        reps = -(-r // (A_all.size // row_bytes))
        return np.tile(A_all, reps)[:r * row_bytes] if reps > 1 else A_all[:r * row_bytes]

    def oracle_mt(r):
        A = rows_of(r)
        per = -(-r // cores)
        chunks = [(i, min(r, i + per)) for i in range(0, r, per)]
        with ThreadPoolExecutor(cores) as ex:
            list(ex.map(lambda c: O.mmq(fmt, A[c[0] * row_bytes:c[1] * row_bytes], Bq, c[1] - c[0], N, K, O.EXACT),
                        chunks))

    def oracle_1(r):
        O.mmq(fmt, rows_of(r), Bq, r, N, K, O.EXACT)

    Bt = torch.from_numpy(Bq.view(np.int8))

    def product_mt(r):
        cpu_mmq(GTYPE[fmt], torch.from_numpy(rows_of(r).view(np.int8)), Bt, r, N, K, threads=cores)

    def leg(run, kind, threads, what):
        r, dt = _timed_rows(run, M, target_s)
        return {"value": 2.0 * r * N * K / dt / 1e12, "unit": "TFLOP/s", "cores": threads, "kind": kind,
                "sample": f"{fmt} rows 0..{r - 1} of N_out={M} x all {N} tokens, K={K}: {what}, {threads} "
                          f"thread(s), {dt:.2f} s; extrapolated full step {dt * M / r:.2f} s",
                "seconds": round(dt, 3), "rows": r, "ms_per_row_token": round(dt * 1e3 / (r * N), 5)}

    main = leg(oracle_mt, "port", cores, "oracle/mmq_oracle.c mode EXACT (kernels/cpu_impls arithmetic, "
                                         "fp16 running sum), row slices over threads")
    one = leg(oracle_1, "port", 1, "oracle/mmq_oracle.c mode EXACT, the reference's loop order")
    vec = leg(product_mt, "port", cores, "kernels.cpu_impls drop-in (csrc/quant/gguf_cpu_mmq.cpp: rows unpacked "
                                         "once, vectorised int8 dots, same outputs bit for bit)")
    ref = REF_CPU_MS_PER_ROW_TOKEN[fmt] * K / 4096.0
    main["reference_python_ms_per_row_token"] = round(ref, 3)
    main["reference_python_source"] = ("kernels/cpu_impls Python loops measured in the survey container "
                                       "(SURVEY.md 6), scaled to this K; 1 thread")
    main["speedup_1thread_port_vs_reference_python"] = round(ref / one["ms_per_row_token"], 1)
    return main, [one, vec]


class ShardedRunner:
    """One rank's part of a row-sharded step: RowShardedMMQ over rotating copies of this rank's
    packed rows (>= 1 GiB), the local MMQ through the C ABI into a padded slab (graph-capturable:
    preallocated workspace, torch's current stream), then the RCCL all_gather + assemble."""

    def __init__(self, fmt, M_global, K, N, dev, world, rank, seed=0):
        import kernels._lib as kl
        from dist.row_shard import RowShardedMMQ, shard_rows
        self.L = kl.lib()
        self.fmt, self.K, self.N, self.dev, self.world = fmt, K, N, dev, world
        self.row0, self.rows, self.R = shard_rows(M_global, world, rank)
        qk, nbytes = BLOCK[fmt]
        wbytes = max(1, self.rows * (K // qk) * nbytes)
        self.ncopies = max(2, math.ceil(ROTATE_BYTES / wbytes))
        base = device_random_blocks(fmt, max(self.rows, 1), K, dev, seed + rank)[:self.rows * (K // qk) * nbytes]
        self.ws_bytes = max(1, kl.workspace_size(GTYPE[fmt], max(self.rows, 1), N, K))
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        self.parts = [RowShardedMMQ(fmt, base if c == 0 else base.clone(), M_global, K, align=64,
                                    compute=self._compute, world=world, rank=rank) for c in range(self.ncopies)]
        g = torch.Generator(device=dev).manual_seed(seed + 1)
        self.B = torch.randn(N, K, device=dev, generator=g).to(torch.float16)
        self.slab = [torch.zeros(N, self.R, dtype=torch.float16, device=dev) for _ in range(2)]
        self.gathered = [torch.empty(world, N, self.R, dtype=torch.float16, device=dev) for _ in range(2)]
        self.gtype = GTYPE[fmt]

    def _compute(self, A_shard, B, rows, N, K, out):
        rc = self.L.gq_mmq(self.gtype, A_shard.data_ptr(), B.data_ptr(), out.data_ptr(), rows, N, K, K,
                           out.stride(0), self.ws.data_ptr(), self.ws_bytes,
                           torch.cuda.current_stream(self.dev).cuda_stream)
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def local(self, i):
        self.parts[i % self.ncopies].local(self.B, self.N, self.slab[i & 1])

    def capture(self, n, first=0):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.local(first)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with torch.cuda.graph(g):
            for i in range(n):
                self.local(first + i)
        return g

    def capture_e2e(self, n):
        """One graph of n whole steps: local MMQ on the compute stream; the all_gather (RCCL,
        captured) and the assemble on a side stream, so step i's exchange overlaps step i+1's
        compute; slab j is rewritten only after the exchange that read it (events)."""
        part = self.parts[0]
        side = torch.cuda.Stream(self.dev)
        done = [torch.cuda.Event() for _ in range(2)]
        out = [None, None]

        def body(i):
            if i >= 2:
                torch.cuda.current_stream(self.dev).wait_event(done[i & 1])
            self.local(i)
            side.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(side):
                part.gather(self.slab[i & 1], self.gathered[i & 1])
                out[i & 1] = part.assemble(self.gathered[i & 1])
                done[i & 1].record(side)

        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):  # warm every op outside capture (RCCL communicator included)
            for i in range(2):
                body(i)
            s.wait_stream(side)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(n):
                body(i)
            torch.cuda.current_stream(self.dev).wait_stream(side)
        return g

    def end_to_end(self, steps):
        """(seconds for `steps` whole steps -- local MMQ + all_gather + assemble -- max over
        ranks, how it ran).  The steps are one captured graph (RCCL collectives captured);
        for a backend that cannot be captured (gloo rehearsals), an eager loop: per step a one-step graph replay and an async
        all_gather on RCCL's stream, one exchange in flight behind the next step's compute."""
        import torch.distributed as dist
        if dist.is_initialized() and dist.get_backend() == "nccl":  # RCCL collectives are capturable
            g = self.capture_e2e(steps)
            g.replay()
            t = min(timed_replay(g, self.dev, True) for _ in range(3))
            return t, "graph"
        # (a failed capture leaves the stream poisoned, so no try: other backends run eagerly)
        how = f"eager ({dist.get_backend() if dist.is_initialized() else 'no'} backend: not capturable)"
        one = [self.capture(1, j) for j in range(2)]
        part = self.parts[0]

        def run(n):
            works = []
            for i in range(n):
                one[i & 1].replay()
                _, w = part.gather(self.slab[i & 1], self.gathered[i & 1], async_op=True)
                works.append((w, i & 1))
                if len(works) > 1:
                    w0, j = works.pop(0)
                    if w0 is not None:
                        w0.wait()
                    part.assemble(self.gathered[j])
            for w0, j in works:
                if w0 is not None:
                    w0.wait()
                part.assemble(self.gathered[j])

        run(4)
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize(self.dev)
        t = time.perf_counter() - t0
        if dist.is_initialized():
            tt = torch.tensor([t], device=self.dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dist.barrier()
            t = float(tt.item())
        return t, how


def dist_backend():
    import torch.distributed as dist
    b = dist.get_backend() if dist.is_initialized() else "none"
    return "nccl = RCCL over xGMI" if b == "nccl" else b


def bench_sharded(name, steps, warmup, dev, dist_on, world, rank, M_global=None):
    """Row-sharded run of config `name` over the ranks: M_global rows in total (default: the
    config's N_out, i.e. strong scaling; weak scaling passes world * N_out)."""
    fmt, M, K, N = CONFIGS[name]
    Mg = M_global or M
    r = ShardedRunner(fmt, Mg, K, N, dev, world, rank, seed=0)
    gw = r.capture(max(1, warmup))
    gw.replay()
    g = r.capture(steps)
    g.replay()
    t_c = min(timed_replay(g, dev, dist_on) for _ in range(3))
    t_e, how = r.end_to_end(steps) if dist_on else (t_c, "graph (1 rank: no exchange)")
    _, _, flops = model(fmt, Mg, K, N)
    qk, nbytes = BLOCK[fmt]
    wbytes = Mg * (K // qk) * nbytes
    out = {"config": name, "fmt": fmt, "N_out_global": Mg, "K": K, "M_tok": N, "ranks": world,
           "rows_per_rank": r.R, "ms_per_step": t_e / steps * 1e3, "compute_ms_per_step": t_c / steps * 1e3,
           "tflops": flops / (t_e / steps) / 1e12, "compute_only_tflops": flops / (t_c / steps) / 1e12,
           "weight_GBps": wbytes / (t_e / steps) / 1e9, "weight_copies": r.ncopies,
           "collective": (f"all_gather_into_tensor (backend {dist_backend()}) + assemble" if dist_on
                          else "none (1 rank)"), "timed_as": how}
    del r, g, gw
    torch.cuda.empty_cache()
    return out


def bench_config(name, steps, warmup, dev):
    """One config on this GPU: the drop-in step (gq_mmq) timed over a graph of `steps` calls,
    and the dominant kernel for the roofline."""
    fmt, M, K, N = CONFIGS[name]
    r = Runner(fmt, M, K, N, dev, steps)
    gw = r.capture(r.step, max(1, warmup))
    gw.replay()
    torch.cuda.synchronize(dev)
    g = r.capture(r.step, steps)
    g.replay()  # first replay pays lazy init
    t = min(timed_replay(g, dev) for _ in range(3))
    # dominant kernel: decode (N <= 4) -- the step IS one launch (fused quantizer + weight
    # stream), so its time is the step's; GEMM -- the MMQ call alone (gemm_kernel [+ split-K
    # reduce]) with the activations prepared once, K launches in a graph
    if N <= 4:
        t_k = t / steps
        kname = "stream_decode_kernel (fused q8_1 + decode)"
    else:
        r.prepare()
        gk = r.capture(r.kernel, steps)
        gk.replay()
        t_k = min(timed_replay(gk, dev) for _ in range(3)) / steps
        kname = "gemm_kernel (+ gemm_reduce_kernel when split-K)"
    wbytes, alg_bytes, flops = model(fmt, M, K, N)
    per_step = t / steps
    out = {
        "config": name, "fmt": fmt, "N_out": M, "K": K, "M_tok": N,
        "ms_per_step": per_step * 1e3,
        "tflops": flops / per_step / 1e12,
        "weight_GBps": wbytes / per_step / 1e9,
        "roofline": dict(roofline(fmt, M, K, N, t_k, load_traffic(name)), kernel=kname),
        "weight_copies": r.ncopies,
    }
    del r
    torch.cuda.empty_cache()
    return out


def bench_layer(Ns, acts, steps, warmup, dev, fuse=True):
    """BASELINE configs[4]: the seven projections of a Llama-7B block under GGUF Q4_K_M (layer 0:
    attn_v and ffn_down in Q6_K, the rest Q4_K), shared inputs quantized once per group
    (kernels.layer_mix.LayerMix; fuse: q+k and gate+up as one call each), for each token count in
    Ns and activation format in acts ("q8_1": the reference's semantics; "fp8": the e4m3 variant).
    Weights rotate over >= 1 GiB."""
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    types = q4_k_m_layer_types(0, 32)
    one = {n: device_random_blocks(types[n], M, K, dev, seed=i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    layer_bytes = sum(t.numel() for t in one.values())
    ncopies = max(2, math.ceil(ROTATE_BYTES / layer_bytes))
    lins = [{n: GGUFLinear(types[n], one[n] if c == 0 else one[n].clone(), *LLAMA_LAYER_SHAPES[n])
             for n in LLAMA_LAYER_SHAPES} for c in range(ncopies)]
    res = []
    for act in acts:
        layers = [LayerMix(lin, act=act, fuse=fuse) for lin in lins]
        for N in Ns:
            g = torch.Generator(device=dev).manual_seed(7)
            x = torch.randn(N, 4096, device=dev, generator=g).to(torch.float16)
            h = torch.randn(N, 11008, device=dev, generator=g).to(torch.float16)
            outs = {n: torch.empty(N, M, dtype=torch.float16, device=dev) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
            flops = sum(2.0 * N * M * K for M, K in LLAMA_LAYER_SHAPES.values())
            for i in range(max(ncopies, warmup)):  # library handles, every copy's buffers: outside capture
                layers[i % ncopies].forward(x, h, out=outs)
            torch.cuda.synchronize(dev)
            gr = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                layers[0].forward(x, h, out=outs)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            with torch.cuda.graph(gr):
                for i in range(steps):
                    layers[i % ncopies].forward(x, h, out=outs)
            gr.replay()
            t = min(timed_replay(gr, dev) for _ in range(3)) / steps
            res.append({"config": f"q4_k_m_llama7b_layer_m{N}", "act": act, "fused": fuse, "fmt": "q4_k+q6_k", "M_tok": N,
                        "us_per_step": round(t * 1e6, 2), "tflops": round(flops / t / 1e12, 3),
                        "weight_GBps": round(layer_bytes / t / 1e9, 1)})
            del gr
    del lins, layers
    torch.cuda.empty_cache()
    return {"config": "q4_k_m_llama7b_layer_msweep", "types": types, "weight_bytes": layer_bytes,
            "weight_copies": ncopies, "points": res}


def bench_fp8(names, steps, warmup, dev):
    """The fp8 activation variant on BASELINE shapes: the step (gq_mmq_ex, GQ_ACT_FP8_E4M3)."""
    out = []
    for name in names:
        fmt, M, K, N = CONFIGS[name]
        r = Runner(fmt, M, K, N, dev, steps, act="fp8")
        gw = r.capture(r.step, max(1, warmup))
        gw.replay()
        g = r.capture(r.step, steps)
        g.replay()
        t = min(timed_replay(g, dev) for _ in range(3)) / steps
        wbytes, _, flops = model(fmt, M, K, N)
        out.append({"config": name + "_fp8act", "act": "fp8", "us_per_step": round(t * 1e6, 2),
                    "tflops": round(flops / t / 1e12, 3), "weight_GBps": round(wbytes / t / 1e9, 1)})
        del r, g, gw
        torch.cuda.empty_cache()
    return out


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


def compact(e):
    """A sweep entry with the roofline reduced to its fraction and kernel time."""
    o = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in e.items() if k != "roofline"}
    if e.get("roofline"):
        rf = e["roofline"]
        o["roofline"] = {"bound": rf["bound"], "frac": rf["frac"], "achieved": rf["achieved"], "unit": rf["unit"],
                         "kernel_us": rf["kernel_us"]}
    return o


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=DEFAULT, choices=sorted(CONFIGS))
    ap.add_argument("--strong", action="store_true", help="headline = strong scaling of Q6_K 28672x8192 x128")
    ap.add_argument("--quick", action="store_true", help="headline only: no per-type sweep")
    ap.add_argument("--sweep", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--layer-only", action="store_true",
                    help="print only the Q4_K_M layer sweep (fused and unfused), one JSON line")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_FORCE_DIST=1: the distributed code path even at world 1 (exercises RCCL graph
    # capture on a 1-GPU box)
    dist_on = world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1"
    # BENCH_BACKEND=gloo: rehearsal of the N > 1 path with every rank on the visible GPUs
    # round-robin (e.g. 2 ranks on a 1-GPU box); the product path is "nccl" = RCCL over xGMI
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    dev = torch.device("cuda", local)
    if dist_on:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)
    if args.layer_only:
        Ns = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512)
        print(json.dumps([bench_layer(Ns, ("q8_1",), max(20, args.steps // 4), args.warmup, dev, fuse=f)
                          for f in (True, False)]), flush=True)
        return
    name = STRONG[1] if args.strong else args.config
    fmt, M, K, N = CONFIGS[name]
    sweep_steps = max(20, args.steps // 4)

    if args.strong:
        head = bench_sharded(name, args.steps, args.warmup, dev, dist_on, world, rank)
        R = head["rows_per_rank"]
        head["roofline"] = dict(roofline(fmt, R, K, N, head["compute_ms_per_step"] / 1e3),
                                kernel="per-rank local step on its R rows (act quant + MMQ), compute only")
    elif dist_on:
        head = bench_sharded(name, args.steps, args.warmup, dev, dist_on, world, rank, M_global=world * M)
        head["roofline"] = dict(roofline(fmt, M, K, N, head["compute_ms_per_step"] / 1e3),
                                kernel="per-rank local step (act quant + MMQ), compute only")
    else:
        head = bench_config(name, args.steps, args.warmup, dev)
    strong = []
    if dist_on and not args.strong:
        for sname in STRONG:
            strong.append(bench_sharded(sname, sweep_steps, args.warmup, dev, dist_on, world, rank))
    sweep = []
    if not args.quick and not args.strong and not dist_on:
        for sname in CONFIGS:
            if sname != name:
                sweep.append(bench_config(sname, sweep_steps, args.warmup, dev))
        sweep.append(bench_layer((1, 2, 4, 8, 16, 32, 64, 128, 256, 512), ("q8_1", "fp8"), sweep_steps, args.warmup,
                                 dev))
        sweep.append(bench_layer((1, 16, 128, 512), ("q8_1",), sweep_steps, args.warmup, dev, fuse=False))
        sweep.append(bench_msweep(sweep_steps, args.warmup, dev))
        sweep.extend(bench_fp8(("q8_0_4096x4096_m128", "q4_k_11008x4096_m128", "q6_k_28672x8192_m128",
                                "q4_k_4096x4096_m1"), sweep_steps, args.warmup, dev))
    cpu, cpu_var = None, None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, cpu_var = cpu_baseline(fmt, M, K, N)

    if rank == 0:
        line = {
            "metric": "effective fp16 TFLOPS (+ quant-weight GB/s) per GGUF type",
            "value": round(head["tflops"], 3),
            "unit": "TFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["ms_per_step"], 6),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f16" if N > 4 else "i8",
            "arith": "q8_1 activations x dequantized GGUF weights on fp16 MFMA, fp32 accumulate" if N > 4 else
                     "q8_1 int8 activations x GGUF int codes on v_dot4_i32_i8, fp32 block scaling",
            "data": "synthetic (random packed blocks, N(0,1) fp16 activations)",
            "config": {"workload": name, "gguf_type": fmt, "N_out": M, "K": K, "M_tok": N,
                       "global_N_out": M if args.strong else M * world,
                       "parallelism": f"rowshard{world}" if world > 1 else "single",
                       "weight_copies_rotated": head["weight_copies"]},
            "weight_GBps": round(head["weight_GBps"], 1),
            "roofline": head["roofline"],
            "cpu_baseline": cpu,
        }
        if "compute_only_tflops" in head:
            line["compute_only_tflops"] = round(head["compute_only_tflops"], 3)
            line["compute_ms_per_step"] = round(head["compute_ms_per_step"], 6)
        if cpu_var:
            line["cpu_baseline_variants"] = cpu_var
        if strong:
            line["strong"] = [compact(e) for e in strong]
        if sweep:
            line["sweep"] = [compact(e) for e in sweep]
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
