#!/usr/bin/env python3
"""bench.py -- GGUF MMQ throughput on MI355X (BASELINE.json metric:
"effective fp16 TFLOPS + quant-weight GB/s per GGUF type, M=1 and M=128").

Default workload = BASELINE.json configs[1]: Q8_0 weights N_out=4096 x K=4096, M_tok=128
fp16 activations on one MI355X.  One "step" = one drop-in call: q8_1 quantization of the
activations + the MMQ over one weight matrix (gq_mmq).  Inputs are resident in HBM before
timing.  K steps are captured into a hipGraph; ceil(copies / K) such graphs together cycle
over >= 1 GiB of distinct weight copies (rotation_plan), whatever K is, and are replayed
round robin, so every timed replay finds its weights evicted from the 256 MB Infinity Cache by
the >= 1 GiB read since.  Time = HIP events around one replay (K steps), bracketed by barrier +
synchronize; the MEDIAN over the replays is reported.

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


def rotation_plan(wbytes: int, steps: int, rotate: int = ROTATE_BYTES):
    """-> (ncopies, plans): ncopies = ceil(rotate / wbytes) (>= 2) distinct weight copies and
    G = ceil(ncopies / steps) graphs of `steps` launches; launch i of graph g uses copy
    (g * steps + i) % ncopies.  Replayed round robin (timed_rotation), every copy is read once
    per round, so >= rotate bytes separate two reads of one copy whatever `steps` is."""
    ncopies = max(2, math.ceil(rotate / max(1, wbytes)))
    G = max(1, math.ceil(ncopies / max(1, steps)))
    return ncopies, [[(g * steps + i) % ncopies for i in range(steps)] for g in range(G)]


def rotated_bytes(wbytes: int, plans) -> int:
    """Distinct weight bytes a rotation's graphs read per round."""
    return wbytes * len({c for p in plans for c in p})


def timed_rotation(graphs, dev, dist_on=False) -> float:
    """Median seconds per replay: one untimed round, then round-robin replays of the graphs
    (at least 6, at least 2 rounds), each timed alone (timed_replay)."""
    for g in graphs:
        g.replay()
    torch.cuda.synchronize(dev)
    rounds = max(2, math.ceil(6 / len(graphs)))
    return float(np.median([timed_replay(g, dev, dist_on) for _ in range(rounds) for g in graphs]))


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
        self.wbytes, _, _ = model(fmt, M, K, N)
        self.ncopies, self.plans = rotation_plan(self.wbytes, steps)
        self.rotated = rotated_bytes(self.wbytes, self.plans)
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

    def step(self, i, copy, c=None):
        A = self.weights[copy]
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

    def kernel(self, i, copy):
        A = self.weights[copy]
        rc = self.L.gq_mmq_prepared_ex(self.gtype, self.act, A.data_ptr(), self.ws.data_ptr(), self.ws_bytes,
                                       self.C[i & 1].data_ptr(), self.M, self.N, self.K, self.M, self._stream())
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def capture(self, fn, copies):
        """One graph of fn(i, copies[i]) for every i."""
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            fn(0, copies[0])  # warm the launch path outside capture
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        with torch.cuda.graph(g):
            for i, c in enumerate(copies):
                fn(i, c)
        return g

    def graphs(self, fn):
        """The rotation's graphs (rotation_plan) of fn."""
        return [self.capture(fn, p) for p in self.plans]

    def timed(self, fn):
        """Median seconds per step of fn over the rotation (timed_rotation)."""
        gs = self.graphs(fn)
        t = timed_rotation(gs, self.dev) / len(self.plans[0])
        del gs
        return t


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


# ---------------------------------------------------------------------------------------
# N > 1: row-sharded strong scaling of BASELINE configs[3] (+ weak scaling as an extra field)

# (fmt, N_out, K) of the strong-scaling matrix and its token counts; the CPU rehearsal
# (BENCH_REHEARSAL=1: no GPU, gloo, the product's CPU MMQ) runs the same code on a small shape
STRONG_SHAPE, STRONG_TOKENS = ("q6_k", 28672, 8192), (1, 128)
WEAK_SHAPE = ("q8_0", 4096, 4096, 128)
# (the rehearsal keeps the 28672-row geometry -- 14336 / 7168 / 3584-row shards at 2 / 4 / 8 ranks,
# each cut into 1 / 2 / 4 chunks of whole 64-row tiles -- with one super-block of K)
REHEARSAL_STRONG, REHEARSAL_TOKENS, REHEARSAL_WEAK = ("q6_k", 28672, 256), (1, 8), ("q8_0", 256, 512, 8)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv, n: int) -> int:
    """--gpus N > 1 outside torch.distributed: run the N ranks (one process per GPU) as a child
    `python -m torch.distributed.run` and return its exit code.  Runs before any GPU call, and
    the parent never replaces itself (no exec)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd).returncode


class ShardStep:
    """One rank's part of a row-sharded MMQ step (dist/row_shard.py's partitioning): its R rows of
    an M_global-row matrix, cut into C row chunks; per chunk the local MMQ into a contiguous (N, Rc)
    slab, an all_gather of the chunk (RCCL over xGMI; gloo in the rehearsal) and its assembly into
    the (N, world * R) output -- chunk c's exchange runs on a side stream under chunk c+1's compute
    ("pipeline the all-gather in chunks").  On a GPU everything is captured into
    HIP graphs (the C ABI on torch's streams); in the CPU rehearsal (cpu=True) the compute is the
    product's CPU MMQ (libgguf_quant) and the timing eager."""

    CHUNKS = (1, 2, 4)

    def __init__(self, fmt, M_global, K, N, dev, world, rank, seed=0, cpu=False, A_shard=None, B=None, steps=1):
        """A_shard / B (tests): this rank's packed rows (dist.row_shard.shard_bytes, align 256) and
        the fp16 activations, instead of random ones."""
        from dist.row_shard import shard_rows
        self.fmt, self.Mg, self.K, self.N, self.dev, self.world, self.cpu = fmt, M_global, K, N, dev, world, cpu
        self.gtype = GTYPE[fmt]
        # R divisible into max(CHUNKS) chunks of whole 64-row tiles
        self.row0, self.rows, self.R = shard_rows(M_global, world, rank, align=64 * max(self.CHUNKS))
        qk, nbytes = BLOCK[fmt]
        self.rb = (K // qk) * nbytes
        nrows = max(self.rows, 1)
        if cpu:
            from utils.quantize.q8_1 import quantize_to_q8_1
            from utils.synth import random_blocks
            self.ncopies, self.plans = 1, [[0] * steps]
            base = torch.from_numpy(random_blocks(fmt, nrows, K, seed=seed + rank).view(np.int8))
            g = torch.Generator().manual_seed(seed + 1)
            self.B = torch.randn(N, K, generator=g).to(torch.float16) if B is None else B
            self.Bq = quantize_to_q8_1(self.B)
        else:
            import kernels._lib as kl
            self.kl, self.L = kl, kl.lib()
            self.ncopies, self.plans = rotation_plan(max(1, self.rows * self.rb), steps)
            base = device_random_blocks(fmt, nrows, K, dev, seed + rank)
            g = torch.Generator(device=dev).manual_seed(seed + 1)
            self.B = torch.randn(N, K, device=dev, generator=g).to(torch.float16) if B is None else B
            self.ws_bytes = max(max(1, kl.workspace_size(self.gtype, self.R // C, N, K)) for C in self.CHUNKS)
            self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        base = base[:self.rows * self.rb] if A_shard is None else A_shard
        assert base.numel() == self.rows * self.rb, "A_shard is not this rank's row range"
        self.weights = [base] + [base.clone() for _ in range(self.ncopies - 1)]
        z = dict(dtype=torch.float16, device=dev)
        # per chunk count, two buffer sets (steps alternate): slabs, gathered chunks, output
        self.slab = {C: [[torch.zeros(N, self.R // C, **z) for _ in range(C)] for _ in range(2)] for C in self.CHUNKS}
        self.gath = {C: [[torch.zeros(world, N, self.R // C, **z) for _ in range(C)] for _ in range(2)]
                     for C in self.CHUNKS}
        self.out = [torch.zeros(N, world * self.R, **z) for _ in range(2)]

    # -- the pieces of a step -------------------------------------------------------------
    def prepare(self):
        """Quantize the activations once per step (GEMM shapes; N <= 4 fuses it per call)."""
        if self.cpu or self.N <= 4:
            return
        rc = self.L.gq_act_prepare(self.B.data_ptr(), self.N, self.K, self.K, self.ws.data_ptr(), self.ws_bytes,
                                   torch.cuda.current_stream(self.dev).cuda_stream)
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def compute(self, copy, C, c, j):
        """Local MMQ of chunk c (of C) of weight copy `copy` into slab set j."""
        Rc = self.R // C
        r0 = c * Rc
        n = max(0, min(self.rows - r0, Rc))
        if n == 0 or self.N == 0:
            return
        A = self.weights[copy]
        out = self.slab[C][j][c]
        if self.cpu:
            from kernels.cpu_impls._cpu import cpu_mmq
            out[:, :n] = cpu_mmq(self.gtype, A[r0 * self.rb:(r0 + n) * self.rb], self.Bq, n, self.N, self.K)
            return
        a_ptr = A.data_ptr() + r0 * self.rb
        st = torch.cuda.current_stream(self.dev).cuda_stream
        if self.N <= 4:
            rc = self.L.gq_mmq(self.gtype, a_ptr, self.B.data_ptr(), out.data_ptr(), n, self.N, self.K, self.K, Rc,
                               self.ws.data_ptr(), self.ws_bytes, st)
        else:
            rc = self.L.gq_mmq_prepared(self.gtype, a_ptr, self.ws.data_ptr(), self.ws_bytes, out.data_ptr(), n,
                                        self.N, self.K, Rc, st)
        if rc:
            raise RuntimeError(self.L.gq_last_error().decode())

    def gather(self, C, c, j, async_op=False):
        import torch.distributed as dist
        g, sl = self.gath[C][j][c], self.slab[C][j][c]
        return dist.all_gather_into_tensor(g.view(self.world * self.N, self.R // C), sl, async_op=async_op)

    def assemble(self, C, c, j):
        """Gathered chunk c -> its column range of every rank's part of the output."""
        Rc = self.R // C
        self.out[j].view(self.N, self.world, self.R)[:, :, c * Rc:(c + 1) * Rc].copy_(
            self.gath[C][j][c].permute(1, 0, 2))

    def result(self, j=0):
        return self.out[j][:, :self.Mg]

    # -- GPU: three graphs ----------------------------------------------------------------
    def _graph(self, body, copies):
        """One graph of body(i, copies[i], warm=False) for every i (two warm steps first, eager)."""
        n = len(copies)
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):  # warm every op outside capture (RCCL communicator included)
            body(0, copies[0], True)
            body(1, copies[1 % n], True)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        if self.world > 1 or _dist_on():
            # let the watchdog reap the warm steps' finished work (it polls every ~100 ms)
            # before anything is recorded inside the capture
            time.sleep(0.3)
        g = torch.cuda.CUDAGraph()
        # thread_local: the process group's watchdog thread polls its work events during capture
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for i, cp in enumerate(copies):
                body(i, cp, False)
        return g

    def graph_compute(self, copies):
        def body(i, cp, warm):
            self.prepare()
            self.compute(cp, 1, 0, i & 1)
        return self._graph(body, copies)

    def graph_overlap(self, copies):
        """Independent steps: step i's exchange (one all_gather) runs on a side stream under step
        i+1's compute; slab set j is rewritten only after the exchange that read it."""
        side = torch.cuda.Stream(self.dev)
        done = [torch.cuda.Event() for _ in range(2)]
        n = len(copies)

        def body(i, cp, warm):
            j = i & 1
            cur = torch.cuda.current_stream(self.dev)
            if i >= 2 and not warm:  # (only events recorded inside this capture)
                cur.wait_event(done[j])
            self.prepare()
            self.compute(cp, 1, 0, j)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self.gather(1, 0, j)
                self.assemble(1, 0, j)
                done[j].record(side)
            if warm or i == n - 1:
                cur.wait_stream(side)
        return self._graph(body, copies)

    def graph_chain(self, copies, C):
        """Dependent steps: step i+1's matmul waits for step i's assembled output; inside a step
        the C chunks pipeline compute against the exchange."""
        side = torch.cuda.Stream(self.dev)
        ev = [torch.cuda.Event() for _ in range(C)]

        def body(i, cp, warm):
            cur = torch.cuda.current_stream(self.dev)
            self.prepare()
            for c in range(C):
                self.compute(cp, C, c, 0)
                ev[c].record(cur)
                side.wait_event(ev[c])
                with torch.cuda.stream(side):
                    self.gather(C, c, 0)
                    self.assemble(C, c, 0)
            cur.wait_stream(side)  # the next step starts from this step's output
        return self._graph(body, copies)

    # -- eager: the same three, launched one by one (the CPU rehearsal, and the GPU when a
    # capture failed on any rank); the GPU forms quantize the activations per step as the graphs do
    def copy_of(self, i):
        p = self.plans[(i // len(self.plans[0])) % len(self.plans)]
        return p[i % len(p)]

    def cpu_compute(self, n):
        for i in range(n):
            self.prepare()
            self.compute(self.copy_of(i), 1, 0, i & 1)

    def cpu_overlap(self, n):
        pending = []
        for i in range(n):
            j = i & 1
            self.prepare()
            self.compute(self.copy_of(i), 1, 0, j)
            pending.append((self.gather(1, 0, j, async_op=True), j))
            if len(pending) > 1:
                w, jj = pending.pop(0)
                w.wait()
                self.assemble(1, 0, jj)
        for w, jj in pending:
            w.wait()
            self.assemble(1, 0, jj)

    def cpu_chain(self, n, C):
        for i in range(n):
            works = []
            self.prepare()
            for c in range(C):
                self.compute(self.copy_of(i), C, c, 0)
                works.append(self.gather(C, c, 0, async_op=True))
            for c, w in enumerate(works):
                w.wait()
                self.assemble(C, c, 0)


def _max_over_ranks(t, dev):
    import torch.distributed as dist
    tt = torch.tensor([t], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def agree_all(ok: bool, dev) -> bool:
    """True on every rank iff `ok` on every rank (one all_reduce MIN): a decision every rank
    must take the same way -- e.g. graphs holding captured all_gathers on some ranks and eager
    collectives on others would pair mismatched collectives and hang the group."""
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def capture_fault_injected() -> bool:
    """BENCH_INJECT_CAPTURE_FAIL=<rank>: that rank's capture step fails (tests of the agreement)."""
    r = os.environ.get("BENCH_INJECT_CAPTURE_FAIL")
    return r is not None and r != "" and int(r) == int(os.environ.get("RANK", "0"))


def time_eager(run, steps, warmup, dev, cpu):
    import torch.distributed as dist
    run(max(1, warmup))
    if not cpu:
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    run(steps)
    if not cpu:
        torch.cuda.synchronize(dev)
    t = time.perf_counter() - t0
    dist.barrier()
    return _max_over_ranks(t, dev) / steps


def time_sharded(ss: ShardStep, steps, warmup):
    """{compute, overlap, chain_C..., graph}: seconds per step, max over ranks (barrier on both
    sides).  GPU: every key's graphs (one per rotation plan) are captured first, then the ranks
    agree (agree_all) -- all replay graphs, or, if a capture failed on ANY rank, all time every
    key eagerly (the same ops, the per-step activation quantization included).  A failed capture
    (hipErrorStreamCaptureUnjoined once in four world-1 runs in round 3, its log not kept) then
    changes the timing mode of the whole line, never of one rank or one key."""
    eager = {"compute": ss.cpu_compute, "overlap": ss.cpu_overlap}
    eager.update({f"chain{C}": (lambda n, C=C: ss.cpu_chain(n, C)) for C in ss.CHUNKS})
    built, ok = {}, True
    if not ss.cpu:
        makers = [("compute", ss.graph_compute), ("overlap", ss.graph_overlap)] + \
                 [(f"chain{C}", (lambda cp, C=C: ss.graph_chain(cp, C))) for C in ss.CHUNKS]
        try:
            if capture_fault_injected():
                raise RuntimeError("injected capture failure (BENCH_INJECT_CAPTURE_FAIL)")
            for key, make in makers:
                built[key] = [make(p) for p in ss.plans]
        except Exception as e:
            print(f"bench: graph capture of the sharded step failed on rank {os.environ.get('RANK', '0')} ({e!r})",
                  file=sys.stderr, flush=True)
            ok = False
            built = {}
            torch.cuda.synchronize(ss.dev)
    elif capture_fault_injected():  # (the CPU rehearsal captures nothing: the agreement alone)
        print(f"bench: injected capture failure (BENCH_INJECT_CAPTURE_FAIL) on rank {os.environ.get('RANK', '0')}",
              file=sys.stderr, flush=True)
        ok = False
    ok = agree_all(ok, ss.dev)
    res = {"graph": ok and not ss.cpu, "capture_agreed": ok}
    for key in eager:
        if res["graph"]:
            res[key] = timed_rotation(built[key], ss.dev, True) / steps
        else:
            res[key] = time_eager(eager[key], steps, warmup, ss.dev, ss.cpu)
    del built
    return res


def time_unsharded(fmt, M, K, N, steps, warmup, dev, cpu, graph=True):
    """The whole matrix on this one device (rank 0's 1-GPU reference for speedup_vs_1gpu): the same
    ShardStep compute as the ranks run, with world 1 (no process-group calls), timed the way the
    ranks' keys were (graph: the rotation's graphs; else eager)."""
    ss = ShardStep(fmt, M, K, N, dev, 1, 0, cpu=cpu, steps=steps)
    if cpu or not graph:
        ss.cpu_compute(max(1, warmup))
        if not cpu:
            torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ss.cpu_compute(steps)
        if not cpu:
            torch.cuda.synchronize(dev)
        t = (time.perf_counter() - t0) / steps
    else:
        gs = [ss.graph_compute(p) for p in ss.plans]
        t = timed_rotation(gs, dev) / steps
        del gs
    del ss
    if not cpu:
        torch.cuda.empty_cache()
    return t


def bench_sharded(fmt, Mg, K, N, steps, warmup, dev, world, rank, cpu, unsharded=True):
    """One row-sharded configuration over the group: compute-only, end-to-end with overlap and the
    dependent chain (per chunk count; the best is `e2e_chain`), and -- rank 0, the other ranks
    waiting -- the unsharded matrix on one device for speedup_vs_1gpu."""
    import torch.distributed as dist
    ss = ShardStep(fmt, Mg, K, N, dev, world, rank, cpu=cpu, steps=steps)
    t = time_sharded(ss, steps, warmup)
    rows_per_rank, ncopies = ss.R, ss.ncopies
    rotated = rotated_bytes(max(1, ss.rows * ss.rb), ss.plans)
    del ss
    if not cpu:
        torch.cuda.empty_cache()
    t1 = None
    if unsharded:
        dist.barrier()
        if rank == 0:
            t1 = time_unsharded(fmt, Mg, K, N, steps, warmup, dev, cpu, graph=t["graph"])
        dist.barrier()
    chains = {C: t[f"chain{C}"] for C in ShardStep.CHUNKS}
    best = min(chains, key=chains.get)
    _, _, flops = model(fmt, Mg, K, N)
    qk, nbytes = BLOCK[fmt]
    wbytes = Mg * (K // qk) * nbytes
    ms = lambda x: round(x * 1e3, 6)  # noqa: E731
    out = {"config": f"{fmt}_{Mg}x{K}_m{N}", "fmt": fmt, "N_out_global": Mg, "K": K, "M_tok": N, "ranks": world,
           "rows_per_rank": rows_per_rank, "weight_copies": ncopies, "weight_bytes_rotated_per_rank": rotated,
           "compute_ms_per_step": ms(t["compute"]), "e2e_overlap_ms_per_step": ms(t["overlap"]),
           "e2e_chain_ms_per_step": ms(chains[best]), "e2e_chain_chunks": best,
           "e2e_chain_ms_by_chunks": {str(C): ms(v) for C, v in chains.items()},
           "compute_tflops": round(flops / t["compute"] / 1e12, 3),
           "e2e_overlap_tflops": round(flops / t["overlap"] / 1e12, 3),
           "e2e_chain_tflops": round(flops / chains[best] / 1e12, 3),
           "e2e_chain_weight_GBps": round(wbytes / chains[best] / 1e9, 1),
           "collective": f"all_gather_into_tensor per row chunk (backend {dist_backend()}) + assemble copy",
           "timing": ("hipGraph replay (median of the rotation's graphs)" if t["graph"] else
                      "eager" + ("" if t["capture_agreed"] else " (a graph capture failed on some rank; every rank "
                                                                    "and the 1-GPU reference timed eagerly)"))}
    if t1 is not None:
        out["unsharded_1dev_ms_per_step"] = ms(t1)
        out["speedup_vs_1gpu"] = {"compute": round(t1 / t["compute"], 3), "e2e_overlap": round(t1 / t["overlap"], 3),
                                  "e2e_chain": round(t1 / chains[best], 3)}
    return out


def _dist_on() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def dist_backend():
    import torch.distributed as dist
    b = dist.get_backend() if dist.is_initialized() else "none"
    return "nccl = RCCL over xGMI" if b == "nccl" else b


def bench_config(name, steps, warmup, dev):
    """One config on this GPU: the drop-in step (gq_mmq) timed over a graph of `steps` calls,
    and the dominant kernel for the roofline."""
    fmt, M, K, N = CONFIGS[name]
    r = Runner(fmt, M, K, N, dev, steps)
    gw = r.capture(r.step, [i % r.ncopies for i in range(max(1, warmup))])
    gw.replay()
    torch.cuda.synchronize(dev)
    del gw
    per_step = r.timed(r.step)
    # dominant kernel: decode (N <= 4) -- the step IS one launch (fused quantizer + weight
    # stream), so its time is the step's; GEMM -- the MMQ call alone (gemm_kernel [+ split-K
    # reduce]) with the activations prepared once, K launches per graph, the same rotation
    import kernels._lib as kl
    if N <= 4:
        t_k = per_step
        kname = kl.route_name(kl.TYPES[fmt], M, N, K) + " (fused q8_1 + decode)"
    else:
        r.prepare()
        t_k = r.timed(r.kernel)
        kname = kl.route_name(kl.TYPES[fmt], M, N, K, prepared=True)  # (the library's own routing)
    wbytes, alg_bytes, flops = model(fmt, M, K, N)
    out = {
        "config": name, "fmt": fmt, "N_out": M, "K": K, "M_tok": N,
        "ms_per_step": per_step * 1e3,
        "tflops": flops / per_step / 1e12,
        "weight_GBps": wbytes / per_step / 1e9,
        "roofline": dict(roofline(fmt, M, K, N, t_k, load_traffic(name)), kernel=kname),
        "weight_copies": r.ncopies,
        "weight_bytes_rotated": r.rotated,
        "graphs_rotated": len(r.plans),
    }
    del r
    torch.cuda.empty_cache()
    return out


def bench_layer(Ns, acts, steps, warmup, dev, fuse=True, grouped="auto", gemm_grouped_min=None):
    """BASELINE configs[4]: the seven projections of a Llama-7B block under GGUF Q4_K_M (layer 0:
    attn_v and ffn_down in Q6_K, the rest Q4_K), shared inputs quantized once per group
    (kernels.layer_mix.LayerMix; fuse: q+k and gate+up as one call each), for each token count in
    Ns and activation format in acts ("q8_1": the reference's semantics; "fp8": the e4m3 variant).
    Weights rotate over >= 1 GiB.  grouped: LayerMix's grouped setting ("auto" / True: the whole
    layer as one gq_mmq_grouped launch at 1..4 tokens and one gq_mmq_grouped_prepared launch from
    17 tokens; False: one launch per set)."""
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GEMM_GROUPED_MIN_TOKENS, GROUPED_MAX_TOKENS, GGUFLinear, LayerMix
    types = q4_k_m_layer_types(0, 32)
    one = {n: device_random_blocks(types[n], M, K, dev, seed=i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    layer_bytes = sum(t.numel() for t in one.values())
    ncopies, plans = rotation_plan(layer_bytes, steps)
    lins = [{n: GGUFLinear(types[n], one[n] if c == 0 else one[n].clone(), *LLAMA_LAYER_SHAPES[n])
             for n in LLAMA_LAYER_SHAPES} for c in range(ncopies)]
    res = []
    for act in acts:
        layers = [LayerMix(lin, act=act, fuse=fuse, grouped=grouped, gemm_grouped_min=gemm_grouped_min) for lin in lins]
        for N in Ns:
            g = torch.Generator(device=dev).manual_seed(7)
            x = torch.randn(N, 4096, device=dev, generator=g).to(torch.float16)
            h = torch.randn(N, 11008, device=dev, generator=g).to(torch.float16)
            # output buffers of the unfused projections (fused ones are column views of the
            # layer's own buffer; a buffer for them would add a copy)
            outs = {n: torch.empty(N, M, dtype=torch.float16, device=dev) for n, (M, K) in LLAMA_LAYER_SHAPES.items()
                    if n not in layers[0].parts}
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
            grs = []
            for p in plans:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    for c in p:
                        layers[c].forward(x, h, out=outs)
                grs.append(gr)
            t = timed_rotation(grs, dev) / steps
            res.append({"config": f"q4_k_m_llama7b_layer_m{N}", "act": act, "fused": fuse,
                        "grouped": act == "q8_1" and N <= GROUPED_MAX_TOKENS[grouped],
                        "gemm_grouped": N >= GEMM_GROUPED_MIN_TOKENS[grouped],
                        "fmt": "q4_k+q6_k", "M_tok": N,
                        "us_per_step": round(t * 1e6, 2), "tflops": round(flops / t / 1e12, 3),
                        "weight_GBps": round(layer_bytes / t / 1e9, 1)})
            del grs
    del lins, layers
    torch.cuda.empty_cache()
    return {"config": "q4_k_m_llama7b_layer_msweep", "types": types, "weight_bytes": layer_bytes,
            "weight_copies": ncopies, "weight_bytes_rotated": rotated_bytes(layer_bytes, plans), "points": res}


def bench_fp8(names, steps, warmup, dev):
    """The fp8 activation variant on BASELINE shapes: the step (gq_mmq_ex, GQ_ACT_FP8_E4M3)."""
    out = []
    for name in names:
        fmt, M, K, N = CONFIGS[name]
        r = Runner(fmt, M, K, N, dev, steps, act="fp8")
        gw = r.capture(r.step, [i % r.ncopies for i in range(max(1, warmup))])
        gw.replay()
        t = r.timed(r.step)
        wbytes, _, flops = model(fmt, M, K, N)
        out.append({"config": name + "_fp8act", "act": "fp8", "us_per_step": round(t * 1e6, 2),
                    "tflops": round(flops / t / 1e12, 3), "weight_GBps": round(wbytes / t / 1e9, 1),
                    "weight_bytes_rotated": r.rotated})
        del r, gw
        torch.cuda.empty_cache()
    return out


def bench_msweep(steps, warmup, dev, fmt="q4_k", M=4096, K=4096):
    """configs[4]'s M sweep: tokens 1..512 on one Q4_K 4096x4096 matrix (the step: gq_mmq)."""
    res = []
    for N in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
        r = Runner(fmt, M, K, N, dev, steps)
        gw = r.capture(r.step, [i % r.ncopies for i in range(max(1, warmup))])
        gw.replay()
        t = r.timed(r.step)
        wbytes, alg_bytes, flops = model(fmt, M, K, N)
        res.append({"M_tok": N, "us_per_step": round(t * 1e6, 2), "tflops": round(flops / t / 1e12, 3),
                    "weight_GBps": round(wbytes / t / 1e9, 1), "alg_GBps": round(alg_bytes / t / 1e9, 1),
                    "weight_bytes_rotated": r.rotated})
        del r, gw
        torch.cuda.empty_cache()
    return {"config": f"{fmt}_{M}x{K}_msweep", "points": res}


def short_kernel(name: str) -> str:
    """The library's route name (gq_debug_route) in a few characters for the compact rows."""
    for k, v in (("stream_decode", "decode"), ("rgemm_kernel (in-launch", "rgemm-ilc"), ("rgemm", "rgemm+reduce"),
                 ("sgemm_grouped", "sgemm-sk+reduce"), ("sgemm", "sgemm+reduce"), ("kstream_kernel +", "kstream+reduce"),
                 ("kstream", "kstream"), ("skinny", "skinny"), ("gemv", "gemv"), ("hipBLASLt", "dequant+blaslt"),
                 ("gemm_kernel", "gemm+reduce")):
        if k in name:
            return v
    return name


# the compact per-type row (bench line "per_type"): what the BASELINE metric asks for, per config
PER_TYPE_COLS = ["config", "step_us", "tflops", "weight_GBps", "bound", "frac", "traffic_over_alg", "kernel"]


def per_type_row(e):
    rf = e["roofline"]
    alg = rf.get("alg_bytes_per_launch") or model(e["fmt"], e["N_out"], e["K"], e["M_tok"])[1]
    tr = rf.get("traffic")
    return [e["config"], round(e["ms_per_step"] * 1e3, 2), round(e["tflops"], 1), round(e["weight_GBps"]),
            rf["bound"], round(rf["frac"], 3), round(tr / alg, 2) if tr else None, short_kernel(rf.get("kernel", ""))]


def compact_sweep(sweep):
    """The sweep blocks as short columns (the whole JSON line has to fit the ~8 KB the driver keeps
    of stdout: round 5's line lost every M = 1 figure to that cut)."""
    out = {}
    for e in sweep:
        c = e.get("config", "")
        if c == "q4_k_m_llama7b_layer_msweep":
            for pt in e["points"]:
                key = f"layer7b_{pt['act']}" + ("" if pt["fused"] else "_unfused")
                d = out.setdefault(key, {"M_tok": [], "us": []})
                d["M_tok"].append(pt["M_tok"])
                d["us"].append(pt["us_per_step"])
        elif c.endswith("_msweep"):
            out[c] = {"M_tok": [p["M_tok"] for p in e["points"]], "us": [p["us_per_step"] for p in e["points"]]}
        elif c.endswith("_fp8act"):
            out.setdefault("fp8act_us", {})[c[:-len("_fp8act")]] = e["us_per_step"]
    if any(k.startswith("layer7b") for k in out):
        out["layer7b_weight_bytes"] = next(e["weight_bytes"] for e in sweep
                                           if e.get("config") == "q4_k_m_llama7b_layer_msweep")
    return out


def single_line(args, name, head, sweep, cpu_b, cpu_var, eager, eager_host):
    """The N = 1 JSON line: the contract's fields for the headline, then one compact row per
    BASELINE config (per_type) and the sweeps as short columns (compact_sweep)."""
    fmt, M, K, N = CONFIGS[name]
    line = {
        "metric": "effective fp16 TFLOPS (+ quant-weight GB/s) per GGUF type",
        "value": round(head["tflops"], 3),
        "unit": "TFLOP/s",
        "n_gpus": 1,
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
        "config": {"workload": name, "gguf_type": fmt, "N_out": M, "K": K, "M_tok": N, "parallelism": "single",
                   "weight_copies": head["weight_copies"], "weight_bytes_rotated": head["weight_bytes_rotated"],
                   "graphs_rotated": head["graphs_rotated"],
                   "timing": "median of round-robin replays of the rotation's graphs, K steps each"},
        "weight_GBps": round(head["weight_GBps"], 1),
        "roofline": head["roofline"],
        "cpu_baseline": cpu_b,
        "eager_us": eager,
        "eager_us_is": "median of 1000 eager kernels.mmq_q4_k.mmq_q4_k(A, B, 4096, 1, 4096) calls, each synchronized",
        "eager_host_us": eager_host,
        "eager_host_us_is": "the same call 1000 times back to back, one synchronize at the end, / 1000 (the "
                            "per-call host cost when the kernel is shorter)",
    }
    if cpu_var:
        line["cpu_baseline_variants"] = [{k: v[k] for k in ("value", "unit", "cores", "kind", "sample")} for v in cpu_var]
    if sweep:
        heads = [head] + [e for e in sweep if "roofline" in e]
        line["per_type_cols"] = PER_TYPE_COLS
        line["per_type"] = [per_type_row(e) for e in heads]
        line.update(compact_sweep(sweep))
    return line


def eager_call_us(dev, n=1000):
    """The drop-in called eagerly, kernels.mmq_q4_k.mmq_q4_k(A, B, 4096, 1, 4096) (the reference's
    callers' form, /root/reference/test/test_mmq_q4_k.py:34): Python + ctypes + output allocation
    + launch.  -> (median wall time of n calls each synchronized, host time per call of n
    back-to-back calls with one synchronize at the end)."""
    from kernels.mmq_q4_k import mmq_q4_k
    A = device_random_blocks("q4_k", 4096, 4096, dev, seed=11)
    B = torch.randn(1, 4096, device=dev).to(torch.float16)
    for _ in range(20):
        mmq_q4_k(A, B, 4096, 1, 4096)
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        mmq_q4_k(A, B, 4096, 1, 4096)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(n):
        mmq_q4_k(A, B, 4096, 1, 4096)
    torch.cuda.synchronize(dev)
    host = (time.perf_counter() - t0) / n
    return round(float(np.median(ts)) * 1e6, 2), round(host * 1e6, 2)


def strong_line(args, world, rank, dev, cpu):
    """The N > 1 line: Q6_K 28672x8192 (BASELINE configs[3]) row-sharded over the ranks at M_tok
    1 and 128 (value = the 128-token dependent-chain end-to-end rate), weak scaling as an extra
    field."""
    fmt, M, K = REHEARSAL_STRONG if cpu else STRONG_SHAPE
    toks = REHEARSAL_TOKENS if cpu else STRONG_TOKENS
    pts = [bench_sharded(fmt, M, K, N, args.steps, args.warmup, dev, world, rank, cpu) for N in toks]
    wf, wM, wK, wN = REHEARSAL_WEAK if cpu else WEAK_SHAPE
    weak = bench_sharded(wf, world * wM, wK, wN, max(20, args.steps // 4) if not cpu else args.steps, args.warmup, dev,
                         world, rank, cpu, unsharded=False)
    head = pts[-1]
    N = head["M_tok"]
    if rank != 0:
        return None
    line = {
        "metric": "effective fp16 TFLOPS (+ quant-weight GB/s) per GGUF type",
        "value": head["e2e_chain_tflops"],
        "unit": "TFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["e2e_chain_ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic (random packed blocks, N(0,1) fp16 activations)",
        "config": {"workload": head["config"] + f"_rowshard{world}", "gguf_type": fmt, "N_out": M, "K": K, "M_tok": N,
                   "parallelism": f"rowshard{world}", "rows_per_rank": head["rows_per_rank"],
                   "value_is": "dependent-chain end-to-end (step i+1 waits for step i's assembled output), "
                               "best row-chunk count"},
        "compute_ms_per_step": head["compute_ms_per_step"],
        "e2e_overlap_ms_per_step": head["e2e_overlap_ms_per_step"],
        "e2e_chain_ms_per_step": head["e2e_chain_ms_per_step"],
        "speedup_vs_1gpu": head.get("speedup_vs_1gpu"),
        "weight_GBps": head["e2e_chain_weight_GBps"],
        "roofline": dict(roofline(fmt, head["rows_per_rank"], K, N, head["compute_ms_per_step"] / 1e3),
                         kernel="rank-local step on its rows (act quant + MMQ), compute only"),
        "cpu_baseline": None,
        "strong": pts,
        "weak": weak,
    }
    if cpu:
        line["rehearsal"] = ("CPU rehearsal (BENCH_REHEARSAL=1): gloo, the product's CPU MMQ, shapes scaled down; "
                             "not a GPU measurement")
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default=DEFAULT, choices=sorted(CONFIGS))
    ap.add_argument("--strong", action="store_true", help="the N > 1 line (Q6_K 28672x8192 row-sharded) at any N")
    ap.add_argument("--quick", action="store_true", help="headline only: no per-type sweep")
    ap.add_argument("--sweep", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--detail", default=None, help="also write the full per-config records to this JSON file")
    ap.add_argument("--layer-only", action="store_true",
                    help="print only the Q4_K_M layer sweep (fused and unfused), one JSON line")
    args = ap.parse_args()

    # --gpus N > 1 outside torch.distributed: the N ranks run as a child process
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: world size {world} != --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    # BENCH_REHEARSAL=1: the N > 1 path on the CPU (gloo, product CPU MMQ, small shapes) -- the
    # CPU test of the launcher and the line; BENCH_FORCE_DIST=1: the N > 1 path at world 1 (RCCL
    # graph capture on a 1-GPU box)
    cpu = os.environ.get("BENCH_REHEARSAL") == "1"
    multi = world > 1 or args.strong or os.environ.get("BENCH_FORCE_DIST") == "1"
    if multi and not cpu:
        # The process group's watchdog thread polls the end events of its enqueued work.  With
        # its event cache on, an event can be recorded again inside a graph capture while a
        # finished work still holds it, and the watchdog's query then fails with
        # hipErrorCapturedEvent ("operation not permitted on an event last recorded in a
        # capturing stream") -- which it rethrows, terminating the process (seen at world 1,
        # profiles/r04/b6_tests.txt).  Fresh events per work, and a watchdog that logs CUDA
        # errors instead of rethrowing them (set before the process group exists).
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        os.environ.setdefault("TORCH_NCCL_RETHROW_CUDA_ERRORS", "0")
    dev = torch.device("cpu") if cpu else torch.device("cuda", local)
    if multi:
        import torch.distributed as dist
        init = None if "MASTER_ADDR" in os.environ else f"tcp://127.0.0.1:{free_port()}"
        if cpu:
            dist.init_process_group("gloo", init_method=init, world_size=world, rank=rank)
        else:
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", init_method=init, world_size=world, rank=rank, device_id=dev)
        line = strong_line(args, world, rank, dev, cpu)
        if line is not None:
            print(json.dumps(line), flush=True)
        dist.destroy_process_group()
        return
    torch.cuda.set_device(dev)
    if args.layer_only:
        Ns = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512)
        print(json.dumps([bench_layer(Ns, ("q8_1",), max(20, args.steps // 4), args.warmup, dev, fuse=f, grouped=g)
                          for f in (True, False) for g in ("auto", False)]), flush=True)
        return
    name = args.config
    fmt, M, K, N = CONFIGS[name]
    sweep_steps = max(20, args.steps // 4)
    head = bench_config(name, args.steps, args.warmup, dev)
    sweep = []
    if not args.quick:
        for sname in CONFIGS:
            if sname != name:
                sweep.append(bench_config(sname, sweep_steps, args.warmup, dev))
        sweep.append(bench_layer((1, 2, 4, 8, 16, 32, 64, 128, 256, 512), ("q8_1", "fp8"), sweep_steps, args.warmup,
                                 dev))
        sweep.append(bench_layer((1, 16, 128, 512), ("q8_1",), sweep_steps, args.warmup, dev, fuse=False))
        sweep.append(bench_msweep(sweep_steps, args.warmup, dev))
        sweep.extend(bench_fp8(("q8_0_4096x4096_m128", "q4_k_11008x4096_m128", "q6_k_28672x8192_m128",
                                "q4_k_4096x4096_m1"), sweep_steps, args.warmup, dev))
    eager, eager_host = eager_call_us(dev)
    cpu_b, cpu_var = (None, None) if args.no_cpu else cpu_baseline(fmt, M, K, N)
    line = single_line(args, name, head, sweep, cpu_b, cpu_var, eager, eager_host)
    if args.detail:  # the full per-config records (every roofline field), for the profiles/ notes
        with open(args.detail, "w") as f:
            json.dump({"head": head, "sweep": sweep, "cpu_baseline_variants": cpu_var}, f)
    print(json.dumps(line, separators=(",", ":")), flush=True)


if __name__ == "__main__":
    main()
