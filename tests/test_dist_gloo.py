"""Row-sharded MMQ across 2 processes (gloo, CPU): shard boundaries, the all-gather and the
(world, N, R) -> (N, M) assembly.  The per-shard compute here is the oracle (test
infrastructure) or the product's CPU MMQ; on GPUs the same classes call the HIP MMQ
(tests/test_gpu_paths.py).  Also bench.py's N > 1 path: the --gpus launcher, the world-size
check, and its chunked pipeline (bench.ShardStep) in the CPU rehearsal mode."""
import os
import sys
import tempfile

import json
import subprocess

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _oracle_compute(fmt):
    import oracle as O

    def run(A_shard, B, rows, N, K, out):
        C = O.mmq_from_fp16(fmt, A_shard.numpy(), B.numpy(), rows, N, K, O.IDEAL)
        out.copy_(torch.from_numpy(C))

    return run


def _worker(rank, world, initfile, fmt, M, N, K, align, q, chunks=1):
    for p in (os.path.join(ROOT, "gguf-triton-kernel_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    from dist.row_shard import RowShardedMMQ, shard_bytes
    from utils.synth import random_activations, random_blocks
    dist.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank, world_size=world)
    try:
        A = torch.from_numpy(random_blocks(fmt, M, K, seed=9).view(np.int8))
        B = torch.from_numpy(random_activations(N, K, seed=4))
        op = RowShardedMMQ(fmt, shard_bytes(fmt, A, M, K, world, rank, align), M, K, align=align,
                           compute=_oracle_compute(fmt))
        C = op(B, N, chunks=chunks)
        if rank == 0:
            q.put(C.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt,M,N,K,align,chunks", [("q4_k", 200, 3, 512, 64, 1), ("q8_0", 130, 1, 96, 16, 1),
                                                    ("q6_k", 64, 5, 256, 64, 1), ("q4_k", 40, 2, 256, 64, 1),
                                                    ("q4_k", 200, 3, 512, 64, 3), ("q8_0", 130, 1, 96, 16, 4),
                                                    ("q6_k", 300, 5, 256, 64, 2)])
def test_row_sharded_matches_single(fmt, M, N, K, align, chunks):
    """One step and the chunk-pipelined step (RowShardedMMQ.pipelined) equal the unsharded
    product bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from utils.synth import random_activations, random_blocks
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        initfile = os.path.join(d, "init")
        ps = [ctx.Process(target=_worker, args=(r, world, initfile, fmt, M, N, K, align, q, chunks))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
        codes = [p.exitcode for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
        assert codes == [0] * world, codes
        got = q.get(timeout=10)
    A = random_blocks(fmt, M, K, seed=9)
    B = random_activations(N, K, seed=4)
    want = O.mmq_from_fp16(fmt, A, B, M, N, K, O.IDEAL)
    assert got.shape == (N, M)
    assert np.array_equal(got.view(np.uint16), want.view(np.uint16))


def test_shard_rows_cover_exactly():
    from dist.row_shard import shard_rows
    for M in (1, 63, 64, 65, 4096, 28672, 11008):
        for world in (1, 2, 3, 4, 8):
            covered = []
            for r in range(world):
                row0, rows, R = shard_rows(M, world, r)
                assert R % 64 == 0 and 0 <= rows <= R
                covered.extend(range(row0, row0 + rows))
            assert covered == list(range(M))


def _bench_worker(rank, world, initfile, fmt, M, N, K, q):
    for p in (ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")):
        sys.path.insert(0, p)
    import bench
    from dist.row_shard import shard_bytes
    from utils.synth import random_activations, random_blocks
    dist.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank, world_size=world)
    try:
        A = torch.from_numpy(random_blocks(fmt, M, K, seed=9).view(np.int8))
        B = torch.from_numpy(random_activations(N, K, seed=4))
        ss = bench.ShardStep(fmt, M, K, N, torch.device("cpu"), world, rank, cpu=True,
                             A_shard=shard_bytes(fmt, A, M, K, world, rank, align=256), B=B)
        res = {}
        for C in ss.CHUNKS:
            ss.cpu_chain(1, C)
            res[f"chain{C}"] = ss.result(0).numpy().copy()
        ss.cpu_overlap(2)
        res["overlap0"], res["overlap1"] = ss.result(0).numpy().copy(), ss.result(1).numpy().copy()
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt,M,N,K", [("q4_k", 700, 3, 512), ("q6_k", 1100, 1, 256), ("q8_0", 520, 6, 96)])
def test_bench_shard_step_pipeline_matches_single(fmt, M, N, K):
    """bench.ShardStep's chunked pipeline (1, 2, 4 row chunks per rank, each gathered and
    assembled on its own) and its overlapped form give the unsharded product's bits."""
    from kernels.cpu_impls._cpu import cpu_mmq
    from utils.quantize.q8_1 import quantize_to_q8_1
    from utils.synth import random_activations, random_blocks
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        initfile = os.path.join(d, "init")
        ps = [ctx.Process(target=_bench_worker, args=(r, world, initfile, fmt, M, N, K, q)) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=120)
        codes = [p.exitcode for p in ps]
        for p in ps:
            if p.is_alive():
                p.kill()
        assert codes == [0] * world, codes
        got = q.get(timeout=10)
    A = torch.from_numpy(random_blocks(fmt, M, K, seed=9).view(np.int8))
    Bq = quantize_to_q8_1(torch.from_numpy(random_activations(N, K, seed=4)))
    want = cpu_mmq({"q8_0": 0, "q4_k": 1, "q6_k": 2}[fmt], A, Bq, M, N, K).contiguous().numpy()
    for k, v in got.items():
        assert v.shape == (N, M), k
        assert np.array_equal(v.view(np.uint16), want.view(np.uint16)), k


def _run_bench(args, env_extra, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` (no torch.distributed environment) starts 2 ranks as a child
    torch.distributed.run and prints the strong-scaling line: n_gpus 2, scaling "strong", the
    compute-only / overlapped / dependent-chain end-to-end times and speedup_vs_1gpu (CPU
    rehearsal mode: gloo, the product's CPU MMQ, small shapes)."""
    r = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1"], {"BENCH_REHEARSAL": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    for k in ("compute_ms_per_step", "e2e_overlap_ms_per_step", "e2e_chain_ms_per_step"):
        assert d[k] > 0, k
    assert set(d["speedup_vs_1gpu"]) == {"compute", "e2e_overlap", "e2e_chain"}
    assert [p["M_tok"] for p in d["strong"]] == [1, 8] and all(p["ranks"] == 2 for p in d["strong"])
    assert d["weak"]["N_out_global"] == 2 * 256
    assert d["value"] == d["strong"][-1]["e2e_chain_tflops"]


def test_bench_world_size_mismatch_fails():
    """A torch.distributed world that is not --gpus ranks is an error (exit 2), before any
    device work."""
    r = _run_bench(["--gpus", "2", "--steps", "2"], {"WORLD_SIZE": "1", "BENCH_REHEARSAL": "1"}, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "world size 1 != --gpus 2" in r.stderr


def test_bench_capture_failure_is_agreed_by_every_rank():
    """A graph capture that fails on ONE rank (injected on rank 1: BENCH_INJECT_CAPTURE_FAIL=1)
    switches EVERY rank, and the 1-GPU reference, to eager timing: rank 0 never failed itself,
    yet its line says the capture failed on some rank; both ranks exit 0 (no rank replays graphs
    holding collectives while another runs them eagerly)."""
    r = _run_bench(["--gpus", "2", "--steps", "2", "--warmup", "1"],
                   {"BENCH_REHEARSAL": "1", "BENCH_INJECT_CAPTURE_FAIL": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for p in d["strong"] + [d["weak"]]:
        assert "capture failed on some rank" in p["timing"], p["timing"]
    assert "injected capture failure" in r.stderr


def test_bench_gpus8_rehearsal_with_rank5_capture_failure():
    """The 8-rank path the driver's 8-GPU node will run, rehearsed on the CPU (gloo): `bench.py
    --gpus 8 --strong` over the Q6_K 28672-row geometry (3584-row shards; K scaled down to one
    super-block), the 8-way agree_all with a capture failure injected on rank 5 only -- every rank
    and the 1-GPU reference switch to eager timing -- and the 1 / 2 / 4-chunk dependent-chain
    pipelines, each with its 8 all_gathers."""
    r = _run_bench(["--gpus", "8", "--strong", "--steps", "2", "--warmup", "1"],
                   {"BENCH_REHEARSAL": "1", "BENCH_INJECT_CAPTURE_FAIL": "5", "OMP_NUM_THREADS": "1"}, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["scaling"] == "strong"
    assert d["config"]["N_out"] == 28672 and d["config"]["rows_per_rank"] == 3584
    for p in d["strong"]:
        assert p["ranks"] == 8 and p["rows_per_rank"] == 3584
        assert set(p["e2e_chain_ms_by_chunks"]) == {"1", "2", "4"}
        assert all(v > 0 for v in p["e2e_chain_ms_by_chunks"].values())
        assert "capture failed on some rank" in p["timing"], p["timing"]
        assert set(p["speedup_vs_1gpu"]) == {"compute", "e2e_overlap", "e2e_chain"}
    assert "capture failed on some rank" in d["weak"]["timing"]
    assert d["weak"]["N_out_global"] == 8 * 256
    assert "injected capture failure (BENCH_INJECT_CAPTURE_FAIL) on rank 5" in r.stderr


def test_bench_rotation_touches_a_gib_at_driver_steps():
    """The driver runs `bench.py --steps 20`: every single-GPU config, the Q4_K_M layer and the
    row-sharded shards still cycle over >= 1 GiB of distinct weights (bench.rotation_plan: several
    20-step graphs replayed round robin), each graph exactly `steps` launches."""
    sys.path.insert(0, ROOT)
    import bench
    steps = 20
    for name, (fmt, M, K, N) in bench.CONFIGS.items():
        wbytes, _, _ = bench.model(fmt, M, K, N)
        ncopies, plans = bench.rotation_plan(wbytes, steps)
        assert all(len(p) == steps for p in plans), name
        assert bench.rotated_bytes(wbytes, plans) >= 1 << 30, name
        assert len({c for p in plans for c in p}) == ncopies, name
    layer_bytes = 129785856
    _, plans = bench.rotation_plan(layer_bytes, steps)
    assert bench.rotated_bytes(layer_bytes, plans) >= 1 << 30
    for world in (1, 2, 4, 8):  # the strong-scaling shard per rank
        rb = 8192 // 256 * 210
        rows = -(-28672 // world)
        _, plans = bench.rotation_plan(rows * rb, steps)
        assert bench.rotated_bytes(rows * rb, plans) >= 1 << 30
    # and the Runner really takes its copies from the plan
    import inspect
    src = inspect.getsource(bench.Runner.__init__)
    assert "rotation_plan(self.wbytes, steps)" in src
