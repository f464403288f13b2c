"""Row-sharded MMQ across 2 processes (gloo, CPU): shard boundaries, the all-gather and the
(world, N, R) -> (N, M) assembly.  The per-shard compute here is the oracle (test
infrastructure); on GPUs the same class calls the HIP MMQ (tests/test_gpu_parity.py)."""
import os
import sys
import tempfile

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


def _worker(rank, world, initfile, fmt, M, N, K, align, q):
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
        C = op(B, N)
        if rank == 0:
            q.put(C.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt,M,N,K,align", [("q4_k", 200, 3, 512, 64), ("q8_0", 130, 1, 96, 16),
                                             ("q6_k", 64, 5, 256, 64), ("q4_k", 40, 2, 256, 64)])
def test_row_sharded_matches_single(fmt, M, N, K, align):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from utils.synth import random_activations, random_blocks
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        initfile = os.path.join(d, "init")
        ps = [ctx.Process(target=_worker, args=(r, world, initfile, fmt, M, N, K, align, q)) for r in range(world)]
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
