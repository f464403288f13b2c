"""Row-sharded MMQ: split a packed GGUF weight matrix by rows over the ranks of a process
group, run the local MMQ, all-gather the fp16 output shards.

A packed row is a whole number of blocks, so any row boundary is a block boundary and a
shard is a zero-copy byte range of the packed tensor: rank g owns rows [g*R, g*R + R) with
R = ceil(M / world) rounded up to `align` (the last shard may be short or empty).  The
activations are replicated.  Each rank writes its (N, R) output into a padded slab and one
all_gather_into_tensor (backend "nccl" = RCCL on ROCm; "gloo" in the CPU tests) collects
(world, N, R); the (N, M) result is that slab viewed with the rank axis moved inside each
token row -- for N = 1 (decode) a free reshape, otherwise one device copy kernel
(gq_assemble_shards, the C ABI's form of this step; gq_mmq_sharded is the whole step in C).

There is no reference counterpart (the reference is single-GPU); this is the north_star's
"N partitioned across up to 8 GPUs of one node with RCCL all-gather".
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

BLOCK = {"q8_0": (32, 34), "q4_k": (256, 144), "q6_k": (256, 210)}


def shard_rows(M: int, world: int, rank: int, align: int = 64):
    """(row0, rows, R): this rank's first row, its real row count, and the padded shard size."""
    R = -(-M // world)
    R = -(-R // align) * align
    row0 = min(M, rank * R)
    rows = max(0, min(M, row0 + R) - row0)
    return row0, rows, R


def shard_bytes(fmt: str, A: torch.Tensor, M: int, K: int, world: int, rank: int, align: int = 64):
    """Byte range of the packed tensor A (flat, M rows) that rank `rank` owns (a view)."""
    qk, nbytes = BLOCK[fmt]
    row_bytes = (K // qk) * nbytes
    row0, rows, _ = shard_rows(M, world, rank, align)
    return A.view(-1)[row0 * row_bytes:(row0 + rows) * row_bytes]


def _default_compute(fmt: str):
    from kernels._lib import TYPES, mmq

    def run(A_shard, B, rows, N, K, out):
        return mmq(TYPES[fmt], A_shard, B, rows, N, K, out=out)

    return run


class RowShardedMMQ:
    """y = (A @ B^T)^T with A's rows spread over the group.

    A_shard: this rank's packed rows (from shard_bytes), on this rank's device.
    compute(A_shard, B, rows, N, K, out) -> writes fp16 (N, rows) into `out`
    (default: the HIP MMQ through the C ABI).
    world / rank: override the process group's (a shard of a G-way split driven outside a
    group, e.g. all G shards on one device in a test); gather() needs the real group.
    """

    def __init__(self, fmt: str, A_shard: torch.Tensor, M: int, K: int, group=None, align: int = 64,
                 compute: Optional[Callable] = None, world: Optional[int] = None, rank: Optional[int] = None):
        self.fmt, self.M, self.K, self.group = fmt, M, K, group
        self.world = world if world is not None else (dist.get_world_size(group) if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist.is_initialized() else 0)
        self.row0, self.rows, self.R = shard_rows(M, self.world, self.rank, align)
        qk, nbytes = BLOCK[fmt]
        assert A_shard.numel() == self.rows * (K // qk) * nbytes, "A_shard is not this rank's row range"
        self.A = A_shard
        self.compute = compute or _default_compute(fmt)

    def local(self, B: torch.Tensor, N: int, slab: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Run the local MMQ into a padded (N, R) slab (pad columns zeroed)."""
        if slab is None:
            slab = torch.empty(N, self.R, dtype=torch.float16, device=B.device)
        if self.rows < self.R:
            slab[:, self.rows:].zero_()
        if self.rows > 0 and N > 0:
            self.compute(self.A, B, self.rows, N, self.K, slab[:, :self.rows])
        return slab

    def gather(self, slab: torch.Tensor, out: Optional[torch.Tensor] = None, async_op: bool = False):
        """all_gather the (N, R) slabs into (world, N, R); returns (tensor, work)."""
        N = slab.shape[0]
        if out is None:
            out = torch.empty(self.world, N, self.R, dtype=slab.dtype, device=slab.device)
        if not dist.is_initialized():
            if self.world != 1:
                raise RuntimeError("gather() needs an initialised process group for world > 1")
            out[0].copy_(slab)
            return out, None
        # concatenated (world*N, R) form: accepted by both RCCL and gloo
        work = dist.all_gather_into_tensor(out.view(self.world * N, self.R), slab, group=self.group,
                                           async_op=async_op)
        return out, work

    def assemble(self, gathered: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """(world, N, R) -> (N, M): a free view at N = 1; otherwise on a ROCm device the C ABI's
        gq_assemble_shards kernel (into `out` when given), on the CPU (gloo tests) a permute."""
        W, N, R = gathered.shape
        if N == 1 and out is None:
            return gathered.view(1, W * R)[:, :self.M]
        if gathered.is_cuda:
            from kernels._lib import assemble_shards
            return assemble_shards(gathered, self.M, out=out)
        C = gathered.permute(1, 0, 2).reshape(N, W * R)[:, :self.M]
        if out is not None:
            out.copy_(C)
            return out
        return C

    def __call__(self, B: torch.Tensor, N: int, chunks: int = 1) -> torch.Tensor:
        if chunks > 1:
            return self.pipelined(B, N, chunks)
        slab = self.local(B, N)
        gathered, _ = self.gather(slab)
        return self.assemble(gathered)

    def pipelined(self, B: torch.Tensor, N: int, chunks: int) -> torch.Tensor:
        """The step in `chunks` row chunks of the shard (pipeline the all-gather):
        chunk c's local MMQ, then its all_gather issued asynchronously (on a GPU it runs on the
        collective's stream under chunk c+1's compute), each gathered chunk placed into its
        column range of every rank's part.  Values: at decode sizes (1..4 tokens) and on the
        skinny route bit-identical to one un-chunked step (a row's arithmetic depends on K and the
        token count only); on the GEMM routes (LDS-DMA, weight-register, resident / streaming
        split-K) the split-K factor -- and the route itself -- follow the chunk's row count, so a
        chunk sums K in another order: equal within the GEMM tolerance, bit-identical only with
        split-K pinned (GQ_GEMM_SPLITS=1 GQ_RGEMM=0, as the GPU tests do)."""
        if not dist.is_initialized() and self.world != 1:
            raise RuntimeError("pipelined() needs an initialised process group for world > 1")
        qk, nbytes = BLOCK[self.fmt]
        rb = (self.K // qk) * nbytes
        Rc = -(-self.R // chunks)
        dev = B.device
        out = torch.empty(N, self.world * self.R, dtype=torch.float16, device=dev)
        parts = []
        for c0 in range(0, self.R, Rc):
            w = min(Rc, self.R - c0)
            n = max(0, min(self.rows - c0, w))
            slab = torch.zeros(N, w, dtype=torch.float16, device=dev)
            if n > 0 and N > 0:
                self.compute(self.A[c0 * rb:(c0 + n) * rb], B, n, N, self.K, slab[:, :n])
            g = torch.empty(self.world, N, w, dtype=torch.float16, device=dev)
            if dist.is_initialized():
                work = dist.all_gather_into_tensor(g.view(self.world * N, w), slab, group=self.group, async_op=True)
            else:
                g[0].copy_(slab)
                work = None
            parts.append((c0, w, g, work))
        view = out.view(N, self.world, self.R)
        for c0, w, g, work in parts:
            if work is not None:
                work.wait()
            view[:, :, c0:c0 + w].copy_(g.permute(1, 0, 2))
        return out[:, :self.M]
