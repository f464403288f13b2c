"""Q6_K x fp16 MMQ -- drop-in for the reference's kernels/mmq_q6_k.py:197 `mmq_q6_k`.

A: packed Q6_K super-blocks (210 B per 256 weights: ql[128], qh[64], int8 scales[16],
fp16 d) as a flat int8 device tensor of M*K/256*210 bytes; B: fp16 (N, K); returns
fp16 (N, M) = (A @ B^T)^T.  Runs in libgguf_mmq.so.
"""
import torch

from ._lib import GQ_Q6_K, mmq

QK_K = 256
Q6_K_SUBBLK_NUM = 16
QK8_1 = 32
Q6_K_BLOCK_SIZE = 210  # bytes
Q8_1_BLOCK_SIZE = 36  # bytes


def mmq_q6_k(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """out = (A @ B.T).T with A in Q6_K (M rows), B fp16 (N, K); fp16 (N, M)."""
    assert (K % 256 == 0)
    return mmq(GQ_Q6_K, A, B, M, N, K)
