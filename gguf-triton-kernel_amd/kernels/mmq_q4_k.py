"""Q4_K x fp16 MMQ -- drop-in for the reference's kernels/mmq_q4_k.py:240 `mmq_q4_k`.

A: packed Q4_K super-blocks (144 B per 256 weights: fp16 d, fp16 dmin, 12 bytes of
6-bit scales/mins, 128 bytes of nibbles) as a flat int8 device tensor of M*K/256*144
bytes; B: fp16 (N, K); returns fp16 (N, M) = (A @ B^T)^T.  Runs in libgguf_mmq.so.
"""
import torch

from ._lib import GQ_Q4_K, mmq

Q4_K_BLOCK_SIZE = 144  # bytes
Q8_1_BLOCK_SIZE = 36  # bytes
Q4_K_SUBBLK_NUM = 8
QK_K = 256
QK8_1 = 32


def mmq_q4_k(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """out = (A @ B.T).T with A in Q4_K (M rows), B fp16 (N, K); fp16 (N, M)."""
    assert (K % 256 == 0)
    return mmq(GQ_Q4_K, A, B, M, N, K)
