"""Q8_0 x fp16 MMQ -- drop-in for the reference's kernels/mmq_q8_0.py:102 `mmq_q8_0`.

A: packed Q8_0 blocks (34 B per 32 weights: fp16 d, int8 qs[32]) as a flat int8 device
tensor of M*K/32*34 bytes; B: fp16 (N, K) device tensor; returns fp16 (N, M) =
(A @ B^T)^T.  The activations are quantized to q8_1 on the device exactly as
utils/quantize/q8_1.py does, then multiplied block by block as kernels/cpu_impls does;
the work runs in libgguf_mmq.so (HIP, gfx950).
"""
import torch

from ._lib import GQ_Q8_0, mmq

QK8_0 = 32
QK8_1 = 32
Q8_0_SIZE = 34  # bytes


def mmq_q8_0(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """out = (A @ B.T).T with A in Q8_0 (M rows), B fp16 (N, K); fp16 (N, M)."""
    assert (K % 32 == 0)
    return mmq(GQ_Q8_0, A, B, M, N, K)
