"""Q4_K-Q8_1 CPU MMQ -- drop-in for the reference's kernels/cpu_impls/mmq_q4_k_q8_1_cpu.py:61.

C = (A @ B.T).T with A packed Q4_K (144 B per 256 weights, M rows), B packed q8_1 (N rows);
returns the (N, M) transposed view of an (M, N) fp16 tensor, equal bit for bit to the
reference's Python loops (fp16 running sum in block order).
"""
import torch

from ._cpu import cpu_mmq


def mmq_q4_k_q8_1_cpu(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int):
    assert K % 256 == 0
    assert A.dtype == torch.int8
    assert B.dtype == torch.int8
    assert A.numel() == M * K / 256 * 144
    assert B.numel() == N * K / 32 * 36
    return cpu_mmq(1, A, B, M, N, K)
