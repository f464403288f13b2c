"""Q8_0-Q8_1 CPU MMQ -- drop-in for the reference's kernels/cpu_impls/mmq_q8_0_q8_1_cpu.py:5.

C = (A @ B.T).T with A packed Q8_0 (34 B per 32 weights, M rows), B packed q8_1 (N rows);
returns the (N, M) transposed view of an (M, N) fp16 tensor, equal bit for bit to the
reference's Python loops (fp16 running sum in block order).
"""
import torch

from ._cpu import cpu_mmq


def mmq_q8_0_q8_1_cpu(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int):
    assert K % 32 == 0
    assert A.dtype == torch.int8
    assert B.dtype == torch.int8
    assert A.numel() == M * K / 32 * 34
    assert B.numel() == N * K / 32 * 36
    return cpu_mmq(0, A, B, M, N, K)
