"""Shared body of the three cpu_impls functions (ctypes -> gq_cpu_mmq)."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from utils.quantize._qlib import lib as _qlib

_BYTES = {0: 34, 1: 144, 2: 210}
_QK = {0: 32, 1: 256, 2: 256}


def cpu_mmq(gtype: int, A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int, threads: int = 0) -> torch.Tensor:
    """(A @ B^T)^T with A packed (gtype), B packed q8_1 -> the (N, M) view of an (M, N) fp16
    tensor, as the reference returns `C.T`."""
    h = _qlib()
    fn = h.gq_cpu_mmq
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                   ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    a = np.ascontiguousarray(A.detach().cpu().numpy().reshape(-1)).view(np.uint8)
    b = np.ascontiguousarray(B.detach().cpu().numpy().reshape(-1)).view(np.uint8)
    C = torch.zeros((M, N), dtype=torch.float16)
    if M and N:
        rc = fn(gtype, a.ctypes.data, b.ctypes.data, M, N, K, C.data_ptr(), threads)
        if rc != 0:
            raise RuntimeError(f"gq_cpu_mmq failed (type {gtype}, K={K})")
    return C.T
