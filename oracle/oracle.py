"""oracle/oracle.py -- numpy/ctypes front end of the CPU checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product (gguf-triton-kernel_amd/) never imports it.

It wraps oracle/mmq_oracle.c, a C restatement of the reference's parity oracle
(kernels/cpu_impls/mmq_{q8_0,q4_k,q6_k}_q8_1_cpu.py) and of its 8-bit quantizers
(utils/quantize/q8_0.py:4-49, utils/quantize/q8_1.py:18-70).  The restatement is pinned
bit-exact against fixtures produced by running the reference itself
(tests/golden/make_golden.py -> tests/golden/*.npz; see tests/test_oracle_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

EXACT = 0  # the reference's own arithmetic: fp16 running sum in block order
IDEAL = 1  # same quantized inputs, exact products, one final rounding

BLOCK_BYTES = {"q8_0": 34, "q4_k": 144, "q6_k": 210, "q8_1": 36}
BLOCK_ELEMS = {"q8_0": 32, "q4_k": 256, "q6_k": 256, "q8_1": 32}


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        src = os.path.join(HERE, "mmq_oracle.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", HERE])
        lib = ctypes.CDLL(path)
        p = ctypes.c_void_p
        i64 = ctypes.c_int64
        for name in ("oracle_quantize_q8_1", "oracle_quantize_q8_0"):
            getattr(lib, name).argtypes = [p, i64, p]
            getattr(lib, name).restype = None
        for fmt in ("q8_0", "q4_k", "q6_k"):
            f = getattr(lib, f"oracle_mmq_{fmt}_q8_1")
            f.argtypes = [p, p, i64, i64, i64, p, ctypes.c_int]
            f.restype = None
        for fmt in ("q8_0", "q8_1", "q4_k", "q6_k"):
            f = getattr(lib, f"oracle_dequant_{fmt}")
            f.argtypes = [p, i64, p]
            f.restype = None
        _LIB = lib
    return _LIB


def _u16(x) -> np.ndarray:
    x = np.ascontiguousarray(x)
    if x.dtype == np.float16:
        x = x.view(np.uint16)
    assert x.dtype == np.uint16, x.dtype
    return x


def _u8(x) -> np.ndarray:
    x = np.ascontiguousarray(x)
    if x.dtype == np.int8:
        x = x.view(np.uint8)
    assert x.dtype == np.uint8, x.dtype
    return x


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def quantize_q8_1(x_f16) -> np.ndarray:
    """fp16 array (any shape, numel % 32 == 0) -> uint8 q8_1 bytes (q8_1.py:18-70)."""
    x = _u16(x_f16).reshape(-1)
    assert x.size % 32 == 0
    out = np.empty(x.size // 32 * 36, np.uint8)
    _lib().oracle_quantize_q8_1(_ptr(x), x.size, _ptr(out))
    return out


def quantize_q8_0(x_f16) -> np.ndarray:
    """fp16 array -> uint8 q8_0 bytes (q8_0.py:4-49)."""
    x = _u16(x_f16).reshape(-1)
    assert x.size % 32 == 0
    out = np.empty(x.size // 32 * 34, np.uint8)
    _lib().oracle_quantize_q8_0(_ptr(x), x.size, _ptr(out))
    return out


def mmq(fmt: str, A, Bq, M: int, N: int, K: int, mode: int = EXACT) -> np.ndarray:
    """C = (A @ B^T)^T with A packed `fmt`, B packed q8_1 -> fp16 (N, M).

    Restates kernels/cpu_impls/mmq_{fmt}_q8_1_cpu.py (see mmq_oracle.c for lines).
    """
    A = _u8(A).reshape(-1)
    Bq = _u8(Bq).reshape(-1)
    qk = BLOCK_ELEMS[fmt]
    assert K % qk == 0
    assert A.size == M * (K // qk) * BLOCK_BYTES[fmt], (A.size, M, K)
    assert Bq.size == N * (K // 32) * 36
    out = np.empty((N, M), np.uint16)
    getattr(_lib(), f"oracle_mmq_{fmt}_q8_1")(_ptr(A), _ptr(Bq), M, N, K, _ptr(out), mode)
    return out.view(np.float16)


def dequant(fmt: str, A) -> np.ndarray:
    """Packed bytes -> fp32 weights in row order (utils/quantize/*.py dequantize_*)."""
    A = _u8(A).reshape(-1)
    nb = A.size // BLOCK_BYTES[fmt]
    assert nb * BLOCK_BYTES[fmt] == A.size
    out = np.empty(nb * BLOCK_ELEMS[fmt], np.float32)
    getattr(_lib(), f"oracle_dequant_{fmt}")(_ptr(A), nb, _ptr(out))
    return out


def mmq_from_fp16(fmt: str, A, B_f16, M: int, N: int, K: int, mode: int = EXACT) -> np.ndarray:
    """What the reference's test does: quantize B with quantize_to_q8_1, run the oracle."""
    return mmq(fmt, A, quantize_q8_1(B_f16), M, N, K, mode)


def allclose(a, b, atol_ratio: float = 0.01) -> bool:
    """utils/test_utils.py:4-8 : torch.allclose(a, b, atol=atol_ratio*max|b|) (rtol 1e-5),
    False when max|b| is NaN."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    mb = np.max(np.abs(b)) if b.size else 0.0
    if np.isnan(mb):
        return False
    return bool(np.all(np.abs(a - b) <= atol_ratio * mb + 1e-5 * np.abs(b)) and not np.isnan(a).any())


def max_rel_err(a, b) -> float:
    """max|a-b| / max|b| in fp32 (0 when b is all zero and a == b)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    mb = float(np.max(np.abs(b))) if b.size else 0.0
    d = float(np.max(np.abs(a - b))) if b.size else 0.0
    return d / mb if mb > 0 else d
