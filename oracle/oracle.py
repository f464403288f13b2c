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


# ---- fp8 activation variant (BASELINE.json configs[4]; no reference counterpart) ----------
# The checker for GQ_ACT_FP8_E4M3 (include/gguf_mmq.h): per 32-element block X = 2^e with e the
# smallest integer such that max|x| <= 448 * 2^e (X = 1 for an all-zero block); codes = OCP
# e4m3fn(x / X) with round-to-nearest-even.  Restated from the OCP 8-bit floating point
# specification (e4m3fn: bias 7, no infinities, max normal 448 = 1.75 * 2^8, subnormal step 2^-9).

def e4m3_encode(v) -> np.ndarray:
    """float32 values with |v| <= 448 -> uint8 e4m3fn codes, round to nearest even."""
    v = np.asarray(v, np.float32)
    a = np.abs(v).astype(np.float64)
    sign = np.signbit(v).astype(np.uint8) << 7
    _, E = np.frexp(a)                             # a = m * 2^E, m in [0.5, 1)
    exp = np.maximum(E - 1, -6)                    # exponent of the leading bit, subnormal floor
    quantum = np.ldexp(1.0, exp - 3)               # 3 mantissa bits
    q = np.rint(a / quantum)                       # RNE (np.rint: half to even)
    val = q * quantum
    sub = val < 2.0 ** -6
    _, Ev = np.frexp(np.where(sub, 1.0, val))
    ev = Ev - 1
    m3 = np.rint((np.where(sub, 1.0, val) / np.ldexp(1.0, ev) - 1.0) * 8).astype(np.int64)
    bits = np.where(sub, q.astype(np.int64), ((ev + 7) << 3) | m3)
    assert np.all(bits <= 0x7E), "e4m3 overflow"
    return (bits.astype(np.uint8) | sign).astype(np.uint8)


def e4m3_decode(c) -> np.ndarray:
    """uint8 e4m3fn codes -> float32 (0x7F / 0xFF NaN codes are never produced here)."""
    c = np.asarray(c, np.uint8).astype(np.int64)
    s = np.where(c & 0x80, -1.0, 1.0)
    e = (c >> 3) & 0xF
    m = c & 7
    mag = np.where(e == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * np.ldexp(1.0, e - 7))
    return (s * mag).astype(np.float32)


def quantize_fp8(x_f16):
    """fp16 (rows, K) -> (codes uint8 (rows, K) in element order, X float32 (rows, K/32))."""
    x = np.asarray(x_f16, np.float16).astype(np.float32)
    rows, K = x.shape
    xb = x.reshape(rows, K // 32, 32)
    amax = np.abs(xb).max(axis=2)
    m, E = np.frexp(amax)
    e = np.where(amax == 0, 0, E - 9 + (m > 0.875))
    X = np.ldexp(np.float32(1.0), e).astype(np.float32)
    codes = e4m3_encode(xb / X[:, :, None]).reshape(rows, K)
    return codes, X


def fp8_permuted(codes) -> np.ndarray:
    """Element order -> the device layout: each 4-group stored (0,2,1,3)."""
    c = np.asarray(codes).reshape(-1, 4)
    return c[:, [0, 2, 1, 3]].reshape(np.asarray(codes).shape)


def mmq_fp8_ideal(fmt: str, A, B_f16, M: int, N: int, K: int) -> np.ndarray:
    """The fp8 variant's exact value: fp32 dequantized weights x e4m3-quantized activations,
    summed in float64, rounded once to fp16 -> (N, M)."""
    W = dequant(fmt, A).reshape(M, K).astype(np.float64)
    codes, X = quantize_fp8(B_f16)
    xt = (e4m3_decode(codes).reshape(N, K // 32, 32) * X[:, :, None]).reshape(N, K).astype(np.float64)
    return (xt @ W.T).astype(np.float16)


def mmq_fp32_dequant(fmt: str, A, B_f16, M: int, N: int, K: int) -> np.ndarray:
    """fp32-dequant reference with UNquantized activations -> (N, M) float32."""
    W = dequant(fmt, A).reshape(M, K).astype(np.float64)
    return (np.asarray(B_f16, np.float16).astype(np.float64) @ W.T).astype(np.float32)
