"""ctypes loader for libgguf_quant.so (include/gguf_quant.h)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "lib",
                         "libgguf_quant.so")
_lib = None
_P, _I64 = ctypes.c_void_p, ctypes.c_int64

BLOCK = {"q8_0": (32, 34), "q8_1": (32, 36), "q4_k": (256, 144), "q6_k": (256, 210)}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} not found: run `make -C gguf-triton-kernel_amd`")
        h = ctypes.CDLL(_LIB_PATH)
        for fmt in BLOCK:
            q = getattr(h, f"gq_quantize_{fmt}")
            q.argtypes, q.restype = [_P, _P, _I64], None
            d = getattr(h, f"gq_dequantize_{fmt}")
            d.argtypes, d.restype = [_P, _P, _I64], None
        _lib = h
    return _lib


def quantize(fmt: str, x: torch.Tensor) -> torch.Tensor:
    """Host quantization of any-shape x (numel % QK == 0) -> flat int8 CPU tensor."""
    qk, nbytes = BLOCK[fmt]
    if fmt in ("q4_k", "q6_k"):
        arr = np.ascontiguousarray(x.detach().cpu().to(torch.float32).numpy().reshape(-1))
    else:
        arr = np.ascontiguousarray(x.detach().cpu().to(torch.float16).numpy().reshape(-1)).view(np.uint16)
    n = arr.size
    if n % qk != 0:
        if qk == 32:
            raise ValueError("The total number of elements must be divisible by 32.")
        raise ValueError(f"Array length must be multiple of {qk} (got {n})")
    out = np.empty(n // qk * nbytes, dtype=np.uint8)
    getattr(lib(), f"gq_quantize_{fmt}")(arr.ctypes.data_as(_P), out.ctypes.data_as(_P), n)
    return torch.from_numpy(out.view(np.int8))


def dequantize(fmt: str, q: torch.Tensor) -> torch.Tensor:
    """Flat packed bytes -> flat fp32 CPU tensor."""
    qk, nbytes = BLOCK[fmt]
    arr = np.ascontiguousarray(q.detach().cpu().numpy().reshape(-1)).view(np.uint8)
    if arr.size % nbytes != 0:
        raise ValueError(f"Invalid quantized tensor size. Expected size divisible by {nbytes}, got {arr.size}.")
    nb = arr.size // nbytes
    out = np.empty(nb * qk, dtype=np.float32)
    getattr(lib(), f"gq_dequantize_{fmt}")(arr.ctypes.data_as(_P), out.ctypes.data_as(_P), nb)
    return torch.from_numpy(out)
