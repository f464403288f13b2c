"""Synthetic packed GGUF weights for benchmarks and size-independent parity tests.

Random bytes are valid blocks for every format except where a byte pair is an fp16 scale,
so those fields are overwritten with fp16(U(0.5, 1.5) * 2^-7); Q6_K's
int8 sub-block scales stay uniformly random (including negative ones).  The kernels have
no data-dependent control flow, so timings do not depend on the values.
"""
from __future__ import annotations

import numpy as np

BLOCK = {"q8_0": (32, 34), "q4_k": (256, 144), "q6_k": (256, 210)}


def _scales(rng, n):
    return (rng.uniform(0.5, 1.5, size=n) * 2.0 ** -7).astype(np.float16).view(np.uint16)


def random_blocks(fmt: str, M: int, K: int, seed: int = 0) -> np.ndarray:
    """uint8 array of M rows of packed `fmt` blocks covering K elements each."""
    qk, nbytes = BLOCK[fmt]
    assert K % qk == 0
    nb = M * (K // qk)
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256, size=(nb, nbytes), dtype=np.uint8)
    u16 = raw.view(np.uint8)
    if fmt == "q8_0":
        d = _scales(rng, nb)
        u16[:, 0] = d & 0xFF
        u16[:, 1] = d >> 8
    elif fmt == "q4_k":
        d, dm = _scales(rng, nb), _scales(rng, nb)
        u16[:, 0], u16[:, 1] = d & 0xFF, d >> 8
        u16[:, 2], u16[:, 3] = dm & 0xFF, dm >> 8
    else:
        d = _scales(rng, nb)
        u16[:, 208], u16[:, 209] = d & 0xFF, d >> 8
    return raw.reshape(-1)


def random_activations(N: int, K: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed + 12345)
    return rng.standard_normal((N, K), dtype=np.float32).astype(np.float16)
