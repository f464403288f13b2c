"""The fp8 variant's CPU checker (oracle/oracle.py e4m3_encode / quantize_fp8) pinned against
the OCP e4m3fn definition itself: every finite code value encodes to itself, midpoints round
to even, and the per-block scale meets its definition.  CPU only."""
import numpy as np

import oracle as O


def test_every_code_roundtrips():
    codes = np.array([c for c in range(256) if c & 0x7F != 0x7F], np.uint8)  # all but NaN
    vals = O.e4m3_decode(codes)
    enc = O.e4m3_encode(vals)
    # +0 / -0 keep their sign bit; every other code maps to itself
    assert np.array_equal(enc, codes)
    assert O.e4m3_decode(np.uint8(0x7E)) == 448.0 and O.e4m3_decode(np.uint8(1)) == 2.0 ** -9


def test_midpoints_round_to_even():
    pos = np.arange(0, 0x7E, dtype=np.uint8)
    lo, hi = O.e4m3_decode(pos), O.e4m3_decode(pos + 1)
    mid = ((lo.astype(np.float64) + hi) / 2).astype(np.float32)
    enc = O.e4m3_encode(mid)
    even = np.where(pos % 2 == 0, pos, pos + 1).astype(np.uint8)
    assert np.array_equal(enc, even)


def test_block_scale_definition():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((7, 256)) * np.exp(rng.uniform(-12, 9, (7, 1)))).astype(np.float16)
    x[0, :32] = 0
    codes, X = O.quantize_fp8(x)
    amax = np.abs(x.astype(np.float32)).reshape(7, 8, 32).max(axis=2)
    assert np.all(X[amax == 0] == 1.0)
    nz = amax > 0
    assert np.all(amax[nz] <= 448 * X[nz]) and np.all(amax[nz] > 224 * X[nz])
    dec = O.e4m3_decode(codes).reshape(7, 8, 32) * X[:, :, None]
    err = np.abs(dec - x.astype(np.float32).reshape(7, 8, 32)).max(axis=2)
    assert np.all(err <= amax * 2.0 ** -4 + 2.0 ** -9 * X)
