"""Host block producers (utils/quantize/*, libgguf_quant.so) are byte-identical to the
reference's producers.  CPU only."""
import os

import numpy as np
import pytest
import torch

import oracle as O
from utils.quantize.q4_k import dequantize_q4_k, quantize_to_q4_k
from utils.quantize.q6_k import dequantize_q6_k, quantize_to_q6_k
from utils.quantize.q8_0 import dequantize_q8_0, quantize_to_q8_0
from utils.quantize.q8_1 import dequantize_q8_1, quantize_to_q8_1
from utils.test_utils import allclose

GOLD = os.path.join(os.path.dirname(__file__), "golden", "golden_quant.npz")
QUANT = {"q8_0": quantize_to_q8_0, "q8_1": quantize_to_q8_1, "q4_k": quantize_to_q4_k, "q6_k": quantize_to_q6_k}


@pytest.mark.parametrize("fmt", sorted(QUANT))
def test_quantizer_bytes_match_reference(fmt):
    z = np.load(GOLD)
    names = sorted({k[:-2] for k in z.files if k.endswith("_x")})
    assert len(names) >= 8
    for name in names:
        x = torch.from_numpy(z[name + "_x"])
        got = QUANT[fmt](x)
        assert got.dtype == torch.int8 and got.dim() == 1
        assert np.array_equal(got.numpy().view(np.uint8), z[f"{name}_{fmt}"]), (fmt, name)


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k", "q6_k"])
def test_quantizer_matches_matmul_fixtures(golden, fmt):
    """The packed A of every matmul fixture came from the reference quantizer; re-packing
    its dequantized values is not required, but q8_1 of every B must match."""
    for c in golden[fmt]:
        got = quantize_to_q8_1(torch.from_numpy(c["B"]))
        assert np.array_equal(got.numpy().view(np.uint8), c["qB"]), (fmt, c["i"])


@pytest.mark.parametrize("fmt,deq", [("q8_0", dequantize_q8_0), ("q8_1", dequantize_q8_1),
                                     ("q4_k", dequantize_q4_k), ("q6_k", dequantize_q6_k)])
def test_dequantize_matches_oracle(fmt, deq):
    z = np.load(GOLD)
    x = z["normal_x"]
    q = QUANT[fmt](torch.from_numpy(x))
    got = deq(q, x.shape)
    assert tuple(got.shape) == x.shape
    assert got.dtype == (torch.float32 if fmt == "q6_k" else torch.float16)
    want = O.dequant(fmt, q.numpy()).reshape(x.shape)
    if fmt != "q6_k":
        want = want.astype(np.float16)
    assert np.array_equal(got.numpy(), want)
    # and the round trip is a faithful quantization
    assert allclose(got.float(), torch.from_numpy(x).float(), 0.1)


def test_quantizer_errors():
    with pytest.raises(ValueError):
        quantize_to_q8_0(torch.zeros(33))
    with pytest.raises(ValueError):
        quantize_to_q8_1(torch.zeros(31))
    with pytest.raises(ValueError):
        quantize_to_q4_k(torch.zeros(255))
    with pytest.raises(ValueError):
        quantize_to_q6_k(torch.zeros(100))


def test_quantizer_threads_deterministic():
    """Large inputs are split over threads by whole blocks; result independent of that."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1024, 1024, generator=g).to(torch.float16)
    a = quantize_to_q4_k(x)
    b = torch.cat([quantize_to_q4_k(x[i:i + 128]) for i in range(0, 1024, 128)])
    assert torch.equal(a, b)
    a = quantize_to_q6_k(x)
    b = torch.cat([quantize_to_q6_k(x[i:i + 128]) for i in range(0, 1024, 128)])
    assert torch.equal(a, b)
