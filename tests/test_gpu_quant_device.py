"""On-device GGUF weight quantization (gq_quantize_weights): the device
producers run the host producers' exact code, so their bytes equal the reference's own
quantizer outputs (tests/golden/golden_quant.npz, produced by the reference's utils/quantize)
and the host library's (utils.quantize, byte-exact to the reference) on large random inputs."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden", "golden_quant.npz")
FMTS = ("q8_0", "q4_k", "q6_k")


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _device_bytes(fmt, x):
    import kernels._lib as kl
    X = torch.from_numpy(np.ascontiguousarray(x)).to(_dev())
    X = X.to(torch.float16 if fmt == "q8_0" else torch.float32)
    y = kl.quantize_weights_device(fmt, X)
    torch.cuda.synchronize()
    return y.cpu().numpy().view(np.uint8)


@pytest.mark.parametrize("fmt", FMTS)
def test_device_quantizer_matches_reference_bytes(fmt):
    z = np.load(GOLD)
    names = sorted({k[:-2] for k in z.files if k.endswith("_x")})
    assert len(names) >= 8
    for name in names:
        assert np.array_equal(_device_bytes(fmt, z[name + "_x"]), z[f"{name}_{fmt}"]), (fmt, name)


@pytest.mark.parametrize("fmt", FMTS)
def test_device_quantizer_matches_host_large(fmt):
    """1024 x 4096 weights whose rows span 2^-20 .. 2^6 in scale, with zero rows, zero blocks,
    fp16 subnormals and sign-heavy rows: device bytes == host bytes."""
    from utils.quantize import _qlib
    rng = np.random.default_rng(11)
    x = rng.standard_normal((1024, 4096)).astype(np.float32) * np.exp2(rng.uniform(-20, 6, (1024, 1))).astype(np.float32)
    x[3] = 0
    x[5, :256] = 0
    x[7] = np.abs(x[7])
    x[9, :64] = np.float32(2.0 ** -20)
    x = x.astype(np.float16)  # the reference's inputs are fp16 weights
    want = _qlib.quantize(fmt, torch.from_numpy(x)).numpy().view(np.uint8)
    assert np.array_equal(_device_bytes(fmt, x), want)


def test_device_quantizer_errors():
    import kernels._lib as kl
    with pytest.raises(RuntimeError):
        kl.quantize_weights_device("q4_k", torch.zeros(100, dtype=torch.float32, device=_dev()))
    with pytest.raises(RuntimeError):
        kl.quantize_weights_device("q8_0", torch.zeros(64, dtype=torch.float32, device=_dev()))
    L = kl.lib()
    assert L.gq_quantize_weights(kl.GQ_Q8_0, None, None, 31, None) != 0
