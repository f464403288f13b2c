"""GPU parity of the fp8 activation variant (GQ_ACT_FP8_E4M3, BASELINE.json configs[4]; the
reference has no fp8 code).  Checked against oracle/oracle.py's fp8 checker:

  * the device quantizer (gq_quantize_fp8) bit for bit: e4m3fn codes (in the (0,2,1,3) group
    order) and the power-of-two block scales; the MMQ path widens the same codes to fp16 x~
    (act_quant F8DEQ: code * 2^e, exact) for the fp16-activation kernels;
  * the MMQ against mmq_fp8_ideal (fp32 dequantized weights x the same e4m3 activations,
    float64 sum): max|d| <= TIGHT_FP8 * max|C|, the fp16-MFMA bound of the q8_1 path (weights
    rounded to fp16 in registers);
  * the stated fp8 bound against the fp32-dequant reference with UNquantized activations
    (SURVEY 8(c)): max|d| <= FP8_BOUND * max|C| -- e4m3 keeps 3 mantissa bits, so each
    activation carries up to 2^-4 relative rounding error (the q8_1 path is ~10x tighter).
"""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT_FP8 = 4e-3
FP8_BOUND = 0.06


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def test_device_fp8_quantizer_bit_exact():
    import kernels._lib as kl
    rng = np.random.default_rng(3)
    rows, K = 37, 512
    x = (rng.standard_normal((rows, K)) * np.exp(rng.uniform(-14, 8, (rows, 1)))).astype(np.float16)
    x[0, :32] = 0                      # all-zero block
    x[1, 32:64] = np.float16(6.1e-5)   # constant block at the fp16 normal floor
    x[2, :] = np.float16(-0.0)
    x[3, 64:96] = rng.standard_normal(32).astype(np.float16) * np.float16(2.0 ** -20)  # fp16 subnormals
    x[4, :32] = np.float16(60000.0)
    codes, scales = kl.quantize_fp8_device(torch.from_numpy(x).to(_dev()))
    want_c, want_X = O.quantize_fp8(x)
    got_c = codes.cpu().numpy()
    assert np.array_equal(got_c, O.fp8_permuted(want_c))
    got_X = scales.cpu().numpy()[:, :rows].T
    assert np.array_equal(got_X, want_X)


@pytest.mark.parametrize("fmt", ("q8_0", "q4_k", "q6_k"))
@pytest.mark.parametrize("M,N,K", [(96, 1, 256), (130, 5, 512), (200, 64, 1024), (257, 128, 2048), (64, 300, 768),
                                   (300, 77, 4096), (520, 2, 4096), (129, 3, 768), (1000, 4, 2048), (333, 16, 1024),
                                   (77, 800, 512)])
def test_fp8_mmq(fmt, M, N, K):
    """Every route of the fp8 variant's x~ (act_quant F8DEQ): the skinny kernel from one token
    (Q4_K, Q8_0), the LDS-DMA and weight-register GEMMs, dequant + hipBLASLt (800 tokens)."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + N)
    B = random_activations(N, K, seed=K - N)
    C = mmq(TYPES[fmt], torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev), M, N, K,
            act="fp8")
    torch.cuda.synchronize()
    got = C.cpu().numpy()
    ideal = O.mmq_fp8_ideal(fmt, qA, B, M, N, K)
    assert O.max_rel_err(got, ideal) <= TIGHT_FP8, O.max_rel_err(got, ideal)
    ref = O.mmq_fp32_dequant(fmt, qA, B, M, N, K)
    assert O.max_rel_err(got, ref) <= FP8_BOUND, O.max_rel_err(got, ref)


def test_fp8_prepared_and_splits(tune):
    import kernels._lib as kl
    dev = _dev()
    M, N, K = 384, 96, 2048
    for fmt in ("q4_k", "q6_k"):
        qA = random_blocks(fmt, M, K, seed=5)
        B = random_activations(N, K, seed=6)
        A_t, B_t = torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev)
        g = kl.TYPES[fmt]
        ws = torch.empty(kl.workspace_size(g, M, N, K, "fp8"), dtype=torch.uint8, device=dev)
        kl.act_prepare(B_t, N, K, ws, act="fp8")
        outs = []
        for splits in ("1", "4"):
            tune(GQ_GEMM_SPLITS=splits)
            outs.append(kl.mmq_prepared(g, A_t, ws, M, N, K, act="fp8").cpu().numpy())
        ideal = O.mmq_fp8_ideal(fmt, qA, B, M, N, K)
        for o in outs:
            assert O.max_rel_err(o, ideal) <= TIGHT_FP8


def test_fp8_rejects_k_not_multiple_of_256():
    from kernels._lib import TYPES, mmq
    dev = _dev()
    qA = random_blocks("q8_0", 8, 96, seed=1)
    with pytest.raises(RuntimeError):
        mmq(TYPES["q8_0"], torch.from_numpy(qA.view(np.int8)).to(dev),
            torch.from_numpy(random_activations(4, 96)).to(dev), 8, 4, 96, act="fp8")


def test_layer_mix_fp8():
    """The Q4_K_M layer mix with fp8 activations (configs[4]'s variant)."""
    from gguf import q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    shapes = {n: (96, 512) for g in LayerMix.GROUPS[:3] for n in g}
    shapes["ffn_down"] = (64, 768)
    raw = {n: random_blocks(types[n], *shapes[n], seed=i) for i, n in enumerate(shapes)}
    layer = LayerMix({n: GGUFLinear(types[n], torch.from_numpy(raw[n].view(np.int8)).to(dev), *shapes[n])
                      for n in shapes}, act="fp8")
    for N in (1, 20):
        x = random_activations(N, 512, seed=N)
        h = random_activations(N, 768, seed=N + 1)
        out = layer.forward(torch.from_numpy(x).to(dev), torch.from_numpy(h).to(dev))
        torch.cuda.synchronize()
        for n, (M, K) in shapes.items():
            ideal = O.mmq_fp8_ideal(types[n], raw[n], x if K == 512 else h, M, N, K)
            assert O.max_rel_err(out[n].cpu().numpy(), ideal) <= TIGHT_FP8, (n, N)


@pytest.mark.parametrize("fmt,M,K", [("q4_k", 4096, 4096), ("q8_0", 2048, 4096), ("q4_k", 1024, 8192),
                                     ("q8_0", 512, 8192), ("q6_k", 4096, 4096), ("q6_k", 1024, 8192),
                                     ("q4_k", 300, 12288)])
def test_fp8_decode_register_cache_bit_identical(fmt, M, K, tune):
    """The fp8 decode form at one token with the lane's x~ kept in registers across its rows
    (GQ_DECODE_F8_ITC=1, the default: one or two units per lane, Q6_K one half super-block pair;
    image and packed Q6_K rings) = the per-row LDS reads (=0), bit for bit; alone and grouped;
    and within the fp8 gate of the fp8-exact product."""
    import kernels._lib as kl
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + K)
    B = random_activations(1, K, seed=K)
    A_t, B_t = torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev)
    got = {}
    for itc in (1, 0):
        tune(GQ_DECODE_F8_ITC=itc)
        C = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, 1, K, act="fp8")
        G = kl.mmq_grouped([(kl.TYPES[fmt], A_t, B_t, M, K, None)], 1, act="fp8")
        assert G is not None, kl.lib().gq_last_error()
        torch.cuda.synchronize()
        got[itc] = (C.view(torch.int16).clone(), G[0].view(torch.int16).clone())
    assert torch.equal(got[1][0], got[0][0])
    assert torch.equal(got[1][1], got[0][1])
    assert torch.equal(got[1][0], got[1][1])
    ideal = O.mmq_fp8_ideal(fmt, qA, B, M, 1, K)
    assert O.max_rel_err(got[1][0].view(torch.float16).cpu().numpy(), ideal) <= TIGHT_FP8
