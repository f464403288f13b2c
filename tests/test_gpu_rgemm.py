"""GPU parity of the resident-split GEMM (csrc/mmq_rgemm.hip: 256 rows x <= 128 tokens x one
super-block per workgroup, split-K over every super-block, fp16 partials + gemm_kernel's reduce).
Every format and token tile (16/32/64/128 tokens: NB 1/2/4/8), ragged rows and tokens, one to 16
super-blocks; the in-kernel activation quantization (gq_mmq: q8_1 and the fp8 variant) against
the prepared x~ (gq_act_prepare + gq_mmq_prepared) bit for bit; at K = 256 (no split) bit for
bit against gemm_kernel (same dequantization, same MFMA sequence); the headline shape at full
size on sampled rows.  Tolerance: TIGHT (fp16 W x fp16 x~, fp32 MFMA accumulation, fp16
partials) vs the oracle's IDEAL mode, and the reference's 1% gate vs EXACT."""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT = 4e-3
FMTS = ("q8_0", "q4_k", "q6_k")


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(_dev())


def _mmq(fmt, qA, B, M, N, K, act="q8_1"):
    import kernels._lib as kl
    C = kl.mmq(kl.TYPES[fmt], qA, B, M, N, K, act=act)
    torch.cuda.synchronize()
    return C


def _prepared(fmt, qA, B, M, N, K, act="q8_1"):
    import kernels._lib as kl
    t = kl.TYPES[fmt]
    ws = torch.empty(kl.workspace_size(t, M, N, K, act), dtype=torch.uint8, device=_dev())
    kl.act_prepare(B, N, K, ws, act=act)
    C = kl.mmq_prepared(t, qA, ws, M, N, K, act=act)
    torch.cuda.synchronize()
    return C


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("M,N,K", [(256, 128, 256), (300, 100, 1024), (1000, 40, 512), (513, 20, 768),
                                   (64, 16, 4096), (256, 128, 4096), (700, 33, 2048)])
def test_rgemm_parity(fmt, M, N, K, tune):
    tune(GQ_RGEMM=1, GQ_SKINNY=0, GQ_KSTREAM=0)
    qA = random_blocks(fmt, M, K, seed=M + N + K)
    B = random_activations(N, K, seed=3 * K + N)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    C = _mmq(fmt, A_t, B_t, M, N, K)
    got = C.cpu().numpy()
    assert np.isfinite(got.astype(np.float32)).all()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT, O.max_rel_err(got, ideal)
    exact = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)
    # the prepared form reads the act_quant x~ the kernel formed itself: same bits
    Cp = _prepared(fmt, A_t, B_t, M, N, K)
    assert torch.equal(Cp.view(torch.int16), C.view(torch.int16))


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("M,N", [(256, 128), (400, 70), (129, 17)])
def test_rgemm_fp8_in_kernel_equals_prepared(fmt, M, N, tune):
    """The fp8 variant quantized inside the kernel (f8_quad) = act_quant's F8DEQ x~ read
    prepared, bit for bit; and within the fp8 gate of tests/test_gpu_fp8.py of the fp8-exact
    product."""
    tune(GQ_RGEMM=1)
    K = 1024
    qA = random_blocks(fmt, M, K, seed=M + 5)
    B = random_activations(N, K, seed=N + 7)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    C = _mmq(fmt, A_t, B_t, M, N, K, act="fp8")
    Cp = _prepared(fmt, A_t, B_t, M, N, K, act="fp8")
    assert torch.equal(Cp.view(torch.int16), C.view(torch.int16))
    ideal = O.mmq_fp8_ideal(fmt, qA, B, M, N, K)
    assert O.max_rel_err(C.cpu().numpy(), ideal) <= TIGHT


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("N", [16, 32, 64, 128, 90])
def test_rgemm_one_superblock_bit_identical_to_gemm(fmt, N, tune):
    """K = 256: one split, no partials -- the resident kernel (256-row tiles) and gemm_kernel
    (128-row tiles) run the same dequantization and MFMA sequence per row: identical bits."""
    M, K = 600, 256
    qA = random_blocks(fmt, M, K, seed=N)
    B = random_activations(N, K, seed=N + 1)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    tune(GQ_RGEMM=1, GQ_SKINNY=0)  # (Q4_K / Q8_0 at 16 tokens would take the skinny kernel)
    C1 = _prepared(fmt, A_t, B_t, M, N, K)
    tune(GQ_RGEMM=0, GQ_GEMM_SPLITS=1)
    C0 = _prepared(fmt, A_t, B_t, M, N, K)
    assert torch.equal(C0.view(torch.int16), C1.view(torch.int16))


def test_rgemm_headline_full_size():
    """BASELINE configs[1] (Q8_0 4096 x 4096, 128 tokens) through the default route -- the
    resident GEMM with in-kernel quantization -- on 48 sampled rows against the oracle."""
    import kernels._lib as kl
    M, N, K = 4096, 128, 4096
    qA = random_blocks("q8_0", M, K, seed=17)
    B = random_activations(N, K, seed=18)
    C = _mmq("q8_0", _t(qA.view(np.int8)), _t(B), M, N, K).cpu().numpy()
    rows = np.sort(np.random.default_rng(1).choice(M, size=48, replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    ideal = O.mmq_from_fp16("q8_0", sub, B, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(C[:, rows], ideal) <= TIGHT
    exact = O.mmq_from_fp16("q8_0", sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, C[:, rows], 0.01)
    assert kl.lib() is not None


# ---- the streaming form (sgemm_kernel): prepared x~, half-super-block stages through an LDS ring


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("M,N,K,S", [(600, 100, 4096, 0), (300, 128, 8192, 3), (257, 40, 2816, 0), (700, 20, 1024, 1),
                                     (129, 17, 3072, 5), (1000, 64, 2048, 2)])
def test_sgemm_parity(fmt, M, N, K, S, tune):
    """Every format and token tile, ragged rows and tokens, uneven split lengths (S not dividing
    the super-blocks), one split (no partials) and the automatic split."""
    tune(GQ_RGEMM=0, GQ_SGEMM=1, GQ_SKINNY=0, GQ_SGEMM_SPLITS=S)
    qA = random_blocks(fmt, M, K, seed=M + 2 * N + K)
    B = random_activations(N, K, seed=5 * K + N)
    C = _prepared(fmt, _t(qA.view(np.int8)), _t(B), M, N, K)
    got = C.cpu().numpy()
    assert np.isfinite(got.astype(np.float32)).all()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT, O.max_rel_err(got, ideal)
    exact = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


@pytest.mark.parametrize("fmt", FMTS)
def test_sgemm_bit_identities(fmt, tune):
    """With one super-block per split the streaming form is the resident form (same partials,
    same reduce): identical bits; with one split it is gemm_kernel's MFMA sequence per row."""
    M, N, K = 520, 96, 2048
    qA = random_blocks(fmt, M, K, seed=3)
    B = random_activations(N, K, seed=4)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    tune(GQ_RGEMM=1, GQ_SKINNY=0)
    Cr = _prepared(fmt, A_t, B_t, M, N, K)
    tune(GQ_RGEMM=0, GQ_SGEMM=1, GQ_SGEMM_SPLITS=K // 256)
    Cs = _prepared(fmt, A_t, B_t, M, N, K)
    assert torch.equal(Cr.view(torch.int16), Cs.view(torch.int16))
    tune(GQ_SGEMM_SPLITS=1)
    C1 = _prepared(fmt, A_t, B_t, M, N, K)
    tune(GQ_SGEMM=0, GQ_GEMM_SPLITS=1)
    C0 = _prepared(fmt, A_t, B_t, M, N, K)
    assert torch.equal(C0.view(torch.int16), C1.view(torch.int16))
