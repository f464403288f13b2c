"""GPU parity of the skinny-token kernel (csrc/mmq_skinny.hip, the 5..32-token path) against the
oracle: token counts 5, 8, 16, 17, 32 and ragged ones, every instantiated rg, K from one
super-block (fewer than the 8 waves' K ranges) to 43, ragged rows; the reference's golden cases;
row independence (what row sharding relies on); prepared and chunked calls bit-identical.
Tolerance: TIGHT (fp16 W x fp16 x~ on fp32 MFMA) vs oracle IDEAL, and the reference's own 1% gate
vs oracle EXACT (kernels/cpu_impls arithmetic)."""
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


def _run(fmt, qA, B, M, N, K):
    from kernels._lib import TYPES, mmq
    dev = _dev()
    C = mmq(TYPES[fmt], torch.from_numpy(np.ascontiguousarray(qA).view(np.int8)).to(dev),
            torch.from_numpy(np.ascontiguousarray(B)).to(dev), M, N, K)
    torch.cuda.synchronize()
    return C.cpu().numpy()


def _check(fmt, qA, B, M, N, K):
    got = _run(fmt, qA, B, M, N, K)
    assert np.isfinite(got.astype(np.float32)).all()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT, O.max_rel_err(got, ideal)
    exact = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("N", [5, 8, 16, 17, 32, 7, 23])
@pytest.mark.parametrize("M,K", [(300, 1024), (64, 256), (1000, 2048), (129, 768)])
def test_skinny_tokens(fmt, N, M, K, tune):
    """Every type at 5..32 tokens through the kernel (forced: by default it takes Q4_K and Q8_0
    at 5..16)."""
    tune(GQ_SKINNY=1)
    qA = random_blocks(fmt, M, K, seed=M + N + K)
    B = random_activations(N, K, seed=K + 3 * N)
    _check(fmt, qA, B, M, N, K)


@pytest.mark.parametrize("fmt,rg", [("q4_k", 1), ("q4_k", 2), ("q4_k", 3), ("q4_k", 4), ("q6_k", 1), ("q6_k", 2),
                                    ("q6_k", 3), ("q8_0", 1), ("q8_0", 2), ("q8_0", 3), ("q8_0", 4)])
@pytest.mark.parametrize("M,N,K", [(520, 16, 4096), (90, 32, 11008), (257, 9, 2816), (33, 20, 512)])
def test_skinny_configs(fmt, rg, M, N, K, tune):
    """Every instantiated rows-per-workgroup (16 * rg), forced."""
    tune(GQ_SKINNY=1, GQ_SKINNY_RG=rg)
    qA = random_blocks(fmt, M, K, seed=M + K)
    B = random_activations(N, K, seed=N + K)
    _check(fmt, qA, B, M, N, K)


@pytest.mark.parametrize("fmt", FMTS)
def test_skinny_golden(golden, fmt, tune):
    """Every golden case of the reference with 5+ tokens and K % 256 == 0 through the kernel."""
    tune(GQ_SKINNY=1)
    n = 0
    for c in golden[fmt]:
        M, N, K = c["M"], c["N"], c["K"]
        if N < 5 or K % 256:
            continue
        got = _run(fmt, c["qA"], c["B"], M, N, K)
        ideal = O.mmq(fmt, c["qA"], c["qB"], M, N, K, O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT, (c["i"], c["kind"])
        if not (fmt == "q8_0" and c["kind"] == "tiny"):
            assert O.allclose(c["C"], got, 0.01), (c["i"], c["kind"])
        if "Ctri" in c:
            assert O.allclose(c["Ctri"], got, 0.01), (c["i"], c["kind"])
        n += 1
    assert n > 0


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("N", [8, 24])
def test_skinny_row_independence(fmt, N, tune):
    """A row's result does not depend on the rows around it or the workgroup shape (the rows
    per unit and units per workgroup differ between the two calls): any row subset computed as
    its own matrix gives the same bits."""
    from kernels._lib import TYPES, mmq
    tune(GQ_SKINNY=1)
    dev = _dev()
    M, K = 9000, 1536
    qA = random_blocks(fmt, M, K, seed=5)
    rb = qA.size // M
    B_t = torch.from_numpy(random_activations(N, K, seed=6)).to(dev)
    full = mmq(TYPES[fmt], torch.from_numpy(qA.view(np.int8)).to(dev), B_t, M, N, K)
    rows = np.array([0, 1, 17, 255, 256, 300, 511, 640, 4097, 8999])
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    part = mmq(TYPES[fmt], torch.from_numpy(sub.view(np.int8)).to(dev), B_t, len(rows), N, K)
    torch.cuda.synchronize()
    assert np.array_equal(part.cpu().numpy().view(np.uint16), full.cpu().numpy()[:, rows].view(np.uint16))


@pytest.mark.parametrize("fmt", FMTS)
def test_skinny_prepared_and_chunked(fmt, tune):
    """gq_act_prepare + gq_mmq_prepared, and a call cut into several launches by the 32-bit
    offset guard (GQ_GEMM_MAX_BYTES lowered), give the same bits as one gq_mmq call."""
    import kernels._lib as kl
    tune(GQ_SKINNY=1)
    dev = _dev()
    M, N, K = 600, 20, 2048
    qA = random_blocks(fmt, M, K, seed=9)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(random_activations(N, K, seed=10)).to(dev)
    one = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
    ws = torch.empty(kl.workspace_size(kl.TYPES[fmt], M, N, K), dtype=torch.uint8, device=dev)
    kl.act_prepare(B_t, N, K, ws)
    prep = kl.mmq_prepared(kl.TYPES[fmt], A_t, ws, M, N, K)
    tune(GQ_GEMM_MAX_BYTES=256 * 1024)
    many = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(one.view(torch.int16), prep.view(torch.int16))
    assert torch.equal(one.view(torch.int16), many.view(torch.int16))


@pytest.mark.parametrize("fmt,N", [("q4_k", 16), ("q4_k", 5), ("q8_0", 16), ("q8_0", 7)])
def test_skinny_default_route(fmt, N, tune):
    """The default route takes the kernel for Q4_K and Q8_0 at 5..16 tokens (GQ_SKINNY=0: the
    LDS-DMA GEMM): both within tolerance, and the two routes differ in bits (the route really
    changed)."""
    M, K = 512, 2048
    qA = random_blocks(fmt, M, K, seed=3)
    B = random_activations(N, K, seed=4)
    a = _run(fmt, qA, B, M, N, K)
    tune(GQ_SKINNY=0)
    b = _run(fmt, qA, B, M, N, K)
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(a, ideal) <= TIGHT and O.max_rel_err(b, ideal) <= TIGHT
    assert not np.array_equal(a.view(np.uint16), b.view(np.uint16))


@pytest.mark.parametrize("fmt", FMTS)
def test_skinny_strided_activations(fmt, tune):
    """A strided activation view (ldb > K) through gq_mmq gives the same bits as the contiguous
    copy and as gq_act_prepare + gq_mmq_prepared."""
    import kernels._lib as kl
    tune(GQ_SKINNY=1)
    dev = _dev()
    M, N, K = 700, 12, 2048
    qA = torch.from_numpy(random_blocks(fmt, M, K, seed=21).view(np.int8)).to(dev)
    wide = torch.from_numpy(random_activations(N, K + 512, seed=22)).to(dev)
    Bv = wide[:, 256:256 + K]
    a = kl.mmq(kl.TYPES[fmt], qA, Bv, M, N, K)
    b = kl.mmq(kl.TYPES[fmt], qA, Bv.contiguous(), M, N, K)
    ws = torch.empty(kl.workspace_size(kl.TYPES[fmt], M, N, K), dtype=torch.uint8, device=dev)
    kl.act_prepare(Bv.contiguous(), N, K, ws)
    c = kl.mmq_prepared(kl.TYPES[fmt], qA, ws, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert torch.equal(a.view(torch.int16), c.view(torch.int16))
