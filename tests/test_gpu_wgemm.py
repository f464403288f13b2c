"""GPU parity of the weight-register GEMM (csrc/mmq_wgemm.hip, the 33+-token path) against the
oracle, over its whole configuration space: tile shapes (RG 1/2 x NB 2/4/8), weight ring depths
(WD 2/3/4), split-K factors, ragged rows/tokens, the split-K partial range, row independence.  Tolerance: TIGHT_GEMM (fp16 W x fp16 x~ on fp32 MFMA) vs oracle IDEAL, and the
reference's own 1% gate vs oracle EXACT (kernels/cpu_impls arithmetic)."""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT_GEMM = 4e-3
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


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("rg,nb,wd", [(1, 8, 4), (1, 8, 3), (1, 8, 2), (1, 4, 4), (1, 2, 4), (2, 8, 2), (2, 8, 3),
                                       (2, 4, 3), (2, 2, 2)])
@pytest.mark.parametrize("M,N,K,splits", [(300, 128, 1024, 0), (257, 100, 768, 3), (64, 200, 512, 1),
                                          (1000, 48, 2048, 0), (130, 33, 256, 0), (520, 256, 1024, 2)])
def test_wgemm_configs(fmt, rg, nb, wd, M, N, K, splits, tune):
    tune(GQ_WGEMM=1, GQ_WGEMM_RG=rg, GQ_WGEMM_NB=nb, GQ_WGEMM_WD=wd, GQ_WGEMM_SPLITS=splits)
    qA = random_blocks(fmt, M, K, seed=M + N + K)
    B = random_activations(N, K, seed=K + 3 * N)
    got = _run(fmt, qA, B, M, N, K)
    assert np.isfinite(got.astype(np.float32)).all()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT_GEMM, O.max_rel_err(got, ideal)
    exact = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


@pytest.mark.parametrize("fmt", FMTS)
def test_wgemm_golden(golden, fmt, tune):
    """Every golden case of the reference with K % 256 == 0, its GEMM-routed ones (5+ tokens)
    through the kernel (forced on: the fixtures hold at most 16 tokens)."""
    tune(GQ_WGEMM=1)
    n = 0
    for c in golden[fmt]:
        M, N, K = c["M"], c["N"], c["K"]
        if K % 256:
            continue
        got = _run(fmt, c["qA"], c["B"], M, N, K)
        ideal = O.mmq(fmt, c["qA"], c["qB"], M, N, K, O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT_GEMM, (c["i"], c["kind"])
        if not (fmt == "q8_0" and c["kind"] == "tiny"):
            assert O.allclose(c["C"], got, 0.01), (c["i"], c["kind"])
        n += 1
    assert n > 0


@pytest.mark.parametrize("fmt", FMTS)
def test_wgemm_row_independence(fmt, tune):
    """Without split-K, a row's arithmetic does not depend on the tile it lands in: any row
    subset computed as its own matrix gives the same bits (what row sharding relies on)."""
    from kernels._lib import TYPES, mmq
    tune(GQ_WGEMM=1, GQ_WGEMM_SPLITS=1)
    dev = _dev()
    M, N, K = 700, 96, 1536
    qA = random_blocks(fmt, M, K, seed=5)
    rb = qA.size // M
    B_t = torch.from_numpy(random_activations(N, K, seed=6)).to(dev)
    full = mmq(TYPES[fmt], torch.from_numpy(qA.view(np.int8)).to(dev), B_t, M, N, K)
    rows = np.array([0, 1, 17, 255, 256, 300, 511, 640, 699])
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    part = mmq(TYPES[fmt], torch.from_numpy(sub.view(np.int8)).to(dev), B_t, len(rows), N, K)
    torch.cuda.synchronize()
    assert np.array_equal(part.cpu().numpy().view(np.uint16), full.cpu().numpy()[:, rows].view(np.uint16))


def test_wgemm_split_partials_cancelling(tune):
    """Split-K partials far outside fp16's range whose total cancels: the fp16 partials carry a
    per-wave power-of-two scale, so nothing overflows and the halves cancel."""
    tune(GQ_WGEMM=1, GQ_WGEMM_SPLITS=8)
    M, N, K = 256, 128, 4096
    half = random_blocks("q8_0", M, K // 2, seed=31).reshape(M, -1)
    qA = np.concatenate([half, half], axis=1).reshape(-1)
    x = (random_activations(N, K // 2, seed=32).astype(np.float32) * 20000).clip(-60000, 60000).astype(np.float16)
    B = np.concatenate([x, -x], axis=1)
    got = _run("q8_0", qA, B, M, N, K).astype(np.float32)
    assert np.isfinite(got).all()
    assert np.abs(got).max() <= 256


@pytest.mark.parametrize("fmt", FMTS)
def test_wgemm_prepared_and_chunked(fmt, tune):
    """gq_act_prepare + gq_mmq_prepared, and calls cut into several launches by the 32-bit
    offset guard (GQ_GEMM_MAX_BYTES lowered), give the same bits as one gq_mmq call."""
    import kernels._lib as kl
    tune(GQ_WGEMM=1, GQ_WGEMM_SPLITS=1)
    dev = _dev()
    M, N, K = 600, 160, 2048
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
