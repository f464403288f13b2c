"""GPU parity of the full-K tile GEMM (csrc/mmq_fgemm.hip: one workgroup per 32*rw rows x 16*nb
tokens x all of K, 8 waves = rw row groups x 8/rw K-interleaved waves summed in LDS; no split-K
partials).  Every tile shape, Q8_0 and Q4_K, ragged rows and tokens, K that is not a multiple
of the K-waves' super-blocks (K = 11008: 43), K = 256 (one super-block: most waves idle);
through gq_mmq_ex (act_quant + the kernel) and the prepared call, which must agree bit for bit.
Tolerance: TIGHT (fp16 W x fp16 x~, fp32 MFMA accumulation) vs the oracle's IDEAL mode, and the
reference's 1% gate (utils/test_utils.py:4-8) vs EXACT."""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT = 4e-3


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(_dev())


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k"])
@pytest.mark.parametrize("rw,nb", [(2, 2), (4, 2), (4, 4), (8, 4)])
@pytest.mark.parametrize("M,N,K", [(256, 128, 4096), (300, 100, 1024), (1000, 40, 11008), (513, 20, 768),
                                   (64, 17, 256), (129, 77, 2304)])
def test_fgemm_parity(fmt, rw, nb, M, N, K, tune):
    import kernels._lib as kl
    tune(GQ_FGEMM=1, GQ_FGEMM_RW=rw, GQ_FGEMM_NB=nb)
    assert kl.route_name(kl.TYPES[fmt], M, N, K).startswith("fgemm_kernel")
    qA = random_blocks(fmt, M, K, seed=M + N + K)
    B = random_activations(N, K, seed=2 * K + N)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    C = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
    ws = torch.empty(kl.workspace_size(kl.TYPES[fmt], M, N, K), dtype=torch.uint8, device=_dev())
    kl.act_prepare(B_t, N, K, ws)
    Cp = kl.mmq_prepared(kl.TYPES[fmt], A_t, ws, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(C.view(torch.int16), Cp.view(torch.int16))
    got = C.cpu().numpy()
    assert np.isfinite(got.astype(np.float32)).all()
    rows = np.sort(np.random.default_rng(M).choice(M, size=min(M, 64), replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    ideal = O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(got[:, rows], ideal) <= TIGHT, O.max_rel_err(got[:, rows], ideal)
    exact = O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, got[:, rows], 0.01)


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k"])
def test_fgemm_headline_full_size_and_repeat(fmt, tune):
    """The M = 128 shapes at full size on sampled rows, and the same bits from call to call."""
    import kernels._lib as kl
    tune(GQ_FGEMM=1)
    M, N, K = 4096, 128, 4096
    qA = random_blocks(fmt, M, K, seed=17)
    B = random_activations(N, K, seed=18)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    C = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
    for _ in range(3):
        assert torch.equal(kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K).view(torch.int16), C.view(torch.int16))
    got = C.cpu().numpy()
    rows = np.sort(np.random.default_rng(1).choice(M, size=48, replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    assert O.max_rel_err(got[:, rows], O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.IDEAL)) <= TIGHT
    assert O.allclose(O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.EXACT), got[:, rows], 0.01)
