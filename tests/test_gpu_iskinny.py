"""GPU parity of the integer-MFMA skinny kernel (csrc/mmq_iskinny.hip, GQ_ISKINNY=1: Q4_K at
5..16 tokens through gq_mmq): nibbles x q8_1 codes in v_mfma_i32_16x16x32_i8 per 32-block,
rescaled by d*sc*d_x, the min term -dmin*m*s_x as an fp32 MFMA -- the reference's per-block
arithmetic.  Against the oracle: EXACT within the reference's 1% gate, IDEAL within the GEMM
tolerance; ragged rows and tokens, every fragment count per unit, K from one super-block to
11008."""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT = 4e-3


@pytest.mark.parametrize("M,N,K", [(4096, 16, 4096), (1000, 5, 1024), (333, 11, 256), (4096, 8, 11008),
                                   (64, 16, 2048), (11008, 13, 4096)])
@pytest.mark.parametrize("rg", [0, 1, 4])
def test_iskinny_q4k_parity(M, N, K, rg, tune):
    import kernels._lib as kl
    assert torch.cuda.is_available()
    dev = torch.device("cuda:0")
    tune(GQ_ISKINNY=1, GQ_ISKINNY_RG=rg)
    assert "iskinny" in kl.route_name(kl.GQ_Q4_K, M, N, K)
    qA = random_blocks("q4_k", M, K, seed=M + N + rg)
    B = random_activations(N, K, seed=K + N)
    C = kl.mmq(kl.GQ_Q4_K, torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev), M, N, K)
    torch.cuda.synchronize()
    got = C.cpu().numpy()
    assert np.isfinite(got.astype(np.float32)).all()
    rows = np.sort(np.random.default_rng(M).choice(M, size=min(M, 48), replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    exact = O.mmq_from_fp16("q4_k", sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, got[:, rows], 0.01)
    ideal = O.mmq_from_fp16("q4_k", sub, B, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(got[:, rows], ideal) <= TIGHT, O.max_rel_err(got[:, rows], ideal)
