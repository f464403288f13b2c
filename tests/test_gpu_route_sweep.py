"""Every route the default tuning can pick, swept over token counts and shapes: the raw call and the
prepared call both run and agree within the GEMM tolerance (they may take different kernels -- e.g.
the resident GEMM raw and the K-chunked stream prepared -- whose fp32 sums over K run in other
orders), the grouped launch accepts every shape its forms cover and gives each item's raw-call
result, and nothing is refused that the header documents as supported.  (A raw grouped launch at
5..32 tokens was refused by the default tuning in round 5 until this sweep's case existed.)"""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

GEMM_TOL = 4e-3


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(_dev())


SHAPES = [(64, 256), (512, 4096), (8192, 4096), (1024, 11008)]
TOKENS = [1, 2, 3, 4, 5, 8, 16, 17, 32, 33, 64, 128, 200]


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("M,K", SHAPES)
def test_raw_and_prepared_agree_over_token_counts(fmt, M, K):
    import kernels._lib as kl
    t = kl.TYPES[fmt]
    A = _t(random_blocks(fmt, M, K, seed=M + K).view(np.int8))
    for N in TOKENS:
        B = _t(random_activations(N, K, seed=N + K))
        raw = kl.mmq(t, A, B, M, N, K)
        ws = torch.empty(kl.workspace_size(t, M, N, K), dtype=torch.uint8, device=_dev())
        kl.act_prepare(B, N, K, ws)
        prep = kl.mmq_prepared(t, A, ws, M, N, K)
        torch.cuda.synchronize()
        r, p = raw.cpu().numpy(), prep.cpu().numpy()
        assert np.isfinite(r.astype(np.float32)).all(), (fmt, M, N, K, kl.route_name(t, M, N, K))
        err = O.max_rel_err(p, r.astype(np.float32))
        assert err <= GEMM_TOL, (fmt, M, N, K, err, kl.route_name(t, M, N, K), kl.route_name(t, M, N, K, prepared=True))


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 9, 16, 24, 32])
def test_grouped_accepts_its_shapes(N):
    """1..4 tokens: the grouped decode; 5..32: the K-chunked stream (K <= 4096, M % 16 == 0).  Each
    item equals its own raw call within the GEMM tolerance (bit-identical on the decode routes)."""
    import kernels._lib as kl
    spec = [("q4_k", 4096, 4096), ("q6_k", 1024, 4096), ("q8_0", 2048, 2816), ("q6_k", 8192, 1024)]
    items, raws = [], []
    for i, (fmt, M, K) in enumerate(spec):
        t = kl.TYPES[fmt]
        A = _t(random_blocks(fmt, M, K, seed=40 + i).view(np.int8))
        B = _t(random_activations(N, K, seed=50 + i))
        items.append((t, A, B, M, K, None))
        raws.append(kl.mmq(t, A, B, M, N, K))
    outs = kl.mmq_grouped(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(zip(outs, raws)):
        if N <= 4:
            assert torch.equal(o.view(torch.int16), r.view(torch.int16)), i
        else:
            assert O.max_rel_err(o.cpu().numpy(), r.cpu().numpy().astype(np.float32)) <= GEMM_TOL, i


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("M,K", [(512, 4096), (8192, 4096)])
def test_fp8_raw_and_prepared_agree_over_token_counts(fmt, M, K):
    """The fp8 activation variant: the same sweep (its decode form at 1..2 tokens, the K-chunked
    stream and the fp16-x~ kernels from 3)."""
    import kernels._lib as kl
    t = kl.TYPES[fmt]
    A = _t(random_blocks(fmt, M, K, seed=M + K + 1).view(np.int8))
    for N in (1, 2, 3, 5, 16, 33, 128):
        B = _t(random_activations(N, K, seed=N + 2 * K))
        raw = kl.mmq(t, A, B, M, N, K, act="fp8")
        ws = torch.empty(kl.workspace_size(t, M, N, K, act="fp8"), dtype=torch.uint8, device=_dev())
        kl.act_prepare(B, N, K, ws, act="fp8")
        prep = kl.mmq_prepared(t, A, ws, M, N, K, act="fp8")
        torch.cuda.synchronize()
        r, p = raw.cpu().numpy(), prep.cpu().numpy()
        assert np.isfinite(r.astype(np.float32)).all(), (fmt, M, N, K)
        assert O.max_rel_err(p, r.astype(np.float32)) <= GEMM_TOL, (fmt, M, N, K, kl.route_name(t, M, N, K, act="fp8"))


@pytest.mark.parametrize("act,Ns", [("q8_1", (1, 2, 3, 4)), ("fp8", (1, 2))])
@pytest.mark.parametrize("fmt,M,K", [("q8_0", 4096, 4096), ("q4_k", 11008, 4096), ("q6_k", 1024, 8192),
                                     ("q4_k", 96, 256)])
def test_prepared_decode_is_the_raw_decode(act, Ns, fmt, M, K):
    """At decode token counts gq_act_prepare keeps a copy of the activations and gq_mmq_prepared
    runs gq_mmq's one-launch decode on it: the same kernel on the same input, so the same bits."""
    import kernels._lib as kl
    t = kl.TYPES[fmt]
    A = _t(random_blocks(fmt, M, K, seed=M + 3 * K).view(np.int8))
    for N in Ns:
        assert kl.route_name(t, M, N, K, act=act) == "stream_decode_kernel", (fmt, M, N, K, act)
        assert kl.route_name(t, M, N, K, act=act, prepared=True) == "stream_decode_kernel", (fmt, M, N, K, act)
        B = _t(random_activations(N, K, seed=7 * N + K))
        raw = kl.mmq(t, A, B, M, N, K, act=act)
        ws = torch.empty(kl.workspace_size(t, M, N, K, act=act), dtype=torch.uint8, device=_dev())
        kl.act_prepare(B, N, K, ws, act=act)
        prep = kl.mmq_prepared(t, A, ws, M, N, K, act=act)
        torch.cuda.synchronize()
        assert torch.equal(raw.view(torch.int16), prep.view(torch.int16)), (fmt, M, N, K, act)
