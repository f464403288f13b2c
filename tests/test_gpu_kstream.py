"""GPU parity of the K-chunked streaming MMQ (csrc/mmq_kstream.hip: 5..32 tokens, x~ in VGPRs with
each of a workgroup's 8 waves one K chunk, weights streamed per wave through private LDS rings,
the waves' tiles summed in LDS by the last arriver; one launch, no split-K partials).

Checked: every format at 5..32 tokens (one and two 16-token tiles, ragged N), K from one
super-block to the longest one launch holds (K = 4096) including K that leaves waves idle or short
(K = 768, 1280, 2816), and longer K in ranges of 16 super-blocks whose fp32 partials a second
launch sums (K = 4352: a one-super-block range; 8192, 11008, 28672); the in-kernel quantization
(gq_mmq_ex) and
the prepared call (act_quant DEQ + the kernel) agree bit for bit; a grouped launch
(gq_mmq_grouped_ex, mixed formats and K) gives every item's own bits; repeated calls give the
same bits.  Tolerance: TIGHT (fp16 W x fp16 x~, fp32 MFMA accumulation) against the oracle's IDEAL
mode, and the reference's own 1% gate (utils/test_utils.py:4-8) against EXACT (= cpu_impls)."""
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


def _check_rows(fmt, qA, B, got, M, N, K, nrows=48, seed=0):
    rows = np.sort(np.random.default_rng(seed).choice(M, size=min(M, nrows), replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    ideal = O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.IDEAL)
    err = O.max_rel_err(got[:, rows], ideal)
    assert err <= TIGHT, (fmt, M, N, K, err)
    exact = O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, got[:, rows], 0.01)


CASES = [(4096, 16, 4096), (256, 5, 4096), (1024, 13, 3072), (512, 8, 256), (768, 16, 768), (4096, 32, 4096),
         (512, 17, 1280), (2048, 24, 2816), (11008, 16, 4096), (64, 9, 1024),
         # K ranges (16 super-blocks each) summed by the second launch
         (1024, 16, 8192), (512, 7, 11008), (256, 32, 4352), (128, 20, 28672),
         # edges: one 16-row item, one super-block (seven of the eight waves idle), the fewest
         # and the most tokens of the two token-group kernels
         (16, 5, 256), (16, 32, 256), (48, 31, 512), (32, 17, 4096)]


@pytest.mark.parametrize("fmt", ["q8_0", "q4_k", "q6_k"])
@pytest.mark.parametrize("M,N,K", CASES)
def test_kstream_parity(fmt, M, N, K, tune):
    import kernels._lib as kl
    tune(GQ_KSTREAM=1)
    t = kl.TYPES[fmt]
    assert kl.route_name(t, M, N, K).startswith("kstream_kernel"), kl.route_name(t, M, N, K)
    qA = random_blocks(fmt, M, K, seed=M + N + K)
    B = random_activations(N, K, seed=2 * K + N)
    A_t, B_t = _t(qA.view(np.int8)), _t(B)
    C = kl.mmq(t, A_t, B_t, M, N, K)
    ws = torch.empty(kl.workspace_size(t, M, N, K), dtype=torch.uint8, device=_dev())
    kl.act_prepare(B_t, N, K, ws)
    assert kl.route_name(t, M, N, K, prepared=True).startswith("kstream_kernel")
    Cp = kl.mmq_prepared(t, A_t, ws, M, N, K)
    C2 = kl.mmq(t, A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(C.view(torch.int16), Cp.view(torch.int16)), "in-kernel q8_1 != prepared x~"
    assert torch.equal(C.view(torch.int16), C2.view(torch.int16)), "repeat call"
    got = C.cpu().numpy()
    assert np.isfinite(got.astype(np.float32)).all()
    _check_rows(fmt, qA, B, got, M, N, K, seed=M)


def test_kstream_grouped_prepared_layer(tune):
    """The 7B Q4_K_M layer's projections at 16 tokens through gq_mmq_grouped_prepared: the K = 4096
    items and ffn_down (K = 11008, three K ranges) in one K-chunked stream launch + its range sum;
    every output equals the item's own prepared call, and the oracle within TIGHT on sampled rows."""
    import kernels._lib as kl
    N = 16
    spec = [("q4_k", 4096, 4096), ("q4_k", 1024, 4096), ("q6_k", 2048, 4096), ("q6_k", 4096, 11008)]
    items, wss, Bs, qAs = [], [], [], []
    for i, (fmt, M, K) in enumerate(spec):
        qA = random_blocks(fmt, M, K, seed=300 + i)
        B = random_activations(N, K, seed=400 + K)
        ws = torch.empty(kl.workspace_size(kl.TYPES[fmt], M, N, K), dtype=torch.uint8, device=_dev())
        kl.act_prepare(_t(B), N, K, ws)
        A_t = _t(qA.view(np.int8))
        items.append((kl.TYPES[fmt], A_t, ws, M, K, None))
        qAs.append(qA)
        Bs.append(B)
    outs = kl.mmq_grouped_prepared(items, N)
    assert outs is not None
    tune(GQ_KSTREAM=1)
    for i, (fmt, M, K) in enumerate(spec):
        single = kl.mmq_prepared(kl.TYPES[fmt], items[i][1], items[i][2], M, N, K)
        torch.cuda.synchronize()
        assert torch.equal(outs[i].view(torch.int16), single.view(torch.int16)), f"item {i}"
        _check_rows(fmt, qAs[i], Bs[i], outs[i].cpu().numpy(), M, N, K, nrows=24, seed=i)


def test_kstream_grouped_bit_identical(tune):
    """A Q4_K_M-style group (mixed formats, K = 4096 and 2816, 16 tokens) in one launch: every
    item's bits equal its own call; two items share one activation."""
    import kernels._lib as kl
    tune(GQ_KSTREAM=1)
    N = 16
    spec = [("q4_k", 4096, 4096), ("q6_k", 1024, 4096), ("q4_k", 2816, 4096), ("q8_0", 512, 2816),
            ("q6_k", 4096, 2816)]
    xs = {K: _t(random_activations(N, K, seed=K)) for K in (4096, 2816)}
    items, singles = [], []
    for i, (fmt, M, K) in enumerate(spec):
        qA = random_blocks(fmt, M, K, seed=100 + i)
        A_t = _t(qA.view(np.int8))
        items.append((kl.TYPES[fmt], A_t, xs[K], M, K, None))
        singles.append(kl.mmq(kl.TYPES[fmt], A_t, xs[K], M, N, K))
    outs = kl.mmq_grouped(items, N)
    assert outs is not None, "grouped kstream refused"
    torch.cuda.synchronize()
    for i, (o, s) in enumerate(zip(outs, singles)):
        assert torch.equal(o.view(torch.int16), s.view(torch.int16)), f"item {i}"


def test_kstream_fp8_matches_prepared_f8deq(tune):
    """The fp8 variant (in-kernel e4m3 quantization) gives the bits of the prepared F8DEQ x~."""
    import kernels._lib as kl
    tune(GQ_KSTREAM=1)
    for fmt, M, N, K in (("q4_k", 2048, 16, 4096), ("q6_k", 1024, 3, 4096), ("q8_0", 512, 32, 4096)):
        t = kl.TYPES[fmt]
        qA = random_blocks(fmt, M, K, seed=7)
        B = random_activations(N, K, seed=8)
        A_t, B_t = _t(qA.view(np.int8)), _t(B)
        C = kl.mmq(t, A_t, B_t, M, N, K, act="fp8")
        ws = torch.empty(kl.workspace_size(t, M, N, K, act="fp8"), dtype=torch.uint8, device=_dev())
        kl.act_prepare(B_t, N, K, ws, act="fp8")
        Cp = kl.mmq_prepared(t, A_t, ws, M, N, K, act="fp8")
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), Cp.view(torch.int16)), fmt

def test_kstream_grouped_default_tuning():
    """gq_mmq_grouped at 5..32 tokens under the default tuning takes the K-chunked stream (its
    own route: no GQ_KSTREAM needed) and gives each item's stream bits (the raw call pinned to the
    stream, GQ_KSTREAM=1, for the 4096-row items the default sends to the resident GEMM)."""
    import kernels._lib as kl
    N = 12
    spec = [("q4_k", 4096, 4096), ("q6_k", 1024, 4096), ("q8_0", 8192, 2816)]
    xs = {K: _t(random_activations(N, K, seed=K + 1)) for K in (4096, 2816)}
    items, As = [], []
    for i, (fmt, M, K) in enumerate(spec):
        A_t = _t(random_blocks(fmt, M, K, seed=200 + i).view(np.int8))
        items.append((kl.TYPES[fmt], A_t, xs[K], M, K, None))
        As.append(A_t)
    outs = kl.mmq_grouped(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    kl.set_tuning("GQ_KSTREAM", 1)
    try:
        for i, (fmt, M, K) in enumerate(spec):
            solo = kl.mmq(kl.TYPES[fmt], As[i], xs[K], M, N, K)
            torch.cuda.synchronize()
            assert torch.equal(outs[i].view(torch.int16), solo.view(torch.int16)), f"item {i}"
    finally:
        kl.reset_tuning()
