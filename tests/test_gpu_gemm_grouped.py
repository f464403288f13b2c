"""GPU tests of the grouped streaming GEMM (gq_mmq_grouped_prepared, csrc/mmq_rgemm.hip
sgemm_grouped_kernel + reduce_grouped_kernel): the projections of a layer, each of its own type,
prepared activations and output, in ONE launch (plus one split-K reduce launch) at 5..767
tokens.  Each projection bit for bit against its own per-matrix call at the same split (one split:
gemm_kernel's MFMA sequence; four: the streaming kernel's own partials and reduce), the full
Llama-7B Q4_K_M layer against the oracle at 16/128/512 tokens (sampled rows; TIGHT vs IDEAL,
the reference's 1% gate vs EXACT), LayerMix's grouped route against its per-call route within
the GEMM tolerance, and what the grouped form cannot take refused without launching."""
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


def _layer(types, seed=0):
    from gguf import LLAMA_LAYER_SHAPES
    dev = _dev()
    raw = {n: random_blocks(types[n], M, K, seed=seed + i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    return raw, {n: torch.from_numpy(raw[n].view(np.int8)).to(dev) for n in raw}


def _prepare(kl, B, N, K, act="q8_1", need=None):
    need = need if need is not None else kl.workspace_size(kl.GQ_Q4_K, 256, N, K, act)
    ws = torch.empty(need, dtype=torch.uint8, device=_dev())
    kl.act_prepare(B, N, K, ws, act=act)
    return ws


def _layer_items(kl, N, layer=0, seed=0):
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    dev = _dev()
    types = q4_k_m_layer_types(layer, 32)
    raw, A = _layer(types, seed=seed)
    x = random_activations(N, 4096, seed=seed + 1)
    h = random_activations(N, 11008, seed=seed + 2)
    xt, ht = torch.from_numpy(x).to(dev), torch.from_numpy(h).to(dev)
    wx = _prepare(kl, xt, N, 4096)
    wh = _prepare(kl, ht, N, 11008)
    items, names, inputs = [], [], []
    for n, (M, K) in LLAMA_LAYER_SHAPES.items():
        names.append(n)
        items.append((kl.TYPES[types[n]], A[n], wh if K == 11008 else wx, M, K, None))
        inputs.append(ht if K == 11008 else xt)
    return types, raw, x, h, items, names, inputs


@pytest.mark.parametrize("N", [5, 16, 40, 128])
@pytest.mark.parametrize("splits", [1, 4])
def test_grouped_gemm_bit_identical_to_per_matrix(N, splits, tune):
    """splits pinned: every projection = its own prepared call with the same split.  One split is
    gemm_kernel's per-row MFMA sequence (GQ_SGEMM=0 GQ_GEMM_SPLITS=1); four the per-matrix
    streaming kernel's (GQ_SGEMM=1 GQ_SGEMM_SPLITS=4), the grouped reduce = gemm_reduce_f16."""
    import kernels._lib as kl
    tune(GQ_SGEMM_SPLITS=splits, GQ_KSTREAM=0)  # (the streaming GEMM's grouped form)
    types, raw, x, h, items, names, inputs = _layer_items(kl, N, layer=0, seed=N)
    outs = kl.mmq_grouped_prepared(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    if splits == 1:
        tune(GQ_SGEMM=0, GQ_RGEMM=0, GQ_SKINNY=0, GQ_GEMM_SPLITS=1)
    else:
        tune(GQ_SGEMM=1, GQ_RGEMM=0, GQ_SKINNY=0, GQ_SGEMM_SPLITS=splits)
    for (t, A, _, M, K, _), n, C, B in zip(items, names, outs, inputs):
        ws = torch.empty(kl.workspace_size(t, M, N, K), dtype=torch.uint8, device=_dev())  # (+ this route's partials)
        kl.act_prepare(B, N, K, ws)
        solo = kl.mmq_prepared(t, A, ws, M, N, K)
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), solo.view(torch.int16)), n


@pytest.mark.parametrize("N", [16, 128, 512])
def test_grouped_gemm_llama_layer_parity(N):
    """The seven Llama-7B projections (layer 0: attn_v / ffn_down in Q6_K) in one grouped launch
    at the automatic split plan (16, 128 tokens; at 512 the layer's 664 tiles exceed one round of
    the chip: refused, and LayerMix's per-call route is what runs), every projection on sampled
    rows against the oracle."""
    import kernels._lib as kl
    from gguf import LLAMA_LAYER_SHAPES
    from kernels.layer_mix import GGUFLinear, LayerMix
    types, raw, x, h, items, names, inputs = _layer_items(kl, N, layer=0, seed=7 * N)
    outs = kl.mmq_grouped_prepared(items, N)
    if N == 512:
        assert outs is None
        lins = {n: GGUFLinear(types[n], A, M, K) for n, (_, A, _, M, K, _) in zip(names, items)}
        xt = inputs[0]
        ht = inputs[names.index("ffn_down")]
        res = LayerMix(lins, fuse=False).forward(xt, ht, attn=xt, x_ffn=xt)
        outs = [res[n] for n in names]
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    rng = np.random.default_rng(N)
    for n, C in zip(names, outs):
        M, K = LLAMA_LAYER_SHAPES[n]
        got = C.cpu().numpy()
        assert np.isfinite(got.astype(np.float32)).all(), n
        rows = np.sort(rng.choice(M, size=16, replace=False))
        rb = raw[n].size // M
        sub = np.concatenate([raw[n][r * rb:(r + 1) * rb] for r in rows])
        B = h if K == 11008 else x
        ideal = O.mmq_from_fp16(types[n], sub, B, len(rows), N, K, O.IDEAL)
        assert O.max_rel_err(got[:, rows], ideal) <= TIGHT, n
        exact = O.mmq_from_fp16(types[n], sub, B, len(rows), N, K, O.EXACT)
        assert O.allclose(exact, got[:, rows], 0.01), n


def test_grouped_gemm_ragged_strided_outputs():
    """Ragged rows and uneven K per item, one shared prepared input, outputs written into column
    ranges of one wide buffer (ldc > M): each range = the item's own call, the rest untouched."""
    import kernels._lib as kl
    dev = _dev()
    N = 70
    specs = [("q8_0", 333, 1024), ("q4_k", 1000, 2048), ("q6_k", 257, 1536), ("q4_k", 64, 2048), ("q8_0", 4096, 4096)]
    X = {K: torch.from_numpy(random_activations(N, K, seed=K)).to(dev) for K in {s[2] for s in specs}}
    ws = {K: _prepare(kl, X[K], N, K) for K in X}
    width = sum(M for _, M, _ in specs) + 5
    buf = torch.full((N, width), -7.0, dtype=torch.float16, device=dev)
    items, col, qs = [], 0, []
    for i, (fmt, M, K) in enumerate(specs):
        qA = torch.from_numpy(random_blocks(fmt, M, K, seed=i).view(np.int8)).to(dev)
        qs.append(qA)
        items.append((kl.TYPES[fmt], qA, ws[K], M, K, buf[:, col:col + M]))
        col += M
    with kl.tuning(GQ_SGEMM_SPLITS=2):
        outs = kl.mmq_grouped_prepared(items, N)
        assert outs is not None, kl.lib().gq_last_error()
        torch.cuda.synchronize()
    with kl.tuning(GQ_SGEMM=1, GQ_RGEMM=0, GQ_SKINNY=0, GQ_SGEMM_SPLITS=2):
        col = 0
        for (fmt, M, K), qA in zip(specs, qs):
            wsi = _prepare(kl, X[K], N, K, need=kl.workspace_size(kl.TYPES[fmt], M, N, K))  # (+ partials)
            solo = kl.mmq_prepared(kl.TYPES[fmt], qA, wsi, M, N, K)
            torch.cuda.synchronize()
            assert torch.equal(buf[:, col:col + M].view(torch.int16), solo.view(torch.int16)), fmt
            col += M
    assert torch.all(buf[:, col:] == -7.0)


def test_grouped_gemm_refuses():
    """Decode sizes (1..4 tokens: the decode form's), K not a multiple of 256, more than 16
    items and more tiles than one round of the chip are refused (None), nothing launched, the
    outputs untouched."""
    import kernels._lib as kl
    dev = _dev()
    qA = torch.from_numpy(random_blocks("q8_0", 64, 1024, seed=1).view(np.int8)).to(dev)
    for N, K, n in ((4, 1024, 1), (8, 1056, 1), (8, 1024, 17)):
        qK = qA if K == 1024 else torch.from_numpy(random_blocks("q8_0", 64, K, seed=2).view(np.int8)).to(dev)
        ws = _prepare(kl, torch.from_numpy(random_activations(N, K, seed=3)).to(dev), N, K)
        outs = [torch.full((N, 64), 3.0, dtype=torch.float16, device=dev) for _ in range(n)]
        assert kl.mmq_grouped_prepared([(kl.GQ_Q8_0, qK, ws, 64, K, o) for o in outs], N) is None
        torch.cuda.synchronize()
        assert all(torch.all(o == 3.0) for o in outs)
    M, K, N = 257 * 256, 256, 16  # 257 row tiles
    qB = torch.from_numpy(random_blocks("q8_0", M, K, seed=4).view(np.int8)).to(dev)
    ws = _prepare(kl, torch.from_numpy(random_activations(N, K, seed=5)).to(dev), N, K)
    out = torch.full((N, M), 3.0, dtype=torch.float16, device=dev)
    # (the streaming GEMM's limit: the K-chunked stream, which takes such items by default, off)
    with kl.tuning(GQ_CUS=256, GQ_KSTREAM=0):
        assert kl.mmq_grouped_prepared([(kl.GQ_Q8_0, qB, ws, M, K, out)], N) is None
    torch.cuda.synchronize()
    assert torch.all(out == 3.0)


@pytest.mark.parametrize("N", [5, 8, 16, 17, 128, 512])
def test_layer_mix_grouped_gemm_route(N):
    """LayerMix from 5 tokens runs the layer as one grouped GEMM launch (the stream-K plan):
    within the GEMM tolerance of its per-call route (grouped=False), `out` buffers honoured."""
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    _, A = _layer(types, seed=3)
    lins = {n: GGUFLinear(types[n], A[n], M, K) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    x, a, y = (torch.from_numpy(random_activations(N, 4096, seed=s)).to(dev) for s in (5, 6, 7))
    h = torch.from_numpy(random_activations(N, 11008, seed=8)).to(dev)
    out = {n: torch.empty(N, M, dtype=torch.float16, device=dev) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    rg = LayerMix(lins, grouped=True, fuse=False).forward(x, h, attn=a, x_ffn=y, out=out)
    ru = LayerMix(lins, grouped=False, fuse=False).forward(x, h, attn=a, x_ffn=y)
    torch.cuda.synchronize()
    for n in LLAMA_LAYER_SHAPES:
        assert rg[n].data_ptr() == out[n].data_ptr(), n
        assert O.max_rel_err(rg[n].cpu().numpy(), ru[n].cpu().numpy()) <= TIGHT, n


@pytest.mark.parametrize("cus", [256, 97, 37])
def test_grouped_gemm_stream_k(cus, tune):
    """The stream-K plan (GQ_SGEMM_STREAMK=1) spreads the (tile, super-block) units evenly over
    the workgroups: a workgroup may end one tile and start the next, a tile's partial sums come from
    a varying number of workgroups (odd workgroup counts forced by GQ_CUS), and tiles one
    workgroup holds whole are stored without partials.  Against the oracle on sampled rows,
    and the same bits call after call."""
    import kernels._lib as kl
    dev = _dev()
    tune(GQ_CUS=cus, GQ_SGEMM_STREAMK=1, GQ_KSTREAM=0)
    N = 40
    specs = [("q4_k", 1000, 4096), ("q6_k", 300, 2816), ("q8_0", 2048, 1024), ("q4_k", 256, 11008), ("q6_k", 64, 256)]
    X = {K: random_activations(N, K, seed=K) for K in {s[2] for s in specs}}
    ws = {K: _prepare(kl, torch.from_numpy(X[K]).to(dev), N, K) for K in X}
    raws, items = [], []
    for i, (fmt, M, K) in enumerate(specs):
        raw = random_blocks(fmt, M, K, seed=10 + i)
        raws.append(raw)
        items.append((kl.TYPES[fmt], torch.from_numpy(raw.view(np.int8)).to(dev), ws[K], M, K, None))
    outs = kl.mmq_grouped_prepared(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    again = kl.mmq_grouped_prepared(items, N)
    torch.cuda.synchronize()
    rng = np.random.default_rng(cus)
    for (fmt, M, K), raw, C, C2 in zip(specs, raws, outs, again):
        assert torch.equal(C.view(torch.int16), C2.view(torch.int16)), fmt
        rows = np.sort(rng.choice(M, size=min(M, 24), replace=False))
        rb = raw.size // M
        sub = np.concatenate([raw[r * rb:(r + 1) * rb] for r in rows])
        got = C.cpu().numpy()[:, rows]
        ideal = O.mmq_from_fp16(fmt, sub, X[K], len(rows), N, K, O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT, (fmt, M, K)


@pytest.mark.parametrize("fmt,M,K,N", [("q6_k", 2048, 8192, 128), ("q4_k", 1000, 4096, 40), ("q8_0", 777, 2816, 20)])
def test_single_matrix_stream_k(fmt, M, K, N, tune):
    """The streaming GEMM of one matrix through the one-part stream-K plan (GQ_SGEMM_STREAMK=1)
    against the oracle, and equal to the whole-tile plan within the GEMM tolerance."""
    import kernels._lib as kl
    dev = _dev()
    raw = random_blocks(fmt, M, K, seed=M)
    B = random_activations(N, K, seed=K)
    A_t, B_t = torch.from_numpy(raw.view(np.int8)).to(dev), torch.from_numpy(B).to(dev)
    tune(GQ_RGEMM=0, GQ_SKINNY=0, GQ_SGEMM=1, GQ_SGEMM_STREAMK=1, GQ_CUS=61, GQ_KSTREAM=0)
    ws = _prepare(kl, B_t, N, K, need=kl.workspace_size(kl.TYPES[fmt], M, N, K))
    C = kl.mmq_prepared(kl.TYPES[fmt], A_t, ws, M, N, K).cpu().numpy()
    tune(GQ_SGEMM_STREAMK=0)
    ws0 = _prepare(kl, B_t, N, K, need=kl.workspace_size(kl.TYPES[fmt], M, N, K))
    C0 = kl.mmq_prepared(kl.TYPES[fmt], A_t, ws0, M, N, K).cpu().numpy()
    assert O.max_rel_err(C, C0) <= TIGHT
    rows = np.sort(np.random.default_rng(M).choice(M, size=24, replace=False))
    rb = raw.size // M
    sub = np.concatenate([raw[r * rb:(r + 1) * rb] for r in rows])
    assert O.max_rel_err(C[:, rows], O.mmq_from_fp16(fmt, sub, B, len(rows), N, K, O.IDEAL)) <= TIGHT


@pytest.mark.parametrize("N", [8, 20, 40, 128])
@pytest.mark.parametrize("knob,pair", [("GQ_SGEMM_FULL", 1)])
def test_stage_schedule_same_bits(N, knob, pair, tune):
    """GQ_SGEMM_FULL (Q4_K 16/32-token tiles streaming whole super-blocks as one 144-byte image
    per row) changes how bytes are requested, not what is computed: the grouped layer and a
    single streaming-GEMM call give the bits of the half-stage schedule."""
    import kernels._lib as kl
    types, raw, x, h, items, names, inputs = _layer_items(kl, N, layer=0, seed=N + pair)
    tune(GQ_KSTREAM=0)  # both sides on the streaming GEMM
    ref = kl.mmq_grouped_prepared(items, N)
    assert ref is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    ref = [r.clone() for r in ref]
    tune(**{knob: pair})
    got = kl.mmq_grouped_prepared(items, N)
    torch.cuda.synchronize()
    for n, a, b in zip(names, ref, got):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16)), n
    one = "ffn_up"  # (a Q4_K projection)
    t, A, _, M, K, _ = items[names.index(one)]
    B = inputs[names.index(one)]
    outs = []
    for p in (0, pair):
        tune(GQ_RGEMM=0, GQ_SKINNY=0, GQ_SGEMM=1, **{knob: p})
        ws = torch.empty(kl.workspace_size(t, M, N, K), dtype=torch.uint8, device=_dev())
        kl.act_prepare(B, N, K, ws)
        outs.append(kl.mmq_prepared(t, A, ws, M, N, K))
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


def test_grouped_more_k_ranges_than_one_stream_launch_holds():
    """16 items at K = 8192 are 32 (item, K range) parts of the K-chunked stream, more than one of
    its launches takes (kKMaxParts = 24): the items past the limit go to the streaming GEMM of the
    same call instead of the call failing; every item against the oracle."""
    import kernels._lib as kl
    kl.reset_tuning()
    dev = _dev()
    N, K, M = 16, 8192, 256
    x = random_activations(N, K, seed=91)
    ws = _prepare(kl, torch.from_numpy(x).to(dev), N, K)
    raws, items = [], []
    for i in range(16):
        fmt = ("q4_k", "q6_k")[i % 2]
        qA = random_blocks(fmt, M, K, seed=100 + i)
        raws.append((fmt, qA))
        items.append((kl.TYPES[fmt], torch.from_numpy(qA.view(np.int8)).to(dev), ws, M, K, None))
    outs = kl.mmq_grouped_prepared(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    for (fmt, qA), C in zip(raws, outs):
        got = C.cpu().numpy()
        ideal = O.mmq_from_fp16(fmt, qA, x, M, N, K, O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT, (fmt, O.max_rel_err(got, ideal))
