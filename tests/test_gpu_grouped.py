"""GPU tests of the grouped decode launch (gq_mmq_grouped, csrc/mmq_decode.hip
stream_decode_grouped_kernel): several matrices of their own types, activations and outputs in
one launch at 1..4 tokens.  Each projection vs the oracle (sampled rows, IDEAL at the decode
tolerance and the reference's 1% gate vs EXACT) and bit for bit vs its own gq_mmq call; the
Llama-7B Q4_K_M layer through LayerMix grouped and ungrouped; what is not a grouped shape is
refused without launching.  The grouped activation prepare (gq_act_prepare_grouped): the same
workspace bytes as one gq_act_prepare per input, and LayerMix at 5+ tokens (one prepare launch
for the layer) bit-identical to one mmq() per projection."""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT_DEC = 3e-3  # int8 x int8 dots, fp32 block scaling: vs IDEAL (as tests/test_gpu_parity.py)


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _layer(types, seed=0):
    from gguf import LLAMA_LAYER_SHAPES
    dev = _dev()
    raw = {n: random_blocks(types[n], M, K, seed=seed + i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    dev_w = {n: torch.from_numpy(raw[n].view(np.int8)).to(dev) for n in raw}
    return raw, dev_w


@pytest.mark.parametrize("N", [1, 2, 3, 4])
@pytest.mark.parametrize("layer", [0, 5])
def test_grouped_llama_layer_bitexact(N, layer):
    """The seven Llama-7B projections (Q4_K_M types of layer `layer`; layer 0: attn_v and
    ffn_down in Q6_K) in one grouped call: every output bit-identical to its own mmq() call, and
    sampled rows against the oracle.  At 3-4 tokens a Q4_K ffn_down (K = 11008) has no one-launch
    decode form (its 4 tokens' activations do not fit LDS beside the ring; its own call is the
    GEMV path), so layer 5's group is refused there."""
    import kernels._lib as kl
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    dev = _dev()
    types = q4_k_m_layer_types(layer, 32)
    raw, A = _layer(types, seed=100 * layer)
    x = random_activations(N, 4096, seed=1 + N)
    h = random_activations(N, 11008, seed=2 + N)
    xt, ht = torch.from_numpy(x).to(dev), torch.from_numpy(h).to(dev)
    items, names = [], []
    for n, (M, K) in LLAMA_LAYER_SHAPES.items():
        names.append(n)
        items.append((kl.TYPES[types[n]], A[n], ht if K == 11008 else xt, M, K, None))
    outs = kl.mmq_grouped(items, N)
    if N >= 3 and types["ffn_down"] == "q4_k":
        assert outs is None
        return
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    rng = np.random.default_rng(N)
    for n, C in zip(names, outs):
        M, K = LLAMA_LAYER_SHAPES[n]
        solo = kl.mmq(kl.TYPES[types[n]], A[n], ht if K == 11008 else xt, M, N, K)
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), solo.view(torch.int16)), n
        rows = np.sort(rng.choice(M, size=24, replace=False))
        rb = raw[n].size // M
        sub = np.concatenate([raw[n][r * rb:(r + 1) * rb] for r in rows])
        B = h if K == 11008 else x
        got = C.cpu().numpy()[:, rows]
        ideal = O.mmq_from_fp16(types[n], sub, B, len(rows), N, K, O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT_DEC, n
        exact = O.mmq_from_fp16(types[n], sub, B, len(rows), N, K, O.EXACT)
        assert O.allclose(exact, got, 0.01), n


def test_grouped_mixed_formats_strides():
    """Q8_0, Q4_K and Q6_K items with ragged rows, K not a multiple of 256 (Q8_0), a shared
    activation tensor, a strided activation view and outputs written into column ranges of one
    wide buffer (ldc > M): bit-identical to the per-item calls, nothing outside the ranges touched."""
    import kernels._lib as kl
    dev = _dev()
    N = 3
    specs = [("q8_0", 333, 1056), ("q4_k", 1000, 2048), ("q6_k", 257, 1536), ("q4_k", 64, 2048), ("q8_0", 4096, 4096)]
    X = {K: torch.from_numpy(random_activations(N, K, seed=K)).to(dev) for K in {s[2] for s in specs}}
    wide = torch.from_numpy(random_activations(N, 2 * 2048, seed=7)).to(dev)
    X[2048] = wide[:, 1000:1000 + 2048]  # row stride 4096
    width = sum(M for _, M, _ in specs) + 5
    buf = torch.full((N, width), -7.0, dtype=torch.float16, device=dev)
    items, col = [], 0
    qs = []
    for i, (fmt, M, K) in enumerate(specs):
        qA = torch.from_numpy(random_blocks(fmt, M, K, seed=i).view(np.int8)).to(dev)
        qs.append(qA)
        items.append((kl.TYPES[fmt], qA, X[K], M, K, buf[:, col:col + M]))
        col += M
    outs = kl.mmq_grouped(items, N)
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    col = 0
    for (fmt, M, K), qA in zip(specs, qs):
        solo = kl.mmq(kl.TYPES[fmt], qA, X[K], M, N, K)
        torch.cuda.synchronize()
        assert torch.equal(buf[:, col:col + M].view(torch.int16), solo.view(torch.int16)), fmt
        col += M
    assert torch.all(buf[:, col:] == -7.0)


def test_grouped_refuses_non_decode_shapes():
    """N = 33 (past the grouped forms: decode 1..4, K-chunked stream 5..32), M = 40 at 8 tokens (not
    whole 16-row items) and an item whose activations do not fit LDS: refused (None), nothing
    launched, the output untouched; mmq() per item is the caller's path then."""
    import kernels._lib as kl
    dev = _dev()
    qA = torch.from_numpy(random_blocks("q4_k", 64, 1024, seed=1).view(np.int8)).to(dev)
    for N, K in ((33, 1024),):
        B = torch.from_numpy(random_activations(N, K, seed=2)).to(dev)
        out = torch.full((N, 64), 3.0, dtype=torch.float16, device=dev)
        assert kl.mmq_grouped([(kl.GQ_Q4_K, qA, B, 64, K, out)], N) is None
        torch.cuda.synchronize()
        assert torch.all(out == 3.0)
    qC = torch.from_numpy(random_blocks("q4_k", 40, 1024, seed=5).view(np.int8)).to(dev)
    B = torch.from_numpy(random_activations(8, 1024, seed=6)).to(dev)
    assert kl.mmq_grouped([(kl.GQ_Q4_K, qC, B, 40, 1024, None)], 8) is None
    K = 131072  # 4 tokens x 128K codes: no room in LDS beside the ring
    qB = torch.from_numpy(random_blocks("q8_0", 16, K, seed=3).view(np.int8)).to(dev)
    B = torch.from_numpy(random_activations(4, K, seed=4)).to(dev)
    assert kl.mmq_grouped([(kl.GQ_Q8_0, qB, B, 16, K, None)], 4) is None


@pytest.mark.parametrize("N", [1, 2, 4])
def test_layer_mix_grouped_matches_ungrouped(N):
    """LayerMix at decode sizes: the grouped launch (default) gives the same bits as one call per
    projection set; `out` buffers are honoured for fused projections too."""
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    _, A = _layer(types, seed=3)
    lins = {n: GGUFLinear(types[n], A[n], M, K) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    g, u = LayerMix(lins, grouped=True), LayerMix(lins, grouped=False)  # (True: grouped at 1..4 tokens)
    x = torch.from_numpy(random_activations(N, 4096, seed=5)).to(dev)
    a = torch.from_numpy(random_activations(N, 4096, seed=6)).to(dev)
    y = torch.from_numpy(random_activations(N, 4096, seed=7)).to(dev)
    h = torch.from_numpy(random_activations(N, 11008, seed=8)).to(dev)
    out = {n: torch.empty(N, M, dtype=torch.float16, device=dev) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    rg = g.forward(x, h, attn=a, x_ffn=y, out=out)
    ru = u.forward(x, h, attn=a, x_ffn=y)
    torch.cuda.synchronize()
    for n in LLAMA_LAYER_SHAPES:
        assert rg[n].data_ptr() == out[n].data_ptr(), n
        assert torch.equal(rg[n].view(torch.int16), ru[n].view(torch.int16)), n


@pytest.mark.parametrize("act", ["q8_1", "fp8"])
def test_act_prepare_grouped_matches_individual(act):
    """gq_act_prepare_grouped writes exactly the bytes gq_act_prepare writes per item: GEMM-form
    items (N >= 5, several per launch, more than one launch's 8), a strided activation view, a
    decode-form item (N <= 4, prepared on its own; fp8: grouped like the rest), an empty item."""
    import kernels._lib as kl
    dev = _dev()
    specs = [(8, 4096), (8, 11008), (3, 2048), (64, 1024), (0, 512), (16, 4096), (5, 2816), (128, 4096),
             (7, 32), (9, 256), (12, 4096), (6, 11008), (1, 4096), (2, 768)]
    if act == "fp8":  # (K % 256 == 0)
        specs = [(N, K) for N, K in specs if K % 256 == 0]
    wide = torch.from_numpy(random_activations(8, 4096 + 512, seed=77)).to(dev)
    items, ref = [], []
    for i, (N, K) in enumerate(specs):
        B = wide[:, 256:256 + K] if i == 0 else torch.from_numpy(random_activations(N, K, seed=i)).to(dev)
        need = kl.workspace_size(kl.GQ_Q4_K, 256, N, K, act) if N else 16
        ws, ws_ref = (torch.zeros(need, dtype=torch.uint8, device=dev) for _ in range(2))
        items.append((B, N, K, ws))
        if N:
            kl.act_prepare(B, N, K, ws_ref, act=act)
        ref.append(ws_ref)
    kl.act_prepare_grouped(items, act=act)
    torch.cuda.synchronize()
    for (B, N, K, ws), ws_ref in zip(items, ref):
        assert torch.equal(ws, ws_ref), (N, K)


@pytest.mark.parametrize("N,act", [(5, "q8_1"), (8, "q8_1"), (16, "q8_1"), (64, "q8_1"), (128, "q8_1"),
                                   (1, "fp8"), (2, "fp8"), (3, "fp8"), (8, "fp8"), (128, "fp8")])
def test_layer_mix_prepared_matches_per_call(N, act, tune):
    """LayerMix from 5 tokens (the four inputs quantized in one gq_act_prepare_grouped launch, every
    projection prepared; grouped=False: one launch per projection, not the grouped GEMM of
    tests/test_gpu_gemm_grouped.py): unfused, every projection bit-identical to its own mmq(); fused (q+k and
    gate+up as one taller matrix, whose split-K plan may differ from the parts') within the GEMM
    tolerance of the unfused result.  GQ_KSTREAM=1: at 5..32 tokens the default routes a prepared call
    to the K-chunked stream but a raw one to the resident GEMM (a different fp32 order over K; see
    test_layer_mix_default_routes_within_tolerance), so both sides are pinned to the stream here."""
    import kernels._lib as kl
    tune(GQ_KSTREAM=1)
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    _, A = _layer(types, seed=9)
    lins = {n: GGUFLinear(types[n], A[n], M, K) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    x = torch.from_numpy(random_activations(N, 4096, seed=15)).to(dev)
    a = torch.from_numpy(random_activations(N, 4096, seed=16)).to(dev)
    y = torch.from_numpy(random_activations(N, 4096, seed=17)).to(dev)
    h = torch.from_numpy(random_activations(N, 11008, seed=18)).to(dev)
    res = LayerMix(lins, act=act, fuse=False, grouped=False).forward(x, h, attn=a, x_ffn=y)
    fused = LayerMix(lins, act=act).forward(x, h, attn=a, x_ffn=y)
    inp = {"attn_q": x, "attn_k": x, "attn_v": x, "attn_output": a, "ffn_gate": y, "ffn_up": y, "ffn_down": h}
    torch.cuda.synchronize()
    for n, (M, K) in LLAMA_LAYER_SHAPES.items():
        solo = kl.mmq(kl.TYPES[types[n]], A[n], inp[n], M, N, K, act=act)
        torch.cuda.synchronize()
        assert torch.equal(res[n].view(torch.int16), solo.view(torch.int16)), n
        assert O.max_rel_err(fused[n].cpu().numpy(), solo.cpu().numpy()) <= 4e-3, n


@pytest.mark.parametrize("N", [8, 16])
def test_layer_mix_default_routes_within_tolerance(N):
    """Default routes at 16 tokens: LayerMix's prepared projections (K-chunked stream) against each
    projection's raw mmq() (resident GEMM) -- the same products summed in another fp32 order, so
    within the GEMM tolerance (4e-3 relative), not bit for bit."""
    import kernels._lib as kl
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    from kernels.layer_mix import GGUFLinear, LayerMix
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    _, A = _layer(types, seed=19)
    lins = {n: GGUFLinear(types[n], A[n], M, K) for n, (M, K) in LLAMA_LAYER_SHAPES.items()}
    x, a, y = (torch.from_numpy(random_activations(N, 4096, seed=s)).to(dev) for s in (25, 26, 27))
    h = torch.from_numpy(random_activations(N, 11008, seed=28)).to(dev)
    res = LayerMix(lins, fuse=False, grouped=False).forward(x, h, attn=a, x_ffn=y)
    inp = {"attn_q": x, "attn_k": x, "attn_v": x, "attn_output": a, "ffn_gate": y, "ffn_up": y, "ffn_down": h}
    for n, (M, K) in LLAMA_LAYER_SHAPES.items():
        solo = kl.mmq(kl.TYPES[types[n]], A[n], inp[n], M, N, K)
        torch.cuda.synchronize()
        assert O.max_rel_err(res[n].cpu().numpy(), solo.cpu().numpy()) <= 4e-3, n


@pytest.mark.parametrize("N", [1, 2, 3])
@pytest.mark.parametrize("layer", [0, 5])
def test_grouped_llama_layer_fp8(N, layer):
    """The fp8 activation variant's grouped decode (gq_mmq_grouped_ex, GQ_ACT_FP8_E4M3: the decode
    kernel's FP8 form, fp16 x~ and v_dot2): the seven Llama-7B projections in one launch, each
    bit-identical to its own mmq(act="fp8") call and within the fp8 tolerance of the fp8-exact
    product; refused (nothing launched) from 3 tokens (no one-launch fp8 decode form).  At 2
    tokens the ffn_down (K = 11008) fits since its x~ image carries no quarter sums there
    (gguf_dot.hpp dot_unit_h NS)."""
    import kernels._lib as kl
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    dev = _dev()
    types = q4_k_m_layer_types(layer, 32)
    raw, A = _layer(types, seed=100 * layer + 1)
    x = random_activations(N, 4096, seed=3 + N)
    h = random_activations(N, 11008, seed=4 + N)
    xt, ht = torch.from_numpy(x).to(dev), torch.from_numpy(h).to(dev)
    items, names = [], []
    for n, (M, K) in LLAMA_LAYER_SHAPES.items():
        names.append(n)
        items.append((kl.TYPES[types[n]], A[n], ht if K == 11008 else xt, M, K, None))
    outs = kl.mmq_grouped(items, N, act="fp8")
    if N >= 3:
        assert outs is None
        return
    assert outs is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    rng = np.random.default_rng(N + 7)
    for n, C in zip(names, outs):
        M, K = LLAMA_LAYER_SHAPES[n]
        solo = kl.mmq(kl.TYPES[types[n]], A[n], ht if K == 11008 else xt, M, N, K, act="fp8")
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), solo.view(torch.int16)), n
        rows = np.sort(rng.choice(M, size=24, replace=False))
        rb = raw[n].size // M
        sub = np.concatenate([raw[n][r * rb:(r + 1) * rb] for r in rows])
        ideal = O.mmq_fp8_ideal(types[n], sub, h if K == 11008 else x, len(rows), N, K)
        assert O.max_rel_err(C.cpu().numpy()[:, rows], ideal) <= 4e-3, n


def test_q8_0_long_k_one_token_grouped_and_solo():
    """Q8_0 at one token with 28672 < K <= 32768 (K = 29568, Qwen2-72B's ffn_down): the decode
    pick() once chose a cached-chunk count (8) that no kernel instantiates -- the grouped launch
    wrote nothing and returned success, the single launch ran the 2-token kernel.  Both forms
    now match the oracle on sampled rows, and each other bit for bit."""
    import kernels._lib as kl
    dev = _dev()
    M, K, N = 512, 29568, 1
    raw = random_blocks("q8_0", M, K, seed=11)
    qA = torch.from_numpy(raw.view(np.int8)).to(dev)
    x = random_activations(N, K, seed=12)
    xt = torch.from_numpy(x).to(dev)
    solo = kl.mmq(kl.GQ_Q8_0, qA, xt, M, N, K)
    out = torch.full((N, M), float("nan"), dtype=torch.float16, device=dev)
    res = kl.mmq_grouped([(kl.GQ_Q8_0, qA, xt, M, K, out)], N)
    torch.cuda.synchronize()
    rows = np.arange(0, M, 37)
    rb = raw.size // M
    sub = np.concatenate([raw[r * rb:(r + 1) * rb] for r in rows])
    ideal = O.mmq_from_fp16("q8_0", sub, x, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(solo.cpu().numpy()[:, rows], ideal) <= TIGHT_DEC
    if res is not None:  # grouped form taken: it must have written every output
        assert torch.equal(out.view(torch.int16), solo.view(torch.int16))
