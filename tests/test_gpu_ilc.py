"""GPU tests of the resident GEMM's in-launch split-K combine (csrc/mmq_rgemm.hip ilc_combine):
the partials summed inside the GEMM's own launch, by the tile's workgroups after a flag hand-off,
instead of by gemm_reduce_f16_kernel.  The arithmetic is the reduce kernel's (the same fp16
partials, summed in split order in fp32), so the bits must equal the two-launch form's
(GQ_RGEMM_ILC=0) on every format, token tile, activation form and ragged shape; the flags need
no zeroed memory, so workspaces full of garbage, of 0xFF, or of an earlier call's flags (another
shape on the same workspace) must not change a bit; and no poll may give up
(gq_debug_sync_timeouts stays 0).  Parity with the oracle itself: tests/test_gpu_rgemm.py and
tests/test_gpu_parity.py, which now run this form by default."""
import numpy as np
import pytest
import torch

from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

FMTS = ("q8_0", "q4_k", "q6_k")


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(_dev())


def _raw(kl, t, A, B, M, N, K, act, ws=None):
    C = torch.full((N, M), float("nan"), dtype=torch.float16, device=_dev())
    need = int(kl.lib().gq_mmq_call_workspace_size(t, kl.ACTS[act], M, N, K))
    if ws is None:
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=_dev())
    assert ws.numel() >= need
    rc = kl.lib().gq_mmq_ex(t, kl.ACTS[act], A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, M, ws.data_ptr(),
                            ws.numel(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    return C


def _prep(kl, t, A, B, M, N, K, act, ws=None):
    need = kl.workspace_size(t, M, N, K, act)
    if ws is None:
        ws = torch.empty(need, dtype=torch.uint8, device=_dev())
    kl.act_prepare(B, N, K, ws, act=act)
    C = torch.full((N, M), float("nan"), dtype=torch.float16, device=_dev())
    kl.mmq_prepared(t, A, ws, M, N, K, out=C, act=act)
    torch.cuda.synchronize()
    return C


def _two_launch(kl, fn, *a):
    kl.set_tuning("GQ_RGEMM_ILC", 0)
    try:
        return fn(kl, *a)
    finally:
        kl.set_tuning("GQ_RGEMM_ILC", 1)


# (the in-launch combine measured 0.3-0.5 us slower than the two launches on every resident shape
# and 1-4 us on the streaming ones, profiles/r06/ilc_ab_v2.txt: it is opt-in, GQ_RGEMM_ILC=1)


SHAPES = [(4096, 128, 4096), (4096, 16, 4096), (4096, 64, 4096), (4096, 33, 4096), (300, 100, 1024),
          (513, 20, 768), (1000, 40, 512), (4096, 128, 2048), (2048, 128, 8192)]


@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_ilc_bits_equal_two_launch(fmt, M, N, K, tune):
    import kernels._lib as kl
    tune(GQ_RGEMM=1, GQ_SKINNY=0, GQ_KSTREAM=0, GQ_RGEMM_ILC=1)
    t = kl.TYPES[fmt]
    A = _t(random_blocks(fmt, M, K, seed=M + K).view(np.int8))
    B = _t(random_activations(N, K, seed=N + 3 * K))
    name = kl.route_name(t, M, N, K)
    assert name.startswith("rgemm_kernel"), name
    before = kl.lib().gq_debug_sync_timeouts()
    for act in ("q8_1", "fp8"):
        for fn in (_raw, _prep):
            got = fn(kl, t, A, B, M, N, K, act)
            ref = _two_launch(kl, fn, t, A, B, M, N, K, act)
            assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), (act, fn.__name__, name)
    assert kl.lib().gq_debug_sync_timeouts() == before


def test_ilc_route_names(tune):
    import kernels._lib as kl
    kl.reset_tuning()
    assert kl.route_name(kl.GQ_Q8_0, 4096, 128, 4096) == "rgemm_kernel + gemm_reduce_f16_kernel"
    tune(GQ_RGEMM_ILC=1)
    assert kl.route_name(kl.GQ_Q8_0, 4096, 128, 4096) == "rgemm_kernel (in-launch split-K sum)"
    assert kl.route_name(kl.GQ_Q8_0, 4096, 128, 4096, prepared=True) == "rgemm_kernel (in-launch split-K sum)"


@pytest.mark.parametrize("fill", [None, 0x00, 0xFF, 0x01])
def test_ilc_workspace_contents_and_reuse(fill, tune):
    """One workspace reused by a sequence of calls of different split counts, tile counts and
    formats (its flag words then hold every kind of stale value), filled first with garbage,
    zeros, 0xFF or 0x01 bytes: every call equals its two-launch result."""
    import kernels._lib as kl
    tune(GQ_RGEMM_ILC=1)
    shapes = [("q8_0", 4096, 128, 4096), ("q4_k", 4096, 128, 2048), ("q8_0", 4096, 128, 4096),
              ("q6_k", 2048, 64, 4096), ("q8_0", 4096, 64, 4096), ("q4_k", 4096, 16, 4096), ("q8_0", 4096, 128, 4096)]
    need = max(int(kl.lib().gq_mmq_call_workspace_size(kl.TYPES[f], 0, M, N, K)) for f, M, N, K in shapes)
    ws = torch.empty(need, dtype=torch.uint8, device=_dev())
    if fill is not None:
        ws.fill_(fill)
    before = kl.lib().gq_debug_sync_timeouts()
    data = {}
    for i, (f, M, N, K) in enumerate(shapes * 2):
        t = kl.TYPES[f]
        if (f, M, N, K) not in data:
            data[(f, M, N, K)] = (_t(random_blocks(f, M, K, seed=i).view(np.int8)), _t(random_activations(N, K, seed=i)))
        A, B = data[(f, M, N, K)]
        got = _raw(kl, t, A, B, M, N, K, "q8_1", ws=ws)
        ref = _two_launch(kl, _raw, t, A, B, M, N, K, "q8_1")
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), (i, f, M, N, K)
    assert kl.lib().gq_debug_sync_timeouts() == before


def test_ilc_graph_replays_and_back_to_back(tune):
    """The headline call captured 8 times in one graph (back-to-back launches on one workspace,
    each advancing the tiles' nonces) and the graph replayed 5 times, C poisoned between
    replays: every output equals the eager two-launch result."""
    import kernels._lib as kl
    tune(GQ_RGEMM_ILC=1)
    t, M, N, K = kl.GQ_Q8_0, 4096, 128, 4096
    A = _t(random_blocks("q8_0", M, K, seed=5).view(np.int8))
    B = _t(random_activations(N, K, seed=6))
    ref = _two_launch(kl, _raw, t, A, B, M, N, K, "q8_1")
    need = int(kl.lib().gq_mmq_call_workspace_size(t, 0, M, N, K))
    ws = torch.empty(need, dtype=torch.uint8, device=_dev())
    Cs = [torch.empty(N, M, dtype=torch.float16, device=_dev()) for _ in range(8)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def call(C):
        rc = kl.lib().gq_mmq_ex(t, 0, A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, K, M, ws.data_ptr(), need,
                                torch.cuda.current_stream().cuda_stream)
        assert rc == 0

    with torch.cuda.stream(s):
        call(Cs[0])
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for C in Cs:
            call(C)
    before = kl.lib().gq_debug_sync_timeouts()
    for _ in range(5):
        for C in Cs:
            C.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        for C in Cs:
            assert torch.equal(C.view(torch.int16), ref.view(torch.int16))
    assert kl.lib().gq_debug_sync_timeouts() == before


SGEMM_SHAPES = [("q6_k", 28672, 128, 8192), ("q6_k", 8192, 128, 28672), ("q4_k", 11008, 128, 4096),
                ("q8_0", 11008, 64, 4096), ("q4_k", 4096, 128, 11008), ("q6_k", 3000, 40, 2048), ("q4_k", 9000, 17, 4096)]


@pytest.mark.parametrize("fmt,M,N,K", SGEMM_SHAPES)
def test_sgemm_ilc_bits_equal_two_launch(fmt, M, N, K, tune):
    """The streaming GEMM's in-launch combine (sgemm_kernel, its splits chosen to fill one round
    of the chip): bit for bit the two-launch form, prepared and raw calls."""
    import kernels._lib as kl
    tune(GQ_SGEMM=1, GQ_RGEMM=0, GQ_SKINNY=0, GQ_KSTREAM=0, GQ_RGEMM_ILC=1)
    t = kl.TYPES[fmt]
    name = kl.route_name(t, M, N, K, prepared=True)
    assert name.startswith("sgemm_kernel"), name
    A = _t(random_blocks(fmt, M, K, seed=M + 7).view(np.int8))
    B = _t(random_activations(N, K, seed=N + 11))
    before = kl.lib().gq_debug_sync_timeouts()
    for fn in (_prep, _raw):
        got = fn(kl, t, A, B, M, N, K, "q8_1")
        ref = _two_launch(kl, fn, t, A, B, M, N, K, "q8_1")
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16)), (fn.__name__, name)
    assert kl.lib().gq_debug_sync_timeouts() == before


@pytest.mark.parametrize("N", [40, 64, 96, 128])
def test_grouped_stream_k_ilc_bits_equal_two_launch(N, tune):
    """The grouped streaming GEMM's stream-K plan (a 7B Q4_K_M layer's seven projections) with
    its split tiles summed in-launch: every projection bit for bit the reduce_grouped_kernel form."""
    import kernels._lib as kl
    from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
    tune(GQ_RGEMM_ILC=1)
    dev = _dev()
    types = q4_k_m_layer_types(0, 32)
    x = _t(random_activations(N, 4096, seed=N))
    h = _t(random_activations(N, 11008, seed=N + 1))
    wx = torch.empty(kl.workspace_size(kl.GQ_Q4_K, 256, N, 4096), dtype=torch.uint8, device=dev)
    wh = torch.empty(kl.workspace_size(kl.GQ_Q4_K, 256, N, 11008), dtype=torch.uint8, device=dev)
    kl.act_prepare(x, N, 4096, wx)
    kl.act_prepare(h, N, 11008, wh)
    items = []
    for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items()):
        A = _t(random_blocks(types[n], M, K, seed=i).view(np.int8))
        items.append((kl.TYPES[types[n]], A, wh if K == 11008 else wx, M, K, None))
    before = kl.lib().gq_debug_sync_timeouts()
    got = kl.mmq_grouped_prepared(items, N)
    assert got is not None, kl.lib().gq_last_error()
    torch.cuda.synchronize()
    kl.set_tuning("GQ_RGEMM_ILC", 0)
    ref = kl.mmq_grouped_prepared(items, N)
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert kl.lib().gq_debug_sync_timeouts() == before
