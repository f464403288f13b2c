"""Every default route on a non-default stream and inside a captured HIP graph.

Round 4's split-K GEMMs launched their reduce on the legacy default stream (the launcher's
stream argument defaulted to nullptr): on torch's default stream the reduce happened to be
ordered after the GEMM, so every parity test passed, but on a side stream it could read the
partials early and under graph capture it ran once, eagerly, outside the graph -- replays never
wrote C.  Here C is filled with NaN before each replay and must come back equal, bit for bit, to
the eager call on the default stream; each shape names the route it exercises."""
import numpy as np
import pytest
import torch

from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

CASES = [
    # fmt, M, N, K, the route's first kernel (gq_debug_route)
    ("q8_0", 4096, 128, 4096, "rgemm_kernel"),    # the headline: 16 splits + reduce
    ("q4_k", 4096, 16, 4096, "rgemm_kernel"),     # (prepared: the K-chunked stream)
    ("q6_k", 8192, 16, 4096, "kstream_kernel"),   # raw and prepared: the K-chunked stream (8192+ rows)
    ("q6_k", 11008, 128, 4096, "sgemm_kernel"),   # streaming GEMM, split-K + reduce
    ("q4_k", 28672, 16, 8192, "skinny_kernel"),
    ("q6_k", 4096, 1, 4096, "stream_decode_kernel"),
    ("q4_k", 4096, 4, 11008, "gemv_kernel"),
    ("q8_0", 1024, 800, 1024, "dequant_kernel"),  # hipBLASLt (warmed before capture)
]


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


@pytest.mark.parametrize("prepared", [False, True])
@pytest.mark.parametrize("fmt,M,N,K,first", CASES)
def test_side_stream_and_graph_replay(fmt, M, N, K, first, prepared):
    import kernels._lib as kl
    dev = _dev()
    t = kl.TYPES[fmt]
    route = kl.route_name(t, M, N, K, prepared=prepared)
    # (a prepared call of a decode shape runs the same one-launch decode on the workspace's copy
    # of the activations -- round 5; it read the SOA form through the GEMV before)
    if prepared and N <= 32 and first == "rgemm_kernel":
        first = "kstream_kernel"  # (prepared 5..32 tokens: the K-chunked stream, one launch)
    assert route.startswith(first), route
    A = torch.from_numpy(random_blocks(fmt, M, K, seed=M + N).view(np.int8)).to(dev)
    B = torch.from_numpy(random_activations(N, K, seed=K + N)).to(dev)
    need = kl.workspace_size(t, M, N, K)

    def run(C, ws):
        if prepared:
            kl.act_prepare(B, N, K, ws)
            kl.mmq_prepared(t, A, ws, M, N, K, out=C)
        else:
            kl.mmq(t, A, B, M, N, K, out=C, workspace=ws)

    ref = torch.empty((N, M), dtype=torch.float16, device=dev)
    run(ref, torch.empty(need, dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()
    assert torch.isfinite(ref.float()).all()

    s = torch.cuda.Stream()
    C = torch.full((N, M), float("nan"), dtype=torch.float16, device=dev)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(C, ws)  # eager on a non-blocking side stream
    s.synchronize()
    assert torch.equal(C.view(torch.int16), ref.view(torch.int16))

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run(C, ws)
    for _ in range(3):
        C.fill_(float("nan"))
        ws.fill_(0xFF)  # (stale partials / activations would show)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), ref.view(torch.int16))


def test_grouped_gemm_and_decode_graph_replay():
    """The grouped streaming GEMM (one launch + its reduce) and the grouped decode, captured
    together on a side stream: replays reproduce the eager outputs bit for bit."""
    import kernels._lib as kl
    dev = _dev()
    K = 4096
    specs = [("q4_k", 4096), ("q6_k", 4096), ("q8_0", 1024)]
    As = [torch.from_numpy(random_blocks(f, M, K, seed=M + i).view(np.int8)).to(dev) for i, (f, M) in enumerate(specs)]
    outs = {}
    for N in (16, 2):
        B = torch.from_numpy(random_activations(N, K, seed=N)).to(dev)
        ws = torch.empty(max(kl.workspace_size(kl.TYPES[f], M, N, K) for f, M in specs), dtype=torch.uint8, device=dev)
        Cs = [torch.empty((N, M), dtype=torch.float16, device=dev) for _, M in specs]

        def run():
            if N >= 5:
                kl.act_prepare(B, N, K, ws)
                r = kl.mmq_grouped_prepared([(kl.TYPES[f], A, ws, M, K, C) for (f, M), A, C in zip(specs, As, Cs)], N)
            else:
                r = kl.mmq_grouped([(kl.TYPES[f], A, B, M, K, C) for (f, M), A, C in zip(specs, As, Cs)], N)
            assert r is not None

        run()
        torch.cuda.synchronize()
        refs = [C.clone() for C in Cs]
        for (f, M), A, R in zip(specs, As, refs):  # each part equals its own call within the GEMM gate
            solo = kl.mmq(kl.TYPES[f], A, B, M, N, K)
            d = (solo.float() - R.float()).abs().max().item()
            assert d <= 4e-3 * max(solo.float().abs().max().item(), 1e-6)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            run()
        for _ in range(2):
            for C in Cs:
                C.fill_(float("nan"))
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            for C, R in zip(Cs, refs):
                assert torch.equal(C.view(torch.int16), R.view(torch.int16))
        outs[N] = refs
