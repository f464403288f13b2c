"""GPU parity of the alternative paths behind the drop-in API, each against the oracle on the
same inputs (run with `pytest -m gpu` on an MI355X):

  * the Q8_0 int8-MFMA GEMM (GQ_GEMM_I8=1: q8_1 codes x weight codes on
    v_mfma_i32_16x16x32_i8, per-block fp32 scaling) -- exact integer dots, so it is held to
    the decode path's tight gate TIGHT_I8 = 1.5e-3 of max|C| against oracle IDEAL, and to the
    reference's 1% gate against oracle EXACT (kernels/cpu_impls arithmetic);
  * the prepared form (gq_act_prepare + gq_mmq_prepared) at every token count, including the
    N <= 4 decode-shaped kernel the fused gq_mmq path does not use;
  * row-sharded MMQ (dist/row_shard.py): the Q6_K Llama-70B matrices split into
    G = 2, 4, 8 row shards, each shard run through RowShardedMMQ.local on this device,
    assembled, compared with the oracle and bit for bit with the unsharded call.
"""
import numpy as np
import pytest
import torch

import oracle as O
from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu

TIGHT_I8 = 1.5e-3
TIGHT_GEMV = 1.5e-3
TIGHT_GEMM = 4e-3


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _run(fmt, qA, B, M, N, K):
    from kernels._lib import TYPES, mmq
    dev = _dev()
    A_t = torch.from_numpy(np.ascontiguousarray(qA).view(np.int8)).to(dev)
    B_t = torch.from_numpy(np.ascontiguousarray(B)).to(dev)
    C = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    return C.cpu().numpy()


@pytest.mark.parametrize("M,N,K,splits", [(128, 5, 256, None), (200, 16, 512, None), (130, 33, 768, "1"),
                                          (64, 64, 1024, None), (300, 100, 2048, "3"), (256, 128, 4096, None),
                                          (96, 128, 4096, "8"), (1000, 77, 1280, None)])
def test_q8_0_int8_mfma_gemm(M, N, K, splits, tune):
    tune(GQ_GEMM_I8=1)  # (the int8 form lives in the LDS-DMA GEMM)
    if splits:
        tune(GQ_GEMM_SPLITS=splits)
    qA = random_blocks("q8_0", M, K, seed=M + 3 * N)
    B = random_activations(N, K, seed=K + N)
    got = _run("q8_0", qA, B, M, N, K)
    ideal = O.mmq_from_fp16("q8_0", qA, B, M, N, K, O.IDEAL)
    err = O.max_rel_err(got, ideal)
    assert err <= TIGHT_I8, (M, N, K, err)
    exact = O.mmq_from_fp16("q8_0", qA, B, M, N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


@pytest.mark.parametrize("M,N,K", [(4096, 128, 4096), (11008, 128, 4096), (4096, 300, 11008)])
def test_q8_0_int8_mfma_full_size(M, N, K, tune):
    """The int8 form at BASELINE sizes (configs[1]: 4096^2 x128; the 7B up/down shapes), every
    token, 48 sampled rows against the oracle (IDEAL at the tight int8 gate, EXACT at the
    reference's 1%)."""
    from kernels._lib import TYPES, mmq
    tune(GQ_GEMM_I8=1)
    dev = _dev()
    qA = random_blocks("q8_0", M, K, seed=M + K)
    B = random_activations(N, K, seed=N + 11)
    C = mmq(TYPES["q8_0"], torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev), M, N, K)
    torch.cuda.synchronize()
    rows = np.sort(np.random.default_rng(M).choice(M, size=48, replace=False))
    rb = qA.size // M
    sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
    got = C.cpu().numpy()[:, rows]
    ideal = O.mmq_from_fp16("q8_0", sub, B, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT_I8
    exact = O.mmq_from_fp16("q8_0", sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


def test_q8_0_int8_mfma_golden(golden, tune):
    """Every golden case of the reference through the int8 form (cases with N >= 5 run it)."""
    tune(GQ_GEMM_I8=1)
    for c in golden["q8_0"]:
        got = _run("q8_0", c["qA"], c["B"], c["M"], c["N"], c["K"])
        if c["kind"] != "tiny":
            assert O.allclose(c["C"], got, 0.01), (c["i"], c["kind"])
        ideal = O.mmq("q8_0", c["qA"], c["qB"], c["M"], c["N"], c["K"], O.IDEAL)
        assert O.max_rel_err(got, ideal) <= TIGHT_I8, (c["i"], c["kind"])


@pytest.mark.parametrize("fmt", ("q8_0", "q4_k", "q6_k"))
@pytest.mark.parametrize("N", (1, 2, 3, 4, 5, 16, 128))
def test_prepared_matches_oracle(fmt, N):
    """gq_act_prepare + gq_mmq_prepared (the LayerMix form) at every path's token counts."""
    import kernels._lib as kl
    dev = _dev()
    M, K = 160, 1024
    qA = random_blocks(fmt, M, K, seed=N + 5)
    B = random_activations(N, K, seed=N + 6)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(B).to(dev)
    g = kl.TYPES[fmt]
    ws = torch.empty(kl.workspace_size(g, M, N, K), dtype=torch.uint8, device=dev)
    kl.act_prepare(B_t, N, K, ws)
    C = kl.mmq_prepared(g, A_t, ws, M, N, K).cpu().numpy()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(C, ideal) <= (TIGHT_GEMV if N <= 4 else TIGHT_GEMM), (fmt, N)
    full = kl.mmq(g, A_t, B_t, M, N, K).cpu().numpy()
    assert O.max_rel_err(C, full) <= 2 * TIGHT_GEMM


@pytest.mark.parametrize("M,K", [(28672, 8192), (8192, 28672)])
@pytest.mark.parametrize("G", (2, 4, 8))
@pytest.mark.parametrize("N", (1, 128))
def test_row_sharded_q6_k_70b(M, K, G, N, tune):
    """Config 4: Q6_K Llama-70B ffn_gate/up (28672x8192) and ffn_down (8192x28672) split into G
    row shards (zero-copy byte ranges), each run through RowShardedMMQ.local, assembled as the
    all-gather would; vs the unsharded call (bit for bit, split-K off on both) and the oracle
    on sampled rows."""
    from dist.row_shard import RowShardedMMQ, shard_bytes
    from kernels._lib import TYPES, mmq
    tune(GQ_GEMM_SPLITS=1)
    dev = _dev()
    qA = random_blocks("q6_k", M, K, seed=M + G)
    B = random_activations(N, K, seed=N + K)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(B).to(dev)
    full = mmq(TYPES["q6_k"], A_t, B_t, M, N, K)
    slabs = []
    for g in range(G):
        part = RowShardedMMQ("q6_k", shard_bytes("q6_k", A_t, M, K, G, g), M, K, world=G, rank=g)
        slabs.append(part.local(B_t, N))
    gathered = torch.stack(slabs)  # what all_gather_into_tensor leaves: (G, N, R)
    C = part.assemble(gathered)
    torch.cuda.synchronize()
    assert C.shape == (N, M)
    assert torch.equal(C.view(torch.int16), full.view(torch.int16))
    rows = np.sort(np.random.default_rng(G).choice(M, size=40, replace=False))
    row_bytes = qA.size // M
    sub = np.concatenate([qA[r * row_bytes:(r + 1) * row_bytes] for r in rows])
    ideal = O.mmq_from_fp16("q6_k", sub, B, len(rows), N, K, O.IDEAL)
    got = C.cpu().numpy()[:, rows]
    assert O.max_rel_err(got, ideal) <= (TIGHT_GEMV if N <= 4 else TIGHT_GEMM)
    exact = O.mmq_from_fp16("q6_k", sub, B, len(rows), N, K, O.EXACT)
    assert O.allclose(exact, got, 0.01)


@pytest.mark.parametrize("fmt", ("q8_0", "q4_k", "q6_k"))
def test_gemm_chunked_launches_bit_exact(fmt, tune):
    """The GEMM path's 32-bit offset guard: calls over GQ_GEMM_MAX_BYTES of weights or of fp16
    activations run as row x token chunks; with a small limit (many chunks in both dims) the
    result equals the one-launch result bit for bit (split-K off on both)."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    M, N, K = 700, 300, 1024
    qA = random_blocks(fmt, M, K, seed=9)
    B = random_activations(N, K, seed=10)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(B).to(dev)
    tune(GQ_GEMM_SPLITS=1, GQ_BLAS_MIN_TOKENS=0)
    one = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    tune(GQ_GEMM_MAX_BYTES=256 * 1024)  # 256 rows / 128 tokens per launch
    many = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(one.view(torch.int16), many.view(torch.int16))
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(many.cpu().numpy(), ideal) <= TIGHT_GEMM


def test_gemm_weights_over_4gib():
    """A 4.5 GB Q8_0 weight tensor (131072 x 32768) at 16 tokens: two row chunks; sampled rows
    from both against the oracle."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    M, N, K = 131072, 16, 32768
    row_bytes = K // 32 * 34
    A_t = torch.empty(M * row_bytes, dtype=torch.int8, device=dev)
    rows = np.array([0, 5, 70000, 100001, M - 1])
    sub = random_blocks("q8_0", len(rows), K, seed=21)
    base = torch.from_numpy(random_blocks("q8_0", 64, K, seed=22).view(np.int8)).to(dev)
    for i in range(0, M, 64):
        A_t[i * row_bytes:(i + 64) * row_bytes] = base
    for j, r in enumerate(rows):
        A_t[r * row_bytes:(r + 1) * row_bytes] = torch.from_numpy(sub[j * row_bytes:(j + 1) * row_bytes].view(np.int8)).to(dev)
    B = random_activations(N, K, seed=23)
    C = mmq(TYPES["q8_0"], A_t, torch.from_numpy(B).to(dev), M, N, K)
    torch.cuda.synchronize()
    got = C[:, torch.from_numpy(rows).to(dev)].cpu().numpy()
    ideal = O.mmq_from_fp16("q8_0", sub, B, len(rows), N, K, O.IDEAL)
    assert O.max_rel_err(got, ideal) <= TIGHT_GEMM
    del A_t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("partial", ("f16", "f32"))
def test_split_k_partials_huge_cancelling_sums(partial, tune):
    """Split-K partial sums far outside fp16's range whose total cancels to ~0: the second half
    of K repeats the first half's weights against negated activations.  fp16 partials carry a
    per-wave power-of-two scale, so neither form overflows (no inf/NaN) and both cancel."""
    from kernels._lib import TYPES, mmq
    tune(GQ_GEMM_PARTIAL=int(partial == "f32"), GQ_GEMM_SPLITS=8)
    dev = _dev()
    M, N, K = 256, 128, 4096
    half = random_blocks("q8_0", M, K // 2, seed=31).reshape(M, -1)
    qA = np.concatenate([half, half], axis=1).reshape(-1)
    x = (random_activations(N, K // 2, seed=32).astype(np.float32) * 20000).clip(-60000, 60000).astype(np.float16)
    B = np.concatenate([x, -x], axis=1)
    C = mmq(TYPES["q8_0"], torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev), M, N, K)
    torch.cuda.synchronize()
    got = C.float().cpu().numpy()
    assert np.isfinite(got).all()
    first = np.abs(O.mmq_from_fp16("q8_0", half.reshape(-1), x, M, N, K // 2, O.IDEAL).astype(np.float32)).max()
    assert first == np.inf or first > 65504  # the half sums overflow fp16 (so do the split partials)
    # the split partials reach ~1e8 (fp32 ulp 8): what is left is a few ulps of the reduce's
    # fp32 summation order (the halves cancel split by split only up to that order)
    assert np.abs(got).max() <= 256


@pytest.mark.parametrize("N", (3, 4))
def test_q6_k_decode_two_token_groups(N):
    """Q6_K at 3-4 tokens with K >= 8192 runs as two 2-token groups (mmq_decode.hip pick()):
    against the oracle, and row shards of the matrix give the same bits (the choice depends on
    K only)."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    M, K = 192, 8192
    qA = random_blocks("q6_k", M, K, seed=40 + N)
    B = random_activations(N, K, seed=41 + N)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(B).to(dev)
    C = mmq(TYPES["q6_k"], A_t, B_t, M, N, K)
    half = qA.size // 2
    C2 = mmq(TYPES["q6_k"], A_t[half:], B_t, M // 2, N, K)
    torch.cuda.synchronize()
    ideal = O.mmq_from_fp16("q6_k", qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(C.cpu().numpy(), ideal) <= TIGHT_GEMV
    assert torch.equal(C2.view(torch.int16), C[:, M // 2:].contiguous().view(torch.int16))


@pytest.mark.parametrize("fmt,K,N", [("q6_k", 28672, 2), ("q6_k", 28672, 4), ("q4_k", 11008, 4), ("q8_0", 14336, 4)])
def test_long_k_small_n_routes(fmt, K, N):
    """2-4 tokens whose q8_1 image does not fit LDS beside the decode ring (long K) take the
    GEMV path (mmq_decode.hip decode_fused_ok); against the oracle."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    M = 96
    qA = random_blocks(fmt, M, K, seed=K + N)
    B = random_activations(N, K, seed=K - N)
    C = mmq(TYPES[fmt], torch.from_numpy(qA.view(np.int8)).to(dev), torch.from_numpy(B).to(dev), M, N, K)
    torch.cuda.synchronize()
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(C.cpu().numpy(), ideal) <= TIGHT_GEMV


@pytest.mark.parametrize("fmt", ("q8_0", "q4_k", "q6_k"))
@pytest.mark.parametrize("M,N,K", [(512, 5, 1024), (300, 16, 2048), (1024, 17, 4096), (640, 32, 1536), (128, 9, 512), (384, 64, 1024), (256, 40, 2048)])
def test_gemm_in_kernel_quantization_bit_identical(fmt, M, N, K, tune):
    """16/32-token tiles quantize their activations inside the GEMM (no act_quant launch): the
    result is the same bits as the act_quant (DEQ) + GEMM path, and matches the oracle."""
    from kernels._lib import TYPES, mmq
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + N)
    B = random_activations(N, K, seed=K + 2 * N)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    # a strided activation view (ldb > K) exercises the row stride of the in-kernel loads
    Bw = torch.zeros(N, K + 64, dtype=torch.float16, device=dev)
    Bw[:, :K] = torch.from_numpy(B).to(dev)
    B_t = Bw[:, :K]
    fused = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    tune(GQ_GEMM_AQ=0)
    staged = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(fused.view(torch.int16), staged.view(torch.int16))
    ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
    assert O.max_rel_err(fused.cpu().numpy(), ideal) <= TIGHT_GEMM


@pytest.mark.parametrize("W,N,R,M,pad", [(2, 5, 64, 100, 0), (8, 128, 3584, 28672, 0), (4, 3, 64, 250, 7),
                                         (3, 17, 128, 384, 0), (8, 1, 1024, 8192, 0)])
def test_assemble_shards_kernel(W, N, R, M, pad):
    """gq_assemble_shards (the all-gather's (world, N, R) -> (N, M) step) against torch's
    permute, vector (16-byte) and scalar (odd M / ldc) forms."""
    from kernels._lib import assemble_shards
    dev = _dev()
    g = torch.randn(W, N, R, generator=torch.Generator().manual_seed(W * N + R)).to(torch.float16).to(dev)
    want = g.permute(1, 0, 2).reshape(N, W * R)[:, :M]
    out = torch.full((N, M + pad), -1.0, dtype=torch.float16, device=dev)[:, :M]
    got = assemble_shards(g, M, out=out)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("fmt,M,N,K,chunks", [("q6_k", 1000, 1, 8192, 3), ("q4_k", 4096, 128, 4096, 4),
                                               ("q8_0", 300, 16, 1024, 2)])
def test_row_sharded_pipelined_world1(fmt, M, N, K, chunks, tune):
    """RowShardedMMQ.pipelined (row chunks of the shard, one all-gather per chunk) at world 1
    through the HIP MMQ: the same bits as the unsharded call (split-K off: the chunk row count
    does not change the arithmetic then)."""
    from dist.row_shard import RowShardedMMQ
    from kernels._lib import TYPES, mmq
    tune(GQ_GEMM_SPLITS=1, GQ_KSTREAM=0)  # (chunks run prepared: keep them off the K-chunked stream too)
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + 3)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(random_activations(N, K, seed=K)).to(dev)
    want = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    got = RowShardedMMQ(fmt, A_t, M, K, world=1, rank=0).pipelined(B_t, N, chunks)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.parametrize("fmt,M,N,K,chunks", [("q6_k", 1000, 1, 8192, 3), ("q4_k", 4096, 128, 4096, 4),
                                               ("q8_0", 4096, 128, 4096, 2), ("q6_k", 2048, 64, 4096, 3)])
def test_row_sharded_pipelined_default_tuning(fmt, M, N, K, chunks):
    """pipelined() with the library's default routing: a row chunk may take another GEMM route
    or split-K factor than the whole matrix (dist/row_shard.py pipelined), so the values agree
    within the GEMM tolerance (fp16 partials), bit for bit at decode sizes."""
    import oracle as O
    from dist.row_shard import RowShardedMMQ
    from kernels._lib import TYPES, mmq
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + 5)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(random_activations(N, K, seed=K + 1)).to(dev)
    want = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    got = RowShardedMMQ(fmt, A_t, M, K, world=1, rank=0).pipelined(B_t, N, chunks)
    torch.cuda.synchronize()
    if N <= 4:
        assert torch.equal(got.view(torch.int16), want.view(torch.int16))
    else:
        assert O.max_rel_err(got.cpu().numpy(), want.cpu().numpy()) <= 4e-3


@pytest.mark.parametrize("fmt,M,N,K", [("q6_k", 1000, 1, 8192), ("q4_k", 4096, 128, 4096), ("q8_0", 300, 16, 1024)])
def test_mmq_sharded_entry_point_world1(fmt, M, N, K):
    """gq_mmq_sharded through the C ABI at world 1 (no communicator): the same bits as gq_mmq."""
    from kernels._lib import TYPES, mmq, mmq_sharded_single
    dev = _dev()
    qA = random_blocks(fmt, M, K, seed=M + N)
    B = random_activations(N, K, seed=K + N)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    B_t = torch.from_numpy(B).to(dev)
    want = mmq(TYPES[fmt], A_t, B_t, M, N, K)
    got = mmq_sharded_single(TYPES[fmt], A_t, B_t, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


def test_mmq_sharded_entry_point_rccl_one_rank():
    """gq_mmq_sharded with a real 1-rank RCCL communicator (created here through RCCL's own C
    API): the run-time-resolved ncclAllGather leg and the assemble give gq_mmq's bits."""
    import ctypes
    import kernels._lib as kl
    dev = _dev()
    rccl = ctypes.CDLL("librccl.so.1")

    class UniqueId(ctypes.Structure):
        _fields_ = [("internal", ctypes.c_char * 128)]

    uid = UniqueId()
    assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    rccl.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    torch.cuda.set_device(dev)
    assert rccl.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
    try:
        fmt, M, N, K = "q6_k", 1000, 8, 2048
        qA = random_blocks(fmt, M, K, seed=5)
        B = random_activations(N, K, seed=6)
        A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
        B_t = torch.from_numpy(B).to(dev)
        want = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
        C = torch.empty(N, M, dtype=torch.float16, device=dev)
        need = int(kl.lib().gq_mmq_sharded_workspace_size(kl.TYPES[fmt], M, N, K, 1))
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        kl._check(kl.lib().gq_mmq_sharded(kl.TYPES[fmt], A_t.data_ptr(), B_t.data_ptr(), C.data_ptr(), M, N, K, K, M,
                                          1, 0, comm, ws.data_ptr(), need, stream))
        torch.cuda.synchronize()
        assert torch.equal(C.view(torch.int16), want.view(torch.int16))
    finally:
        rccl.ncclCommDestroy(comm)


@pytest.mark.parametrize("M,K", [(300, 4096), (4096, 4096), (97, 2048), (1000, 8192), (64, 11008), (40, 28672), (33, 256)])
def test_q6_k_decode_aligned_image_bit_identical(M, K, tune):
    """The Q6_K decode ring as an aligned image (224-B super-blocks, per-piece DMA sources:
    mmq_decode.hip kImgSB; the default for K <= 4096) gives the same bits as the packed ring at
    1-4 tokens -- whole-row tasks of 1..16 rows, row segments (K = 11008, 28672), short rows --
    alone and inside a grouped launch, and matches the oracle."""
    from kernels._lib import TYPES, mmq, mmq_grouped
    dev = _dev()
    qA = random_blocks("q6_k", M, K, seed=M + K)
    A_t = torch.from_numpy(qA.view(np.int8)).to(dev)
    for N in (1, 2, 3, 4):
        B = random_activations(N, K, seed=N + K)
        B_t = torch.from_numpy(B).to(dev)
        outs = {}
        for img in (0, 1):
            tune(GQ_DECODE_Q6_IMG=img)
            outs[img] = mmq(TYPES["q6_k"], A_t, B_t, M, N, K)
            g = mmq_grouped([(TYPES["q6_k"], A_t, B_t, M, K, None), (TYPES["q4_k"], A_t[: 144 * (K // 256)], B_t, 1, K, None)], N)
            if g is not None:
                assert torch.equal(g[0].view(torch.int16), outs[img].view(torch.int16)), (img, N)
        torch.cuda.synchronize()
        assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16)), N
        ideal = O.mmq_from_fp16("q6_k", qA, B, M, N, K, O.IDEAL)
        assert O.max_rel_err(outs[1].cpu().numpy(), ideal) <= TIGHT_GEMV
