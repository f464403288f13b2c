"""The oracle is pinned before it is trusted: oracle/mmq_oracle.c against vectors produced by
running the reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

import oracle as O

FMTS = ("q8_0", "q4_k", "q6_k")


@pytest.mark.parametrize("fmt", FMTS)
def test_oracle_matmul_bit_exact(golden, fmt):
    """mode EXACT reproduces kernels/cpu_impls/mmq_*_q8_1_cpu bit for bit on every case."""
    for c in golden[fmt]:
        got = O.mmq(fmt, c["qA"], c["qB"], c["M"], c["N"], c["K"], O.EXACT)
        assert got.shape == (c["N"], c["M"])
        assert np.array_equal(got.view(np.uint16), c["C"].view(np.uint16)), (fmt, c["i"], c["kind"])


@pytest.mark.parametrize("fmt", FMTS)
def test_oracle_q8_1_bit_exact(golden, fmt):
    """oracle quantize_q8_1 == utils/quantize/q8_1.py bytes for every activation fixture."""
    for c in golden[fmt]:
        assert np.array_equal(O.quantize_q8_1(c["B"]), c["qB"]), (fmt, c["i"])


def test_oracle_q8_0_and_q8_1_quantizers():
    z = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "golden_quant.npz"))
    names = sorted({k[:-2] for k in z.files if k.endswith("_x")})
    for name in names:
        x = z[name + "_x"]
        assert np.array_equal(O.quantize_q8_0(x), z[name + "_q8_0"]), name
        assert np.array_equal(O.quantize_q8_1(x), z[name + "_q8_1"]), name


@pytest.mark.parametrize("fmt", FMTS)
def test_oracle_ideal_close_to_reference(golden, fmt):
    """IDEAL (exact products, one rounding) stays within the reference's own 1% gate of the
    reference output, except where the reference's fp16 arithmetic underflows
    (Q8_0 'tiny': fp16(dA*dB) flushes to 0 in mmq_q8_0_q8_1_cpu.py:47)."""
    for c in golden[fmt]:
        if fmt == "q8_0" and c["kind"] == "tiny":
            assert np.all(c["C"] == 0)
            continue
        ideal = O.mmq(fmt, c["qA"], c["qB"], c["M"], c["N"], c["K"], O.IDEAL)
        assert O.allclose(c["C"], ideal, 0.01), (fmt, c["i"], O.max_rel_err(c["C"], ideal))


@pytest.mark.parametrize("fmt", FMTS)
def test_reference_gpu_semantics_vs_oracle(golden, fmt):
    """The reference's own Triton kernel (run under TRITON_INTERPRET=1 when the fixtures were
    made) against its 1% gate vs cpu_impls -- the gate the build is held to as well.  It
    fails exactly one captured case: Q8_0 M=N=1, K=32 (a single output; its fp32 on-the-fly
    activation quantization differs by one code from q8_1.py: 2.2% off).  The build uses the
    q8_1 semantics, so it does not inherit that miss (test_gpu_parity.test_golden_cases)."""
    failing = []
    for c in golden[fmt]:
        if "Ctri" in c and not O.allclose(c["C"], c["Ctri"], 0.01):
            failing.append((c["M"], c["N"], c["K"]))
    assert failing == ([(1, 1, 32)] if fmt == "q8_0" else []), failing


def test_dequant_matches_formula():
    """oracle dequantizers agree with the matmul oracle: W @ x~ from dequantized W equals
    the IDEAL matmul (x~ = dequantized q8_1 activation) to fp32 rounding."""
    rng = np.random.default_rng(3)
    for fmt, qk, nbytes in (("q8_0", 32, 34), ("q4_k", 256, 144), ("q6_k", 256, 210)):
        M, N, K = 5, 3, 512
        raw = rng.integers(0, 256, size=(M * K // qk, nbytes), dtype=np.uint8)
        if fmt == "q8_0":
            raw[:, 1] = 0x20
        elif fmt == "q4_k":
            raw[:, 1] = 0x20
            raw[:, 3] = 0x20
        else:
            raw[:, 209] = 0x20
        A = raw.reshape(-1)
        B = rng.standard_normal((N, K)).astype(np.float16)
        W = O.dequant(fmt, A).reshape(M, K).astype(np.float64)
        Bq = O.quantize_q8_1(B)
        X = O.dequant("q8_1", Bq).reshape(N, K).astype(np.float64)
        want = (X @ W.T).astype(np.float16)
        got = O.mmq(fmt, A, Bq, M, N, K, O.IDEAL)
        assert O.max_rel_err(got, want) < 2e-3, fmt
