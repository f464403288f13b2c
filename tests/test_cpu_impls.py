"""The drop-in `kernels.cpu_impls` package (the reference's CPU MMQ functions,
kernels/cpu_impls/mmq_*_q8_1_cpu.py) through the build's own modules: the imports the
reference's test scripts make (test/test_mmq_q4_k.py:10-15) resolve, and the outputs equal
the reference's bit for bit on every golden case (tests/golden, produced by running the
reference).  CPU only: these functions are backed by libgguf_quant.so, not by oracle/."""
import numpy as np
import pytest
import torch

FMTS = ("q8_0", "q4_k", "q6_k")


def _fn(fmt):
    if fmt == "q8_0":
        from kernels.cpu_impls.mmq_q8_0_q8_1_cpu import mmq_q8_0_q8_1_cpu as f
    elif fmt == "q4_k":
        from kernels.cpu_impls.mmq_q4_k_q8_1_cpu import mmq_q4_k_q8_1_cpu as f
    else:
        from kernels.cpu_impls.mmq_q6_k_q8_1_cpu import mmq_q6_k_q8_1_cpu as f
    return f


def test_reference_test_imports_resolve():
    """The import block of the reference's test scripts, unchanged."""
    from kernels.cpu_impls.mmq_q4_k_q8_1_cpu import mmq_q4_k_q8_1_cpu  # noqa: F401
    from kernels.cpu_impls.mmq_q6_k_q8_1_cpu import mmq_q6_k_q8_1_cpu  # noqa: F401
    from kernels.cpu_impls.mmq_q8_0_q8_1_cpu import mmq_q8_0_q8_1_cpu  # noqa: F401
    from kernels.mmq_q4_k import mmq_q4_k  # noqa: F401
    from utils.quantize.q4_k import quantize_to_q4_k  # noqa: F401
    from utils.quantize.q8_1 import quantize_to_q8_1  # noqa: F401
    from utils.test_utils import allclose  # noqa: F401


@pytest.mark.parametrize("fmt", FMTS)
def test_cpu_impls_bit_exact_vs_reference(golden, fmt):
    f = _fn(fmt)
    for c in golden[fmt]:
        A = torch.from_numpy(c["qA"].view(np.int8).copy())
        B = torch.from_numpy(c["qB"].view(np.int8).copy())
        C = f(A, B, c["M"], c["N"], c["K"])
        assert C.shape == (c["N"], c["M"]) and C.dtype == torch.float16
        assert not C.is_contiguous() or c["M"] == 1 or c["N"] == 1  # the reference returns C.T
        got = C.contiguous().numpy().view(np.uint16)
        assert np.array_equal(got, c["C"].view(np.uint16)), (fmt, c["i"], c["kind"])


@pytest.mark.parametrize("fmt", FMTS)
def test_cpu_impls_thread_count_independent(fmt):
    from kernels.cpu_impls._cpu import cpu_mmq
    from utils.synth import random_activations, random_blocks
    from utils.quantize.q8_1 import quantize_to_q8_1
    M, N, K = 37, 5, 512
    A = torch.from_numpy(random_blocks(fmt, M, K, seed=4).view(np.int8))
    B = quantize_to_q8_1(torch.from_numpy(random_activations(N, K, seed=5)))
    g = {"q8_0": 0, "q4_k": 1, "q6_k": 2}[fmt]
    one = cpu_mmq(g, A, B, M, N, K, threads=1).contiguous()
    many = cpu_mmq(g, A, B, M, N, K, threads=7).contiguous()
    assert torch.equal(one.view(torch.int16), many.view(torch.int16))


def test_cpu_impls_reference_script_flow():
    """The reference test's own flow (quantize A and B on the host, run the CPU MMQ, gate with
    utils.test_utils.allclose) against an fp32 A@B^T of the dequantized operands."""
    from kernels.cpu_impls.mmq_q4_k_q8_1_cpu import mmq_q4_k_q8_1_cpu
    from utils.quantize.q4_k import dequantize_q4_k, quantize_to_q4_k
    from utils.quantize.q8_1 import dequantize_q8_1, quantize_to_q8_1
    from utils.test_utils import allclose
    g = torch.Generator().manual_seed(0)
    M, N, K = 16, 4, 1024
    fa = torch.randn(M, K, generator=g).to(torch.float16)
    fb = torch.randn(N, K, generator=g).to(torch.float16)
    qa, qb = quantize_to_q4_k(fa), quantize_to_q8_1(fb)
    C = mmq_q4_k_q8_1_cpu(qa, qb, M, N, K)
    W = dequantize_q4_k(qa, (M, K)).float()
    X = dequantize_q8_1(qb, (N, K)).float()
    assert allclose(C.float(), (X @ W.T), 0.01)


def test_cpu_impls_asserts_like_reference():
    from kernels.cpu_impls.mmq_q4_k_q8_1_cpu import mmq_q4_k_q8_1_cpu
    with pytest.raises(AssertionError):
        mmq_q4_k_q8_1_cpu(torch.zeros(144, dtype=torch.int8), torch.zeros(36 * 8, dtype=torch.int8), 1, 1, 255)
    with pytest.raises(AssertionError):  # wrong A byte count
        mmq_q4_k_q8_1_cpu(torch.zeros(143, dtype=torch.int8), torch.zeros(36 * 8, dtype=torch.int8), 1, 1, 256)
