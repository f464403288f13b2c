"""The library's routing as measured (gq_debug_route: the kernels a call launches).  Pins the
defaults DESIGN.md §5 "Round 4" reports, so a routing change is a visible test change."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fmt,M,N,K,prepared,want", [
    ("q8_0", 4096, 1, 4096, False, "stream_decode_kernel"),
    ("q6_k", 28672, 1, 8192, False, "stream_decode_kernel"),
    ("q8_0", 4096, 128, 4096, False, "rgemm_kernel"),        # the headline: resident split, q8_1 in-kernel
    ("q4_k", 4096, 128, 4096, True, "rgemm_kernel"),
    ("q4_k", 4096, 16, 4096, False, "rgemm_kernel"),         # ahead of the skinny kernel
    ("q4_k", 11008, 16, 4096, False, "kstream_kernel"),      # raw 5..16 tokens on >= 8192 rows (round 5)
    ("q8_0", 11008, 16, 4096, False, "kstream_kernel"),
    ("q4_k", 11008, 32, 4096, False, "rgemm_kernel"),        # up to four resident rounds at <= 32 tokens
    ("q6_k", 11008, 16, 4096, True, "kstream_kernel"),      # prepared 5..32 tokens, K <= 4096 (round 5)
    ("q4_k", 4096, 16, 4096, True, "kstream_kernel"),
    ("q4_k", 22016, 16, 4096, False, "kstream_kernel"),
    ("q4_k", 22016, 24, 4096, False, "rgemm_kernel"),
    ("q8_0", 28672, 16, 8192, False, "skinny_kernel"),        # (more than four rounds)
    ("q6_k", 28672, 16, 8192, True, "sgemm_kernel"),
    ("q6_k", 28672, 128, 8192, True, "sgemm_kernel"),
    ("q4_k", 11008, 128, 4096, True, "sgemm_kernel"),
    ("q6_k", 28672, 512, 8192, True, "sgemm_kernel"),
    ("q4_k", 4096, 1024, 4096, True, "hipBLASLt"),
])
def test_default_routes(fmt, M, N, K, prepared, want):
    import kernels._lib as kl
    assert torch.cuda.is_available()
    got = kl.route_name(kl.TYPES[fmt], M, N, K, prepared=prepared)
    assert want in got, got


def test_route_knobs(tune):
    import kernels._lib as kl
    tune(GQ_GEMM_SPLITS=4)  # a GEMM knob pins the LDS-DMA GEMM
    assert "gemm_kernel" in kl.route_name(kl.GQ_Q8_0, 4096, 128, 4096) and "rgemm" not in kl.route_name(kl.GQ_Q8_0, 4096, 128, 4096)
    tune(GQ_GEMM_SPLITS=0, GQ_SGEMM_STREAMK=1)
    assert "stream-K" in kl.route_name(kl.GQ_Q6_K, 28672, 128, 8192, prepared=True)
