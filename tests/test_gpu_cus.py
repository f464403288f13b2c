"""GPU tests of the compute-unit count the plans size their grids by (gq_capi.hip num_cus():
hipDeviceAttributeMultiprocessorCount, queried once per device; GQ_CUS overrides it).  A
partitioned or shared GPU has fewer CUs than the 256 the plans once assumed: with a smaller
count forced, the grouped decode, the skinny kernel and the GEMM (split-K pinned, since the
split factor is what the count chooses there) give the same bits as with the device's count."""
import numpy as np
import pytest
import torch

from utils.synth import random_activations, random_blocks

pytestmark = pytest.mark.gpu


def _dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    return torch.device("cuda:0")


def _bits(t):
    torch.cuda.synchronize()
    return t.view(torch.int16).clone()


@pytest.mark.parametrize("cus", [200, 96])
def test_smaller_cu_count_bit_identical(cus, tune):
    import kernels._lib as kl
    dev = _dev()
    cases = []  # (name, fn)
    # grouped decode: three matrices at 1 and 2 tokens
    specs = [("q4_k", 4096, 4096), ("q6_k", 1024, 4096), ("q8_0", 2048, 4096)]
    qs = [torch.from_numpy(random_blocks(f, M, K, seed=i).view(np.int8)).to(dev) for i, (f, M, K) in enumerate(specs)]
    for N in (1, 2):
        x = torch.from_numpy(random_activations(N, 4096, seed=N)).to(dev)
        items = [(kl.TYPES[f], q, x, M, K, None) for (f, M, K), q in zip(specs, qs)]
        cases.append((f"grouped N={N}", lambda items=items, N=N: torch.cat([o for o in kl.mmq_grouped(items, N)], 1)))
    # skinny (Q4_K at 16 tokens) and the GEMM (Q8_0 at 128 tokens, splits pinned)
    x16 = torch.from_numpy(random_activations(16, 4096, seed=16)).to(dev)
    cases.append(("skinny", lambda: kl.mmq(kl.GQ_Q4_K, qs[0], x16, 4096, 16, 4096)))
    x128 = torch.from_numpy(random_activations(128, 4096, seed=128)).to(dev)
    cases.append(("gemm", lambda: kl.mmq(kl.GQ_Q8_0, qs[2], x128, 2048, 128, 4096)))
    tune(GQ_GEMM_SPLITS=8, GQ_SKINNY_RG=1, GQ_RGEMM=0)  # the plans the count could change, pinned
    ref = {name: _bits(fn()) for name, fn in cases}
    tune(GQ_CUS=cus)
    for name, fn in cases:
        assert torch.equal(_bits(fn()), ref[name]), name
