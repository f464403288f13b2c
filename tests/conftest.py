import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gguf-triton-kernel_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(fmt):
        z = np.load(os.path.join(ROOT, "tests", "golden", f"golden_{fmt}.npz"))
        n = len([k for k in z.files if k.endswith("_MNK")])
        cases = []
        for i in range(n):
            M, N, K = (int(v) for v in z[f"c{i}_MNK"])
            case = dict(i=i, M=M, N=N, K=K, kind=str(z[f"c{i}_kind"]), B=z[f"c{i}_B"], qA=z[f"c{i}_qA"],
                        qB=z[f"c{i}_qB"], C=z[f"c{i}_C"])
            if f"c{i}_Ctri" in z.files:
                case["Ctri"] = z[f"c{i}_Ctri"]
            cases.append(case)
        return cases

    return {fmt: load(fmt) for fmt in ("q8_0", "q4_k", "q6_k")}


@pytest.fixture
def tune():
    """tune(GQ_GEMM_SPLITS=8, GQ_RGEMM=0, ...): override the library's tuning defaults for this
    test (gq_debug_set_tuning; the library reads GQ_* from the environment once, so setting
    os.environ in a test has no effect); everything is reset after the test."""
    import kernels._lib as kl

    def set_(**kw):
        for k, v in kw.items():
            kl.set_tuning(k, int(v))

    yield set_
    kl.reset_tuning()
