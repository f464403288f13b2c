"""Run GPU tests against a diagnostic build of libgguf_mmq.so (never the product):
python tools/lib_parity.py LIB.so [pytest args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.abspath(sys.argv[1])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[2:]))
