#!/usr/bin/env python3
"""Kernel-trace probe of the grouped decode vs one launch per matrix (Q4_K_M Llama-7B layer 0
at 1 token): run under `bash tools/gpu.sh prof NAME -- python3 tools/grouped_probe.py`."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
import kernels._lib as kl  # noqa: E402
from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types  # noqa: E402

dev = torch.device("cuda:0")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1
types = q4_k_m_layer_types(0, 32)
A = {n: bench.device_random_blocks(types[n], M, K, dev, seed=i) for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
x = torch.randn(N, 4096, device=dev).half()
h = torch.randn(N, 11008, device=dev).half()
items = [(kl.TYPES[types[n]], A[n], h if K == 11008 else x, M, K, None) for n, (M, K) in LLAMA_LAYER_SHAPES.items()]
for _ in range(20):
    kl.mmq_grouped(items, N)
torch.cuda.synchronize()
for _ in range(20):
    for it in items:
        kl.mmq(it[0], it[1], it[2], it[3], N, it[4])
torch.cuda.synchronize()
# single-item groups (same body as the solo kernel, only the grid differs)
for it in items:
    for _ in range(10):
        kl.mmq_grouped([it], N)
torch.cuda.synchronize()
