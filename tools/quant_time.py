#!/usr/bin/env python3
"""On-device weight quantization (gq_quantize_weights) vs the host library (utils.quantize,
all cores): ms per matrix for the BASELINE weight shapes.  python tools/quant_time.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kernels._lib as kl  # noqa: E402
from utils.quantize import _qlib  # noqa: E402

dev = torch.device("cuda:0")
for fmt, M, K in (("q8_0", 4096, 4096), ("q4_k", 4096, 4096), ("q4_k", 11008, 4096), ("q6_k", 4096, 4096),
                  ("q6_k", 28672, 8192)):
    x16 = torch.randn(M, K, dtype=torch.float16, device=dev)
    X = x16 if fmt == "q8_0" else x16.float()
    kl.quantize_weights_device(fmt, X)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        y = kl.quantize_weights_device(fmt, X)
    e1.record()
    torch.cuda.synchronize()
    dev_ms = e0.elapsed_time(e1) / 3
    row = {"fmt": fmt, "M": M, "K": K, "device_ms": round(dev_ms, 3), "GB_per_s_in": round(X.numel() * X.element_size() / dev_ms / 1e6, 1)}
    if M * K <= 4096 * 11008:
        xc = x16.cpu()
        t = time.perf_counter()
        h = _qlib.quantize(fmt, xc)
        row["host_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        row["host_threads"] = min(os.cpu_count() or 1, 32)
        row["bytes_equal"] = bool(np.array_equal(h.numpy(), y.cpu().numpy()))
    print(json.dumps(row), flush=True)
