#!/usr/bin/env python3
"""Where an eager drop-in call's host time goes (M=1, Q4_K 4096^2): the whole call, and its
pieces timed alone (median of 1000, each synchronized like bench.eager_call_us)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import kernels._lib as kl  # noqa: E402
from kernels.mmq_q4_k import mmq_q4_k  # noqa: E402

dev = torch.device("cuda:0")
A = bench.device_random_blocks("q4_k", 4096, 4096, dev, seed=1)
B = torch.randn(1, 4096, device=dev).half()
C = torch.empty(1, 4096, dtype=torch.float16, device=dev)
need = kl.workspace_size(kl.GQ_Q4_K, 4096, 1, 4096)
ws = torch.empty(need, dtype=torch.uint8, device=dev)
L = kl.lib()
st = torch.cuda.current_stream().cuda_stream


def med(fn, n=1000, sync=True):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 2)


print("workspace bytes", need)
print("eager mmq_q4_k (synced)          ", med(lambda: mmq_q4_k(A, B, 4096, 1, 4096)))
print("raw gq_mmq, buffers preallocated ", med(lambda: L.gq_mmq(1, A.data_ptr(), B.data_ptr(), C.data_ptr(), 4096, 1, 4096, 4096, 4096, ws.data_ptr(), need, st)))
print("synchronize alone                ", med(lambda: None))
print("torch.empty C (no sync)          ", med(lambda: torch.empty(1, 4096, dtype=torch.float16, device=dev), sync=False))
print("torch.empty ws (no sync)         ", med(lambda: torch.empty(need, dtype=torch.uint8, device=dev), sync=False))
print("workspace_size ctypes (no sync)  ", med(lambda: kl.workspace_size(kl.GQ_Q4_K, 4096, 1, 4096), sync=False))
print("current_stream (no sync)         ", med(lambda: torch.cuda.current_stream(dev).cuda_stream, sync=False))
print("mmq_q4_k (no sync)               ", med(lambda: mmq_q4_k(A, B, 4096, 1, 4096), sync=False))
print("raw gq_mmq (no sync)             ", med(lambda: L.gq_mmq(1, A.data_ptr(), B.data_ptr(), C.data_ptr(), 4096, 1, 4096, 4096, 4096, ws.data_ptr(), need, st), sync=False))


def b2b(fn, n=1000):
    """Back-to-back: n calls, one synchronize at the end, divided by n (host-bound when the
    kernel is shorter than the call's host time)."""
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


print("b2b mmq_q4_k                     ", b2b(lambda: mmq_q4_k(A, B, 4096, 1, 4096)))
print("b2b raw gq_mmq                   ", b2b(lambda: L.gq_mmq(1, A.data_ptr(), B.data_ptr(), C.data_ptr(), 4096, 1, 4096, 4096, 4096, ws.data_ptr(), need, st)))
print("_check_weights                   ", med(lambda: kl._check_weights(kl.GQ_Q4_K, A, 4096, 4096), sync=False))
print("_check_acts                      ", med(lambda: kl._check_acts(B, 1, 4096), sync=False))
print("_check_out                       ", med(lambda: kl._check_out(None, 1, 4096, dev), sync=False))
print("_stream                          ", med(lambda: kl._stream(dev), sync=False))
print("current_device                   ", med(lambda: torch.cuda.current_device(), sync=False))
print("data_ptr x3                      ", med(lambda: (A.data_ptr(), B.data_ptr(), C.data_ptr()), sync=False))
