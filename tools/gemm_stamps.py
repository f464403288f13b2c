"""Per-wave time breakdown of the MFMA GEMM (diagnostic build: make stamps
STAMPS_FLAGS=-DGQ_GEMM_STAMPS STAMPS_SO=gstamps), s_memtime ticks from the wave's start:
first sub-stage wait (prologue DMA round trip), later waits summed, loop end, epilogue end
(split-K partial stores drained).  Usage: python tools/gemm_stamps.py CONFIG..."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib", "libgguf_mmq_gstamps.so")
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for cfg in sys.argv[1:] or ["q8_0_4096x4096_m128"]:
    fmt, M, K, N = bench.CONFIGS[cfg]
    r = bench.Runner(fmt, M, K, N, dev, 4)
    r.prepare()
    for i in range(8):
        r.kernel(i, i % r.ncopies)
    torch.cuda.synchronize()
    buf = np.zeros((65536, 8), np.uint64)
    kl.lib().gq_debug_gemm_stamps.restype = ctypes.c_int
    assert kl.lib().gq_debug_gemm_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    u = buf[buf[:, 5] > 0].astype(np.float64)
    first, wait, loop, end, subs = u[:, 0], u[:, 1], u[:, 2], u[:, 3], u[:, 4]
    med = lambda v: np.median(v)
    print(f"{cfg}: waves={len(u)} sub-stages/wave={med(subs):.0f}  ticks med: first wait={med(first):.0f} "
          f"later waits={med(wait):.0f} ({med(wait / np.maximum(loop - first, 1)) * 100:.0f}% of the rest of the loop) "
          f"loop end={med(loop):.0f} epilogue={med(end - loop):.0f} total={med(end):.0f} max={end.max():.0f}  "
          f"(setup done by {med(u[:, 5] - 1):.0f}, prologue DMAs issued by {med(u[:, 7]):.0f})", flush=True)
    # launch skew inside each workgroup (8 waves, one CU, one clock): the first barrier waits
    # for the last wave to arrive
    t0 = buf[:len(buf) // 8 * 8, 6].reshape(-1, 8).astype(np.float64)
    t0 = t0[(t0 > 0).all(axis=1)]
    if len(t0):
        print(f"   wave start spread inside a workgroup: med={np.median(t0.max(1) - t0.min(1)):.0f} "
              f"max={(t0.max(1) - t0.min(1)).max():.0f} ticks", flush=True)
    del r
