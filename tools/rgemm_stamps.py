"""Per-wave timeline of the resident GEMM (diagnostic build `make -C gguf-triton-kernel_amd rabl
RABL=0 RABL_FLAGS=-DGQ_RGEMM_STAMPS RABL_SO=stamps`, never the product): where a launch's time
goes, phase by phase, and how the waves' phases line up across the chip.

  python tools/rgemm_stamps.py [CONFIG ...]     (default q8_0_4096x4096_m128; bench.py names)

s_memtime ticks per phase (medians over waves, p90 in brackets); the wave start / end spread
from s_memrealtime (100 MHz, chip-wide), in us."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib", "libgguf_mmq_rablstamps.so")
import torch  # noqa: E402

import bench  # noqa: E402

PHASES = [(1, 2, "issue loads"), (2, 3, "x~ ready (wait/quantize)"), (3, 4, "activation barrier"),
          (4, 5, "own half 0 lands"), (5, 6, "multiply half 0"), (6, 7, "own half 1 lands"),
          (7, 8, "multiply half 1"), (8, 9, "partial stores issued"), (9, 10, "stores complete")]


def main():
    dev = torch.device("cuda:0")
    L = kl.lib()
    fn = L.gq_debug_rgemm_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int
    for cfg in sys.argv[1:] or ["q8_0_4096x4096_m128"]:
        if cfg in bench.CONFIGS:
            fmt, M, K, N = bench.CONFIGS[cfg]
        else:
            fmt = cfg[:4]
            mk, n = cfg[5:].split("_m")
            M, K = map(int, mk.split("x"))
            N = int(n)
        print(f"{cfg}: route {kl.route_name(kl.TYPES[fmt], M, N, K)}")
        r = bench.Runner(fmt, M, K, N, dev, 4)
        for prepared in (False, True):
            if prepared:
                r.prepare()
            for i in range(6):
                (r.kernel if prepared else r.step)(i, i % r.ncopies)
            torch.cuda.synchronize()
            buf = np.zeros((65536, 14), np.uint64)
            assert fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
            used = buf[buf[:, 1] > 0].astype(np.float64)
            print(f"  {'prepared x~' if prepared else 'in-kernel quantization'}: {len(used)} waves")
            for a, b, name in PHASES:
                d = used[:, b] - used[:, a]
                print(f"    {name:28s} med {np.median(d):7.0f}  p90 {np.percentile(d, 90):7.0f}  ticks")
            tot = used[:, 10] - used[:, 1]
            print(f"    {'total':28s} med {np.median(tot):7.0f}  p90 {np.percentile(tot, 90):7.0f}")
            t0 = used[:, 0].min()
            s, e = (used[:, 0] - t0) / 100.0, (used[:, 11] - t0) / 100.0
            print(f"    wave starts (us after the first): med {np.median(s):.2f} p90 {np.percentile(s, 90):.2f} "
                  f"max {s.max():.2f};  ends: p10 {np.percentile(e, 10):.2f} med {np.median(e):.2f} "
                  f"p90 {np.percentile(e, 90):.2f} max {e.max():.2f}")
            xcc = used[:, 13].astype(int)
            per = [np.median(e[xcc == x]) for x in range(8) if (xcc == x).any()]
            print("    median end per XCC (us): " + " ".join(f"{v:.2f}" for v in per))
            buf[:] = 0
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
