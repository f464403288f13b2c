"""Per-wave phase ticks of the K-chunked streaming MMQ (diagnostic build `make -C
gguf-triton-kernel_amd kstamps`, never the product): prologue (activation loads + quantization
+ ring fill), ring waits, item reduces, main loop; s_memtime ticks, medians over waves (p90).

  python tools/kstream_stamps.py [CONFIG[:prepared] ...]   (fmt_MxK_mN names)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib", "libgguf_mmq_kstamps.so")
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    L = kl.lib()
    fn = L.gq_debug_kstream_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int
    kl.set_tuning("GQ_KSTREAM", 1)
    for spec in sys.argv[1:] or ["q4_k_22016x4096_m16"]:
        cfg, _, mode = spec.partition(":")
        fmt = cfg[:4]
        mk, n = cfg[5:].split("_m")
        M, K = map(int, mk.split("x"))
        N = int(n)
        r = bench.Runner(fmt, M, K, N, dev, 4)
        prepared = mode == "prepared"
        if prepared:
            r.prepare()
        buf = np.zeros((65536, 12), np.uint64)
        for i in range(3):  # warm, then the stamped call alone
            (r.kernel if prepared else r.step)(i, i % r.ncopies)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
        (r.kernel if prepared else r.step)(0, 0)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
        used = buf[buf[:, 5] > 0].astype(np.float64)
        pro, wait, red, loop, ntask, items = (used[:, i] for i in range(6))
        q = lambda v: f"{np.median(v):8.0f} ({np.percentile(v, 90):8.0f})"
        print(f"{spec}: waves {len(used)}, items/wave {np.median(items):.1f}, tasks/wave {np.median(ntask):.1f}")
        print(f"   prologue {q(pro)}  loop {q(loop)}  = waits {q(wait)} + reduces {q(red)} + rest {q(loop - wait - red)}")
        print(f"   per task: wait {np.median(wait / np.maximum(ntask, 1)):.0f}  rest {np.median((loop - wait - red) / np.maximum(ntask, 1)):.0f}"
              f"  per item reduce {np.median(red / np.maximum(items, 1)):.0f}")
        del r
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
