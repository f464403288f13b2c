"""Per-workgroup balance of the grouped K-chunked stream on the 7B Q4_K_M layer (diagnostic build
`make -C gguf-triton-kernel_amd kstamps`, never the product): per wave the s_memtime ticks of its
prologues and loops and its 16-row super-block tasks by format; prints the workgroup time spread
(max wave per workgroup) and a least-squares fit loop = a * Q4_K tasks + b * Q6_K tasks + c * items
-- the per-format cost the launch's deal weights (bytes - 55 per super-block) stand for.

  python tools/kstream_layer_stamps.py [N ...]   (default 16 32)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib",
                           "libgguf_mmq_%s.so" % os.environ.get("GQ_KSTAMPS_SO", "kstamps"))
import torch  # noqa: E402

import bench  # noqa: E402
from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types  # noqa: E402
from kernels.layer_mix import GGUFLinear, LayerMix  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    fn = kl.lib().gq_debug_kstream_stamps
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_size_t], ctypes.c_int
    types = q4_k_m_layer_types(0, 32)
    lin = {n: GGUFLinear(types[n], bench.device_random_blocks(types[n], M, K, dev, seed=i), M, K)
           for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
    layer = LayerMix(lin, act="q8_1", fuse=True, grouped=True)
    buf = np.zeros((65536, 12), np.uint64)
    for N in [int(a) for a in sys.argv[1:]] or [16, 32]:
        g = torch.Generator(device=dev).manual_seed(7)
        x = torch.randn(N, 4096, device=dev, generator=g).to(torch.float16)
        h = torch.randn(N, 11008, device=dev, generator=g).to(torch.float16)
        for _ in range(3):
            layer.forward(x, h)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
        layer.forward(x, h)
        torch.cuda.synchronize()
        assert fn(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
        ids = np.nonzero(buf[:, 5] > 0)[0]
        u = buf[ids].astype(np.float64)
        pro, wait, red, loop, items, q4, q6 = u[:, 0], u[:, 1], u[:, 2], u[:, 3], u[:, 5], u[:, 6], u[:, 7]
        spin, parts, nsum, tsum = u[:, 8], u[:, 9], u[:, 10], u[:, 11]
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez(os.path.join(ROOT, "gpurun_out", f"klayer_stamps_n{N}.npz"), ids=ids, u=u)
        wg = ids // 8
        tot = pro + loop
        wgs = np.unique(wg)
        wt = np.array([tot[wg == w].max() for w in wgs])
        # per workgroup: its slowest wave against its tasks (summed over its waves / 8) and items
        wq4 = np.array([q4[wg == w].sum() / 8 for w in wgs])
        wq6 = np.array([q6[wg == w].sum() / 8 for w in wgs])
        wit = np.array([items[wg == w].max() for w in wgs])
        wpa = np.array([parts[wg == w].max() for w in wgs])
        A = np.stack([wq4, wq6, wit, wpa], 1)
        coef, *_ = np.linalg.lstsq(A, wt, rcond=None)
        resid = wt - A @ coef
        print(f"N={N}: waves {len(ids)} in {len(wgs)} workgroups; workgroup time (max wave, ticks) "
              f"p10 {np.percentile(wt, 10):.0f} p50 {np.median(wt):.0f} p90 {np.percentile(wt, 90):.0f} "
              f"max {wt.max():.0f}; mean/max {wt.mean() / wt.max():.3f}")
        print(f"   per wave: prologue med {np.median(pro):.0f}, loop med {np.median(loop):.0f} (waits {np.median(wait):.0f}, "
              f"reduces {np.median(red):.0f} of which hand-off spin {np.median(spin):.0f}); tasks Q4_K mean {q4.mean():.1f}, "
              f"Q6_K {q6.mean():.1f}, items {items.mean():.1f}, parts {parts.mean():.2f}")
        print(f"   fit workgroup time = {coef[0]:.0f} * Q4_K task + {coef[1]:.0f} * Q6_K task + {coef[2]:.0f} * item "
              f"+ {coef[3]:.0f} * part  (per wave; Q6_K / Q4_K {coef[1] / coef[0]:.2f}, deal weights 155 / 89 = 1.74); "
              f"residual rms {np.sqrt(np.mean(resid ** 2)):.0f}")
        # who sums: per workgroup, the share of its hand-offs summed by its most frequent summer
        # (1/8 if the last arrival rotates, 1 if one wave is always last)
        share = np.array([nsum[wg == w].max() / max(nsum[wg == w].sum(), 1) for w in wgs])
        wv = ids % 8
        print(f"   summing: ticks per summed hand-off med {np.median(tsum[nsum > 0] / nsum[nsum > 0]):.0f}; "
              f"top summer's share per workgroup med {np.median(share):.2f} p90 {np.percentile(share, 90):.2f}; "
              f"hand-offs summed by wave index 0..7: {[int(nsum[wv == k].sum()) for k in range(8)]}")
        for name, sel in (("Q4_K-only", wq6 == 0), ("Q6_K-only", wq4 == 0), ("mixed", (wq4 > 0) & (wq6 > 0))):
            if sel.any():
                print(f"   {name} workgroups {sel.sum()}: time mean {wt[sel].mean():.0f} max {wt[sel].max():.0f}, "
                      f"items mean {wit[sel].mean():.1f}")
        slow = wgs[np.argsort(wt)[-5:]]
        for w in slow:
            m = wg == w
            print(f"   slow workgroup {w}: max {tot[m].max():.0f} prologue {pro[m].mean():.0f} loop {loop[m].mean():.0f} "
                  f"Q4_K {q4[m].sum():.0f} Q6_K {q6[m].sum():.0f} items {items[m].max():.0f} spin {spin[m].mean():.0f}")


if __name__ == "__main__":
    main()
