"""Per-wave time breakdown of the decode kernel (diagnostic build -DGQ_DECODE_STAMPS):
prologue (staging + quantization), waiting for weight DMAs, multiply loop.  s_memtime ticks."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib",
                           "libgguf_mmq_%s.so" % os.environ.get("GQ_STAMPS_SO", "stamps"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for cfg in sys.argv[1:] or ["q6_k_28672x8192_m1"]:
    fmt, M, K, N = bench.CONFIGS[cfg]
    r = bench.Runner(fmt, M, K, N, dev, 4)
    for i in range(8):
        r.step(i, i % r.ncopies)
    torch.cuda.synchronize()
    buf = np.zeros((65536, 13), np.uint64)
    assert kl.lib().gq_debug_decode_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes) == 0
    ids = np.nonzero(buf[:, 3] > 0)[0]
    used = buf[ids].astype(np.float64)
    pro, wait, loop, nt = used[:, 0], used[:, 1], used[:, 2], used[:, 3]
    xw, qd, t0, t1 = used[:, 4], used[:, 5], used[:, 6], used[:, 7]
    tot = pro + loop
    print(f"{cfg}: waves={len(used)} tasks/wave={nt.mean():.1f}  ticks: total med={np.median(tot):.0f} "
          f"max={tot.max():.0f}  prologue med={np.median(pro):.0f}  loop med={np.median(loop):.0f}  "
          f"dma-wait med={np.median(wait):.0f} ({np.median(wait / loop) * 100:.0f}% of loop)  "
          f"compute/task={np.median((loop - wait) / nt):.0f}")
    print(f"   prologue: x-arrival med={np.median(xw):.0f}  quantized med={np.median(qd):.0f}  "
          f"barrier med={np.median(pro - qd):.0f}")
    w0, c0, tp = used[:, 8], used[:, 9], used[:, 10]
    T0 = t0.min()
    print(f"   kernel span={t1.max() - T0:.0f}  wave starts: med={np.median(t0 - T0):.0f} max={(t0 - T0).max():.0f}  "
          f"ends: med={np.median(t1 - T0):.0f}  first DMA landed after barrier: med={np.median(w0 - tp):.0f}  "
          f"first task compute: med={np.median(c0 - w0):.0f}")
    # where the spread of wave durations lies: inside a workgroup (one CU) or between workgroups
    bx, xcc = used[:, 11].astype(np.int64), used[:, 12].astype(np.int64)
    wmax = np.array([tot[bx == b].max() for b in np.unique(bx)])
    wmin = np.array([tot[bx == b].min() for b in np.unique(bx)])
    print(f"   per workgroup: max-min med={np.median(wmax - wmin):.0f} p90={np.percentile(wmax - wmin, 90):.0f};  "
          f"workgroup max p10/p50/p90/max={np.percentile(wmax, 10):.0f}/{np.median(wmax):.0f}/"
          f"{np.percentile(wmax, 90):.0f}/{wmax.max():.0f};  workgroup mean med={np.median([tot[bx == b].mean() for b in np.unique(bx)]):.0f}")
    print("   per XCC: med/max duration " + "  ".join(
        f"{x}:{np.median(tot[xcc == x]):.0f}/{tot[xcc == x].max():.0f}" for x in np.unique(xcc)))
    # by the wave's index in its workgroup (waves i and i + DW/2 share a SIMD): duration against the
    # workgroup mean, and how often that index is the workgroup's slowest
    DW = int(os.environ.get("GQ_DECODE_DW", "8"))
    widx = ids % DW
    rel = np.array([tot[i] / tot[bx == bx[i]].mean() for i in range(len(tot))])
    slow = np.array([ids[bx == b][np.argmax(tot[bx == b])] % DW for b in np.unique(bx)])
    print("   by wave index: duration / workgroup mean " + " ".join(f"{k}:{rel[widx == k].mean():.3f}" for k in range(DW))
          + ";  slowest-wave share " + " ".join(f"{k}:{(slow == k).mean():.2f}" for k in range(DW)))
    for q in (10, 50, 90):
        print(f"   p{q}: start={np.percentile(t0 - T0, q):.0f} barrier={np.percentile(tp - T0, q):.0f} "
              f"dma0={np.percentile(w0 - T0, q):.0f} end={np.percentile(t1 - T0, q):.0f}")
    del r
