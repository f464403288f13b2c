"""GEMM tuning / ablation sweep on one GPU: kernel time (HIP events over a graph of launches,
activations prepared once) for bench.py configs under env overrides.

Usage: python tools/gemm_tune.py [--abl] CONFIG[:ENV=V,ENV=V...] ...
  CONFIG: a bench.py config name or fmt_MxK_mN (e.g. q4_k_28672x8192_m128)
  --abl   load build/abl/libgguf_mmq_abl.so (make -C gguf-triton-kernel_amd abl) so that
          GQ_ABLATE=<mask> selects the ablation variants of mmq_gemm.hip.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

args = sys.argv[1:]
STEP = "--step" in args  # time the whole drop-in step (gq_mmq: fused decode / act quant + GEMM)
args = [a for a in args if a != "--step"]
for a in list(args):
    if a.startswith("--lib="):  # a diagnostic build of libgguf_mmq.so (never the product)
        kl.LIB_PATH = os.path.abspath(a[6:])
        args.remove(a)
if args and args[0] == "--abl":
    kl.LIB_PATH = os.path.join(ROOT, "gguf-triton-kernel_amd", "lib", "libgguf_mmq_abl.so")
    args = args[1:]
import torch  # noqa: E402

import bench  # noqa: E402

if os.environ.get("GQ_TUNE_ROTATE"):  # weight-rotation bytes (default bench.ROTATE_BYTES, 1 GiB: cold)
    bench.ROTATE_BYTES = int(os.environ["GQ_TUNE_ROTATE"])

dev = torch.device("cuda:0")
for spec in args:
    # overrides through the library's tuning entry point (the GQ_* environment is read once, at
    # the first call, so setting os.environ here would not reach later specs)
    cfg, _, envs = spec.partition(":")
    kl.reset_tuning()
    for kv in filter(None, envs.split(",")):
        k, v = kv.split("=")
        kl.set_tuning(k, int(v))
    if cfg in bench.CONFIGS:
        fmt, M, K, N = bench.CONFIGS[cfg]
    else:  # fmt_MxK_mN, e.g. q4_k_28672x8192_m128
        fmt = cfg[:4]
        mk, n = cfg[5:].split("_m")
        M, K = map(int, mk.split("x"))
        N = int(n)
    r = bench.Runner(fmt, M, K, N, dev, 40)
    r.prepare()
    g = r.capture(r.step if STEP else r.kernel, [i % r.ncopies for i in range(40)])
    g.replay()
    t = min(bench.timed_replay(g, dev) for _ in range(5)) / 40
    _, alg_bytes, flops = bench.model(fmt, M, K, N)
    print(f"{spec:60s} kernel_us={t * 1e6:8.2f}  {flops / t / 1e12:7.1f} TF/s  {alg_bytes / t / 1e9:7.1f} GB/s",
          flush=True)
    del r, g
    torch.cuda.empty_cache()
