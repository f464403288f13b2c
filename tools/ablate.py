"""Ablation timing of the GEMM kernel (diagnostic build with -DGQ_ABLATION, see mmq_gemm.hip).
Usage: GQ_ABLATE=<mask> python tools/ablate.py <config> [lib path]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

kl.LIB_PATH = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gguf-triton-kernel_amd", "lib",
                                                                   "libgguf_mmq_abl.so")
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1]
out = bench.bench_config(cfg, 50, 5, torch.device("cuda:0"), False, 1, 0)
print(f"ablate={os.environ.get('GQ_ABLATE', '0'):>3} {cfg}: kernel_us={out['roofline']['kernel_us']:.2f} "
      f"step_us={out['ms_per_step'] * 1e3:.2f}", flush=True)
