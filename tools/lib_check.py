"""Parity of a diagnostic build of libgguf_mmq.so: each config's raw call against the same
library's call with the streaming, resident and K-chunked GEMMs and the fused decode switched off (another kernel, other fp32
summation order): max |difference| over max |reference| (the GEMM tolerance is 4e-3).

Usage: python tools/lib_check.py --lib=PATH CONFIG ...   (CONFIG: fmt_MxK_mN)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

args = sys.argv[1:]
for a in list(args):
    if a.startswith("--lib="):
        kl.LIB_PATH = os.path.abspath(a[6:])
        args.remove(a)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from utils.synth import random_activations, random_blocks  # noqa: E402

dev = torch.device("cuda:0")
worst = 0.0
for cfg in args:
    fmt = cfg[:4]
    mk, n = cfg[5:].split("_m")
    M, K = map(int, mk.split("x"))
    N = int(n)
    t = kl.TYPES[fmt]
    A = torch.from_numpy(random_blocks(fmt, M, K, seed=M + K).view(np.int8)).to(dev)
    B = torch.from_numpy(random_activations(N, K, seed=N + K)).to(dev)
    kl.reset_tuning()
    route = kl.route_name(t, M, N, K)
    out = kl.mmq(t, A, B, M, N, K).float().cpu().numpy()
    kl.set_tuning("GQ_SGEMM", 0)
    kl.set_tuning("GQ_RGEMM", 0)
    kl.set_tuning("GQ_KSTREAM", 0)
    kl.set_tuning("GQ_NO_FUSED_DECODE", 1)
    ref = kl.mmq(t, A, B, M, N, K).float().cpu().numpy()
    alt = kl.route_name(t, M, N, K)
    kl.reset_tuning()
    err = float(np.abs(out - ref).max() / max(np.abs(ref).max(), 1e-30))
    worst = max(worst, err)
    print(f"{cfg:30s} {route} vs {alt}: max_rel_err={err:.2e} finite={np.isfinite(out).all()}", flush=True)
print("WORST", worst)
sys.exit(0 if worst <= 4e-3 else 1)
