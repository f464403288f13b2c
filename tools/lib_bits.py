"""Output digest of a build of libgguf_mmq.so under tuning overrides, for bit-identity checks
between builds (two runs, diff the lines): prepared and raw call per config.

Usage: python tools/lib_bits.py [--lib=PATH] [--tune=KEY=V,...] CONFIG ...   (CONFIG: fmt_MxK_mN)
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import kernels._lib as kl  # noqa: E402

args = sys.argv[1:]
tune = []
for a in list(args):
    if a.startswith("--lib="):
        kl.LIB_PATH = os.path.abspath(a[6:])
        args.remove(a)
    elif a.startswith("--tune="):
        tune = [kv.split("=") for kv in a[7:].split(",") if kv]
        args.remove(a)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from utils.synth import random_activations, random_blocks  # noqa: E402

dev = torch.device("cuda:0")
kl.reset_tuning()
for k, v in tune:
    kl.set_tuning(k, int(v))
for cfg in args:
    fmt = cfg[:4]
    mk, n = cfg[5:].split("_m")
    M, K = map(int, mk.split("x"))
    N = int(n)
    t = kl.TYPES[fmt]
    A = torch.from_numpy(random_blocks(fmt, M, K, seed=M + K).view(np.int8)).to(dev)
    B = torch.from_numpy(random_activations(N, K, seed=N + K)).to(dev)
    ws = torch.empty(kl.workspace_size(t, M, N, K), dtype=torch.uint8, device=dev)
    kl.act_prepare(B, N, K, ws)
    outs = [kl.mmq_prepared(t, A, ws, M, N, K), kl.mmq(t, A, B, M, N, K)]
    torch.cuda.synchronize()
    h = [hashlib.sha1(o.cpu().numpy().tobytes()).hexdigest()[:16] for o in outs]
    print(cfg, kl.route_name(t, M, N, K, prepared=True), *h, flush=True)
