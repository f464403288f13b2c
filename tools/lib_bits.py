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
    if cfg.startswith("layer_m"):  # the 7B Q4_K_M layer (LayerMix, grouped), every projection's output
        import bench
        from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
        from kernels.layer_mix import GGUFLinear, LayerMix
        N = int(cfg[7:])
        types = q4_k_m_layer_types(0, 32)
        lin = {n: GGUFLinear(types[n], bench.device_random_blocks(types[n], M, K, dev, seed=i), M, K)
               for i, (n, (M, K)) in enumerate(LLAMA_LAYER_SHAPES.items())}
        g = torch.Generator(device=dev).manual_seed(7)
        x = torch.randn(N, 4096, device=dev, generator=g).to(torch.float16)
        h = torch.randn(N, 11008, device=dev, generator=g).to(torch.float16)
        outs = LayerMix(lin, act="q8_1", fuse=True, grouped=True).forward(x, h)
        torch.cuda.synchronize()
        print(cfg, *(f"{n}:{hashlib.sha1(o.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]}" for n, o in sorted(outs.items())),
              flush=True)
        continue
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
