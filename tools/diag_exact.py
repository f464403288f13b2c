"""Diagnostic: determinism and exact scale-by-2 behaviour of each path (GPU)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gguf-triton-kernel_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
from utils.synth import random_blocks, random_activations
import kernels._lib as kl
dev = torch.device("cuda:0")
for fmt in ("q8_0", "q4_k", "q6_k"):
    for (M, K) in ((4096, 4096), (256, 512)):
        qA = torch.from_numpy(random_blocks(fmt, M, K, seed=M + K).view(np.int8)).to(dev)
        for N in (1, 4, 16, 128):
            B = torch.from_numpy(random_activations(N, K, seed=N)).to(dev)
            C1 = kl.mmq(kl.TYPES[fmt], qA, B, M, N, K)
            C1b = kl.mmq(kl.TYPES[fmt], qA, B, M, N, K)
            C2 = kl.mmq(kl.TYPES[fmt], qA, B * 2, M, N, K)
            torch.cuda.synchronize()
            det = torch.equal(C1, C1b)
            d = (C2.float() != C1.float() * 2)
            nbad = int(d.sum())
            msg = ""
            if nbad:
                idx = d.nonzero()[:3].tolist()
                msg = " ".join(f"[{i},{j}] C={C1[i,j].item()} C2={C2[i,j].item()}" for i, j in idx)
            qb1 = kl.quantize_q8_1_device(B); qb2 = kl.quantize_q8_1_device(B * 2)
            v1 = qb1.view(-1, 36); v2 = qb2.view(-1, 36)
            codes_same = torch.equal(v1[:, 4:], v2[:, 4:])
            print(f"{fmt} M={M} K={K} N={N}: deterministic={det} scale2_mismatch={nbad} codes_same={codes_same} {msg}", flush=True)
