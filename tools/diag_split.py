"""Diagnostic: GEMM split-K vs no split on the same inputs, each vs the oracle (GPU)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gguf-triton-kernel_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import oracle as O
from utils.synth import random_blocks, random_activations
import kernels._lib as kl
dev = torch.device("cuda:0")
for fmt in ("q8_0", "q4_k", "q6_k"):
    for (M, N, K) in ((64, 64, 1024), (128, 32, 512), (64, 16, 2048), (256, 128, 1024)):
        qA = random_blocks(fmt, M, K, seed=1)
        B = random_activations(N, K, seed=2)
        ideal = O.mmq_from_fp16(fmt, qA, B, M, N, K, O.IDEAL)
        A_t = torch.from_numpy(qA.view(np.int8)).to(dev); B_t = torch.from_numpy(B).to(dev)
        res = []
        for S in ("1", "2", "4"):
            os.environ["GQ_GEMM_SPLITS"] = S
            C = kl.mmq(kl.TYPES[fmt], A_t, B_t, M, N, K)
            torch.cuda.synchronize()
            c = C.cpu().numpy()
            err = O.max_rel_err(c, ideal)
            # which rows/tokens are wrong
            bad = np.abs(c.astype(np.float32) - ideal.astype(np.float32)) > 0.01 * np.abs(ideal).max()
            rows_bad = np.unique(np.nonzero(bad)[1])[:8].tolist(); toks_bad = np.unique(np.nonzero(bad)[0])[:8].tolist()
            res.append(f"S={S}: err={err:.3g} nbad={int(bad.sum())} rows={rows_bad} toks={toks_bad}")
        os.environ.pop("GQ_GEMM_SPLITS")
        print(fmt, (M, N, K), " | ".join(res), flush=True)
