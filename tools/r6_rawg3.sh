#!/bin/bash
# (measured, not taken: profiles/r06/kstream_rawg3_ab.txt; needs the round-6 tree of commit 21ac05f..e0e596f)
# Round 6: 3..4 q8_1 tokens on the 7B layer with the raw grouped launch's K-chunked stream for the
# K = 4096 calls (lib/libgguf_mmq_rawg3.so: -DGQ_KSTREAM_RAWG_NMIN=3; LayerMix --raw-split 3: the
# K = 11008 call on its own) against the one grouped decode launch (the product).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VL=gguf-triton-kernel_amd/lib/libgguf_mmq_rawg3.so
timeout -k 10 300 python3 - <<'PY' > gpurun_out/r6_rawg3_check.txt 2>&1 || exit $?
import os, sys
sys.path[:0] = ["oracle", "gguf-triton-kernel_amd", "."]
import kernels._lib as kl
kl.LIB_PATH = os.path.abspath("gguf-triton-kernel_amd/lib/libgguf_mmq_rawg3.so")
import numpy as np, torch
import oracle as O
from utils.synth import random_activations, random_blocks
dev = torch.device("cuda:0")
for N in (3, 4):
    spec = [("q4_k", 4096, 4096), ("q6_k", 1024, 4096), ("q8_0", 512, 4096)]
    B = random_activations(N, 4096, seed=N)
    Bt = torch.from_numpy(B).to(dev)
    items, qAs = [], []
    for i, (f, M, K) in enumerate(spec):
        qA = random_blocks(f, M, K, seed=10 + i)
        qAs.append(qA)
        items.append((kl.TYPES[f], torch.from_numpy(qA.view(np.int8)).to(dev), Bt, M, K, None))
    outs = kl.mmq_grouped(items, N)
    torch.cuda.synchronize()
    for (f, M, K), qA, o in zip(spec, qAs, outs):
        rows = np.arange(0, M, M // 32)
        rb = qA.size // M
        sub = np.concatenate([qA[r * rb:(r + 1) * rb] for r in rows])
        ideal = O.mmq_from_fp16(f, sub, B, len(rows), N, K, O.IDEAL)
        err = O.max_rel_err(o.cpu().numpy()[:, rows], ideal)
        print(N, f, M, K, "max rel err", err, "OK" if err <= 4e-3 else "FAIL")
        assert err <= 4e-3
print("sync timeouts", kl.lib().gq_debug_sync_timeouts())
PY
cat gpurun_out/r6_rawg3_check.txt
for r in 1 2; do
  timeout -k 10 300 python3 tools/layer_time.py 2,3,4,5 --grouped-only | sed "s/^/prod /" || exit $?
  timeout -k 10 300 python3 tools/layer_time.py 2,3,4,5 --grouped-only --lib $VL --raw-split 3 | sed "s/^/rawg3 /" || exit $?
done 2>&1 | grep points | tee gpurun_out/r6_rawg3_layer.txt
