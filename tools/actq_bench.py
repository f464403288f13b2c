"""Graph-replayed time of the activation quantizer alone (gq_act_prepare: q8_1 -> fp16 x~ for
N >= 5) beside a plain device copy of the same bytes, per (N, K).
Usage: python tools/actq_bench.py [N:K ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gguf-triton-kernel_amd")]
import torch  # noqa: E402

import kernels._lib as kl  # noqa: E402


def timed(fn, reps=100):
    dev = torch.device("cuda:0")
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


dev = torch.device("cuda:0")
for spec in sys.argv[1:] or ["128:4096", "128:8192", "128:11008", "128:28672", "512:4096", "16:4096"]:
    N, K = map(int, spec.split(":"))
    x = torch.randn(N, K, device=dev).to(torch.float16)
    ws = torch.empty(kl.workspace_size(kl.TYPES["q4_k"], 4096, N, K), dtype=torch.uint8, device=dev)
    t_q = timed(lambda: kl.act_prepare(x, N, K, ws))
    y = torch.empty_like(x)
    t_c = timed(lambda: y.copy_(x))
    print(f"N={N:4d} K={K:6d}: act_prepare {t_q:6.2f} us   copy {t_c:6.2f} us   ({2 * N * K / 1e6:.2f} MB in)",
          flush=True)
