"""What the vendor library does on the same GEMM shapes with fp16 weights (a reference point, not a
product path): torch.matmul (hipBLASLt) of fp16 x[N, K] by fp16 W[M, K]^T, graph-replayed over
>= 1 GiB of weight copies (cold in the 256 MB Infinity Cache), and a plain device copy of the
same weight bytes (the achievable HBM read rate).

  python tools/ref_gemm.py [M,K,N ...]      (default: the BASELINE M=128 shapes)"""
import math
import sys

import torch


def timed(fn, n, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    dev = torch.device("cuda:0")
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [
        (4096, 4096, 128), (11008, 4096, 128), (4096, 11008, 128), (28672, 8192, 128), (4096, 4096, 16)]
    for M, K, N in shapes:
        wb = M * K * 2
        nc = max(2, math.ceil((1 << 30) / wb))
        Ws = [torch.randn(M, K, device=dev, dtype=torch.float16) * 0.02 for _ in range(nc)]
        x = torch.randn(N, K, device=dev, dtype=torch.float16)
        outs = [torch.empty(N, M, device=dev, dtype=torch.float16) for _ in range(2)]
        us = timed(lambda i: torch.matmul(x, Ws[i % nc].t(), out=outs[i % 2]), 40)
        dst = torch.empty_like(Ws[0])
        cus = timed(lambda i: dst.copy_(Ws[i % nc]), 40)
        fl = 2.0 * M * N * K
        print(f"M={M} K={K} N={N}: hipBLASLt fp16 {us:.2f} us = {fl / us / 1e6:.1f} TF/s, W read {wb / us / 1e3:.0f} GB/s; "
              f"copy of W {cus:.2f} us = {2 * wb / cus / 1e3:.0f} GB/s (read+write)", flush=True)
        del Ws, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
