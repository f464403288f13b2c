"""tests/golden/make_golden.py -- capture golden vectors from the reference itself.

Run in the build container only (needs /root/reference; the GPU box never has it):

    make -C oracle ref            # compiles the reference's q4_k_ref.c / q6_k_ref.c
    python tests/golden/make_golden.py

The reference's quantizers load lib*_ref.so from their own directory
(utils/quantize/q4_k.py:39-46, q6_k.py:49-56) and /root/reference is read-only, so the
script copies the reference tree to a temporary directory OUTSIDE the repo, drops the
oracle/_ref/*.so next to the loaders, and imports from there.  Only data (inputs and the
reference's outputs) is written into tests/golden/*.npz; no reference source travels.

Produces, per format f in {q8_0, q4_k, q6_k}:
  golden_{f}.npz    matmul vectors: sweep of the reference test shapes
                    (test/test_mmq_*.py:17-21) with fixed seeds, BASELINE-config row
                    slices, edge cases.  Keys per case i:
                      c{i}_MNK      int64[3]
                      c{i}_B        fp16 (N, K) activations
                      c{i}_qA       uint8 packed weights   (reference quantizer)
                      c{i}_qB       uint8 q8_1 activations (utils/quantize/q8_1.py)
                      c{i}_C        fp16 (N, M) kernels/cpu_impls output
                      c{i}_Ctri     fp16 (N, M) reference Triton kernel, TRITON_INTERPRET=1
                                    (sweep cases only)
  golden_quant.npz  quantizer vectors: fp16 inputs -> reference bytes for
                    quantize_to_{q8_0,q8_1,q4_k,q6_k}.
"""
import os
import shutil
import sys
import tempfile
import time

import numpy as np

os.environ.setdefault("TRITON_INTERPRET", "1")
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = os.environ.get("GGUF_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")


def _import_reference():
    refso = os.path.join(REPO, "oracle", "_ref")
    for so in ("libq4_k_ref.so", "libq6_k_ref.so"):
        if not os.path.exists(os.path.join(refso, so)):
            raise SystemExit("run `make -C oracle ref` first")
    tmp = tempfile.mkdtemp(prefix="gguf_ref_")
    dst = os.path.join(tmp, "ref")
    shutil.copytree(REF, dst)
    for so in ("libq4_k_ref.so", "libq6_k_ref.so"):
        shutil.copy(os.path.join(refso, so), os.path.join(dst, "utils", "quantize", so))
    sys.path.insert(0, dst)
    from utils.quantize.q8_0 import quantize_to_q8_0
    from utils.quantize.q8_1 import quantize_to_q8_1
    from utils.quantize.q4_k import quantize_to_q4_k
    from utils.quantize.q6_k import quantize_to_q6_k
    from kernels.cpu_impls.mmq_q8_0_q8_1_cpu import mmq_q8_0_q8_1_cpu
    from kernels.cpu_impls.mmq_q4_k_q8_1_cpu import mmq_q4_k_q8_1_cpu
    from kernels.cpu_impls.mmq_q6_k_q8_1_cpu import mmq_q6_k_q8_1_cpu
    from kernels.mmq_q8_0 import mmq_q8_0
    from kernels.mmq_q4_k import mmq_q4_k
    from kernels.mmq_q6_k import mmq_q6_k
    return dict(
        quant={"q8_0": quantize_to_q8_0, "q4_k": quantize_to_q4_k, "q6_k": quantize_to_q6_k},
        q8_1=quantize_to_q8_1,
        cpu={"q8_0": mmq_q8_0_q8_1_cpu, "q4_k": mmq_q4_k_q8_1_cpu, "q6_k": mmq_q6_k_q8_1_cpu},
        tri={"q8_0": mmq_q8_0, "q4_k": mmq_q4_k, "q6_k": mmq_q6_k},
        tmp=tmp,
    )


def _np16(t):
    return t.contiguous().numpy().view(np.uint16).view(np.float16)


def _u8(t):
    return t.contiguous().numpy().view(np.uint8)


def matmul_cases(fmt):
    """(M_w, N_tok, K, kind, seed, with_triton) list."""
    cases = []
    kpows = range(5, 10) if fmt == "q8_0" else range(8, 11)
    seed = 0
    for mp in range(0, 6, 2):  # test/test_mmq_*.py:17-21
        for np_ in range(0, 6, 2):
            for kp in kpows:
                cases.append((2 ** mp, 2 ** np_, 2 ** kp, "sweep", seed, True))
                seed += 1
    # BASELINE-config row slices (BASELINE.json configs 1-4): few weight rows, full K
    if fmt == "q8_0":
        big = [(8, 1, 4096), (8, 16, 4096)]
    elif fmt == "q4_k":
        big = [(8, 1, 4096), (8, 16, 4096), (8, 1, 11008), (8, 4, 11008)]
    else:
        big = [(8, 1, 8192), (8, 4, 8192), (4, 1, 28672), (4, 4, 28672)]
    for (m, n, k) in big:
        cases.append((m, n, k, "slice", 1000 + seed, False))
        seed += 1
    # edge cases: zero activation block, zero weight block, huge/tiny scales
    k0 = 512 if fmt != "q8_0" else 256
    for kind in ("zero_act_block", "zero_weight_block", "large", "tiny", "outlier"):
        cases.append((4, 3, k0, kind, 2000 + seed, False))
        seed += 1
    return cases


def make_inputs(M, N, K, kind, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, K, generator=g, dtype=torch.float32).to(torch.float16)
    B = torch.randn(N, K, generator=g, dtype=torch.float32).to(torch.float16)
    if kind == "zero_act_block":
        B[:, 32:64] = 0
        B[-1, :] = 0
    elif kind == "zero_weight_block":
        A[0, :256] = 0
        A[1, :] = 0
    elif kind == "large":
        A = (A.float() * 30).to(torch.float16)
        B = (B.float() * 10).to(torch.float16)
    elif kind == "tiny":
        A = (A.float() * 1e-3).to(torch.float16)
        B = (B.float() * 1e-2).to(torch.float16)
    elif kind == "outlier":
        A[:, 5] = 40.0
        B[:, 7] = -50.0
    return A, B


def gen_matmul(ref, fmt):
    arrays = {}
    t0 = time.time()
    for i, (M, N, K, kind, seed, with_tri) in enumerate(matmul_cases(fmt)):
        A, B = make_inputs(M, N, K, kind, seed)
        qA = ref["quant"][fmt](A)
        qB = ref["q8_1"](B)
        C = ref["cpu"][fmt](qA, qB, M, N, K)
        arrays[f"c{i}_MNK"] = np.array([M, N, K], np.int64)
        arrays[f"c{i}_kind"] = np.array(kind)
        arrays[f"c{i}_B"] = _np16(B)
        arrays[f"c{i}_qA"] = _u8(qA)
        arrays[f"c{i}_qB"] = _u8(qB)
        arrays[f"c{i}_C"] = _np16(C)
        if with_tri:
            Ct = ref["tri"][fmt](qA, B, M, N, K)
            arrays[f"c{i}_Ctri"] = _np16(Ct)
        print(f"  {fmt} case {i} M={M} N={N} K={K} {kind} ({time.time() - t0:.1f}s)", flush=True)
    np.savez_compressed(os.path.join(OUT, f"golden_{fmt}.npz"), **arrays)


def quant_inputs():
    """Named fp16 inputs (flattened rows of 256-multiples) for the quantizer vectors."""
    g = torch.Generator().manual_seed(7)
    ins = {}
    ins["normal"] = torch.randn(64, 256, generator=g).to(torch.float16)
    ins["uniform"] = (torch.rand(32, 256, generator=g) * 2 - 1).to(torch.float16)
    ins["positive"] = torch.rand(16, 256, generator=g).to(torch.float16)
    ins["negative"] = (-torch.rand(16, 256, generator=g)).to(torch.float16)
    ins["scaled_big"] = (torch.randn(16, 256, generator=g) * 1000).to(torch.float16)
    ins["scaled_small"] = (torch.randn(16, 256, generator=g) * 1e-3).to(torch.float16)
    z = torch.randn(16, 256, generator=g).to(torch.float16)
    z[0] = 0
    z[1, :32] = 0
    z[2, 100:140] = 0
    z[3] = 1.5
    z[4, ::2] = 0
    z[5, 17] = 300.0
    ins["special"] = z
    ins["heavy_tail"] = (torch.randn(32, 256, generator=g) ** 3).to(torch.float16)
    ins["llm_like"] = (torch.randn(64, 256, generator=g) * 0.02).to(torch.float16)
    return ins


def gen_quant(ref):
    arrays = {}
    for name, x in quant_inputs().items():
        arrays[f"{name}_x"] = _np16(x)
        for fmt in ("q8_0", "q4_k", "q6_k"):
            arrays[f"{name}_{fmt}"] = _u8(ref["quant"][fmt](x))
        arrays[f"{name}_q8_1"] = _u8(ref["q8_1"](x))
    np.savez_compressed(os.path.join(OUT, "golden_quant.npz"), **arrays)


def main():
    torch.set_num_threads(4)
    ref = _import_reference()
    try:
        gen_quant(ref)
        for fmt in ("q8_0", "q4_k", "q6_k"):
            gen_matmul(ref, fmt)
    finally:
        shutil.rmtree(ref["tmp"], ignore_errors=True)


if __name__ == "__main__":
    main()
