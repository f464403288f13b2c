"""Drop-in replacement for the reference's `kernels` package (MI355X / gfx950, HIP).

    from kernels.mmq_q8_0 import mmq_q8_0
    from kernels.mmq_q4_k import mmq_q4_k
    from kernels.mmq_q6_k import mmq_q6_k

Each computes C = (A @ B^T)^T with A a packed GGUF weight tensor (int8, flat) and B fp16
activations (N, K), returning fp16 (N, M) -- the reference's signature and layout.
"""
