"""Q6_K producer -- drop-in for the reference's utils/quantize/q6_k.py.

Super-block (210 B per 256 weights): ql[128] low nibbles, qh[64] high 2-bit pairs, int8
scales[16], fp16 d; w = d*sc*(q - 32).  GGML's reference algorithm, byte-identical.
"""
import torch

from ._qlib import dequantize, quantize

QK_K = 256
K_SCALE_SIZE = 16


def quantize_to_q6_k(input_tensor: torch.Tensor) -> torch.Tensor:
    """Any-shape tensor (numel % 256 == 0) -> flat int8 CPU tensor of numel/256*210 bytes (q6_k.py:97)."""
    return quantize("q6_k", input_tensor)


def dequantize_q6_k(quantized_tensor: torch.Tensor, original_shape) -> torch.Tensor:
    """Packed Q6_K bytes -> fp32 tensor of original_shape (q6_k.py:138; the reference returns fp32 here)."""
    return dequantize("q6_k", quantized_tensor).reshape(original_shape)
