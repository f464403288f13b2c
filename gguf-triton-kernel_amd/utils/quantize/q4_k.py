"""Q4_K producer -- drop-in for the reference's utils/quantize/q4_k.py.

Super-block (144 B per 256 weights): fp16 d, fp16 dmin, 12 bytes of 6-bit (scale, min)
pairs for 8 sub-blocks, 128 bytes of 4-bit codes; w = d*sc*q - dmin*m.  Produced by GGML's
reference algorithm (restated in csrc/quant/gguf_quant.cpp), byte-identical.
"""
import torch

from ._qlib import dequantize, quantize

QK_K = 256
K_SCALE_SIZE = 12


def quantize_to_q4_k(input_tensor: torch.Tensor) -> torch.Tensor:
    """Any-shape tensor (numel % 256 == 0) -> flat int8 CPU tensor of numel/256*144 bytes (q4_k.py:87)."""
    return quantize("q4_k", input_tensor)


def dequantize_q4_k(quantized_tensor: torch.Tensor, original_shape) -> torch.Tensor:
    """Packed Q4_K bytes -> fp16 tensor of original_shape (q4_k.py:146)."""
    return dequantize("q4_k", quantized_tensor).to(torch.float16).reshape(original_shape)
