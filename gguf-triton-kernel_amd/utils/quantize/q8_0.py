"""Q8_0 producer -- drop-in for the reference's utils/quantize/q8_0.py.

Block (34 B): fp16 d = amax/127 (1.0 for an all-zero block) | int8 qs[32] = rne(x/d).
"""
import torch

from ._qlib import dequantize, quantize


def quantize_to_q8_0(input_tensor: torch.Tensor) -> torch.Tensor:
    """Any-shape tensor (numel % 32 == 0) -> flat int8 CPU tensor of numel/32*34 bytes (q8_0.py:4)."""
    return quantize("q8_0", input_tensor)


def dequantize_q8_0(quantized_tensor: torch.Tensor, original_shape) -> torch.Tensor:
    """Packed Q8_0 bytes -> fp16 tensor of original_shape (q8_0.py:52)."""
    if quantized_tensor.dtype != torch.int8:
        raise ValueError("Quantized tensor must be of type int8")
    if quantized_tensor.numel() % 34 != 0:
        raise ValueError("Invalid quantized tensor size. Expected size divisible by 34 "
                         "(2 scale bytes + 32 quantized values per group).")
    return dequantize("q8_0", quantized_tensor).to(torch.float16).reshape(original_shape)
