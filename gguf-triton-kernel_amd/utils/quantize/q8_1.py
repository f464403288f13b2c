"""Q8_1 producer (activations) -- drop-in for the reference's utils/quantize/q8_1.py.

Block (36 B): fp16 d = amax/127 (0 for an all-zero block) | fp16 s = d*sum(qs) | int8 qs[32].
Device tensors are quantized on the GPU (libgguf_mmq.so, bit-identical); host tensors by
libgguf_quant.so.
"""
import torch

from ._qlib import dequantize, quantize


def quantize_to_q8_1(input_tensor: torch.Tensor) -> torch.Tensor:
    """Any-shape tensor (numel % 32 == 0) -> flat int8 tensor of numel/32*36 bytes on the
    input's device (q8_1.py:18)."""
    if input_tensor.is_cuda:
        import os
        import sys
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        if root not in sys.path:
            sys.path.insert(0, root)
        from kernels._lib import quantize_q8_1_device
        if input_tensor.numel() % 32 != 0:
            raise ValueError("The total number of elements must be divisible by 32.")
        return quantize_q8_1_device(input_tensor.reshape(1, -1))
    return quantize("q8_1", input_tensor)


def dequantize_q8_1(quantized_tensor: torch.Tensor, original_shape) -> torch.Tensor:
    """Packed Q8_1 bytes -> fp16 tensor of original_shape (q8_1.py:73)."""
    if quantized_tensor.dtype != torch.int8:
        raise ValueError("Quantized tensor must be of type int8")
    if quantized_tensor.numel() % 36 != 0:
        raise ValueError("Invalid quantized tensor size. Expected size divisible by 36 "
                         "(4 scale bytes + 32 quantized values per group).")
    return dequantize("q8_1", quantized_tensor).to(torch.float16).reshape(original_shape)
