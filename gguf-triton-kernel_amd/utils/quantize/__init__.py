"""GGUF block producers: quantize_to_{q8_0,q8_1,q4_k,q6_k} and dequantize_* (host side).

Byte-identical to the reference's utils/quantize/*.py (tests/golden/golden_quant.npz);
the work is done by libgguf_quant.so (csrc/quant/gguf_quant.cpp).
"""
