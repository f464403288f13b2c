"""GGUF container I/O (reader + writer) and the Q4_K_M layer-type map."""
from .file import GGML_TYPES, GGUFTensor, read_gguf, write_gguf  # noqa: F401
from .mix import LLAMA_LAYER_SHAPES, q4_k_m_layer_types  # noqa: F401
