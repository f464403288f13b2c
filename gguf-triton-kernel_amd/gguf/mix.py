"""The Q4_K_M layer-type mix of a Llama block (BASELINE.json configs[4]).

llama.cpp's Q4_K_M recipe (not in the reference): every weight Q4_K except attn_v and
ffn_down, which are Q6_K on a subset of layers -- the first eighth, the last eighth and every
third layer in between (use_more_bits(i, n) = i < n/8 || i >= 7n/8 || (i - n/8) % 3 == 2).
"""

# Llama-7B projection shapes (rows M = out features, K = in features)
LLAMA_LAYER_SHAPES = {
    "attn_q": (4096, 4096), "attn_k": (4096, 4096), "attn_v": (4096, 4096), "attn_output": (4096, 4096),
    "ffn_gate": (11008, 4096), "ffn_up": (11008, 4096), "ffn_down": (4096, 11008),
}


def _more_bits(i, n):
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def q4_k_m_layer_types(layer: int, n_layers: int = 32):
    """{projection: gguf type} of layer `layer` of an n_layers model under Q4_K_M."""
    hi = "q6_k" if _more_bits(layer, n_layers) else "q4_k"
    return {name: (hi if name in ("attn_v", "ffn_down") else "q4_k") for name in LLAMA_LAYER_SHAPES}
