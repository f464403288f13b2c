"""GGUF container round trip and the Q4_K_M type map (CPU); the mixed-type layer on the GPU
is in test_gpu_parity.py::test_layer_mix_from_gguf."""
import numpy as np

from gguf import GGML_TYPES, q4_k_m_layer_types, read_gguf, write_gguf
from utils.synth import random_blocks


def test_gguf_round_trip(tmp_path):
    tensors = {
        "blk.0.attn_q.weight": ("q4_k", (8, 512), random_blocks("q4_k", 8, 512, seed=1)),
        "blk.0.attn_v.weight": ("q6_k", (5, 256), random_blocks("q6_k", 5, 256, seed=2)),
        "blk.0.ffn_down.weight": ("q8_0", (3, 96), random_blocks("q8_0", 3, 96, seed=3)),
    }
    p = tmp_path / "t.gguf"
    write_gguf(p, tensors, {"general.architecture": "llama", "llama.block_count": 1})
    meta, got = read_gguf(p)
    assert meta["general.architecture"] == "llama" and meta["llama.block_count"] == 1
    assert set(got) == set(tensors)
    for name, (t, shape, raw) in tensors.items():
        g = got[name]
        assert g.type_name == t and g.shape == shape and g.offset % 32 == 0
        assert np.array_equal(np.asarray(g.data), raw.view(np.uint8).reshape(-1))


def test_gguf_type_table():
    assert GGML_TYPES[12] == ("q4_k", 256, 144) and GGML_TYPES[14] == ("q6_k", 256, 210)
    assert GGML_TYPES[8] == ("q8_0", 32, 34)


def test_q4_k_m_mix():
    n = 32
    hi = [i for i in range(n) if q4_k_m_layer_types(i, n)["ffn_down"] == "q6_k"]
    # first and last eighth, every third layer in between (llama.cpp use_more_bits)
    assert hi[:4] == [0, 1, 2, 3] and hi[-4:] == [28, 29, 30, 31] and 6 in hi and 5 not in hi
    for i in range(n):
        t = q4_k_m_layer_types(i, n)
        assert t["attn_q"] == t["ffn_gate"] == "q4_k" and t["attn_v"] == t["ffn_down"]
