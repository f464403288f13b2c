"""Host-side LayerMix fusion plan (no GPU): which projections become one call, and that the fused
weight is the members' packed rows end to end, byte for byte."""
import numpy as np
import torch

from gguf import LLAMA_LAYER_SHAPES, q4_k_m_layer_types
from kernels.layer_mix import GGUFLinear, LayerMix


def _linears(types, shapes, row_bytes=8):
    out = {}
    for i, (n, (M, K)) in enumerate(shapes.items()):
        A = torch.from_numpy(np.full(M * row_bytes, i, dtype=np.int8))
        out[n] = GGUFLinear(types[n], A, M, K)
    return out


def test_fusion_plan_q4_k_m_layers():
    for layer, v_type in ((0, "q6_k"), (5, "q4_k")):
        types = q4_k_m_layer_types(layer, 32)
        assert types["attn_v"] == v_type
        lm = LayerMix(_linears(types, LLAMA_LAYER_SHAPES))
        keys = [[k for k, _ in c] for c in lm.calls]
        qkv = ["attn_q+attn_k", "attn_v"] if v_type == "q6_k" else ["attn_q+attn_k+attn_v"]
        assert keys == [qkv, ["attn_output"], ["ffn_gate+ffn_up"], ["ffn_down"]], keys
        assert lm.parts["ffn_up"] == ("ffn_gate+ffn_up", 11008, 11008)
        fused = dict(lm.calls[2])["ffn_gate+ffn_up"]
        assert fused.M == 22016 and fused.K == 4096 and fused.type_name == "q4_k"


def test_fused_bytes_end_to_end():
    types = q4_k_m_layer_types(5, 32)
    lins = _linears(types, LLAMA_LAYER_SHAPES)
    lm = LayerMix(lins)
    fused = dict(lm.calls[0])["attn_q+attn_k+attn_v"]
    want = torch.cat([lins[n].A.reshape(-1) for n in ("attn_q", "attn_k", "attn_v")])
    assert torch.equal(fused.A, want)


def test_unfused_plan():
    types = q4_k_m_layer_types(0, 32)
    lm = LayerMix(_linears(types, LLAMA_LAYER_SHAPES), fuse=False)
    assert not lm.parts
    assert [[k for k, _ in c] for c in lm.calls] == [["attn_q", "attn_k", "attn_v"], ["attn_output"],
                                                      ["ffn_gate", "ffn_up"], ["ffn_down"]]
