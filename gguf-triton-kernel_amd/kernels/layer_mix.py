"""Mixed-format (GGUF Q4_K_M) projection stack of a Llama block on the MMQ kernels.

BASELINE.json configs[4] / SURVEY.md 8(f)4 (no reference counterpart).  Each projection is a
packed GGUF weight of its own type (gguf.mix.q4_k_m_layer_types); projections that share an
input (q/k/v, gate/up) quantize it once (gq_act_prepare) and run gq_mmq_prepared per
weight -- the dispatch is by type, per matrix, with no repacking.  At decode sizes (N <= 4)
every call is the one-launch fused decode kernel instead (its quantizer is in-kernel).
"""
from __future__ import annotations

import torch

from . import _lib


class GGUFLinear:
    """y = x @ W^T for a packed GGUF weight W (M rows of K elements) on the device."""

    def __init__(self, type_name: str, A: torch.Tensor, M: int, K: int):
        self.type_name, self.gtype = type_name, _lib.TYPES[type_name]
        self.A, self.M, self.K = A, M, K

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return _lib.mmq(self.gtype, self.A, x, self.M, x.shape[0], self.K)

    def workspace_bytes(self, N: int, act: str = "q8_1") -> int:
        return _lib.workspace_size(self.gtype, self.M, N, self.K, act)


class LayerMix:
    """The seven projections of one Llama block, grouped by the input they read:
    attn_q/k/v read the attention-normed hidden state x (K = 4096), attn_output the attention
    output `attn`, ffn_gate/up the FFN-normed hidden state `x_ffn`, ffn_down the gated FFN
    activation h (K = 11008).  forward(x, h, attn, x_ffn) -> {name: (N, M) fp16}; attn and
    x_ffn default to x (the benchmark feeds one synthetic input to every K = 4096 group)."""

    GROUPS = (("attn_q", "attn_k", "attn_v"), ("attn_output",), ("ffn_gate", "ffn_up"), ("ffn_down",))

    def __init__(self, linears: dict, act: str = "q8_1"):
        self.lin = linears
        self.act = act  # "q8_1" (the reference's activation quantization) or "fp8" (e4m3 variant)

    @classmethod
    def from_gguf(cls, tensors: dict, layer: int, device="cuda", act: str = "q8_1"):
        """From read_gguf() tensors named blk.<layer>.<proj>.weight."""
        lins = {}
        for group in cls.GROUPS:
            for name in group:
                t = tensors[f"blk.{layer}.{name}.weight"]
                M, K = t.shape
                lins[name] = GGUFLinear(t.type_name, t.to_device(device), M, K)
        return cls(lins, act)

    def forward(self, x: torch.Tensor, h: torch.Tensor, attn: torch.Tensor | None = None,
                x_ffn: torch.Tensor | None = None, out: dict | None = None) -> dict:
        res = {}
        inputs = (x, x if attn is None else attn, x if x_ffn is None else x_ffn, h)
        for group, inp in zip(self.GROUPS, inputs):
            N, K = inp.shape
            if N <= 4 and self.act == "q8_1":  # decode: each call quantizes its tokens in LDS (one launch)
                for n in group:
                    L = self.lin[n]
                    res[n] = _lib.mmq(L.gtype, L.A, inp, L.M, N, K, out=None if out is None else out[n])
                continue
            ws_bytes = max(self.lin[n].workspace_bytes(N, self.act) for n in group)
            ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=inp.device)
            _lib.act_prepare(inp, N, K, ws, act=self.act)
            for n in group:
                L = self.lin[n]
                res[n] = _lib.mmq_prepared(L.gtype, L.A, ws, L.M, N, K, None if out is None else out[n], act=self.act)
        return res
