"""Mixed-format (GGUF Q4_K_M) projection stack of a Llama block on the MMQ kernels.

BASELINE.json configs[4] / SURVEY.md 8(f)4 (no reference counterpart).  Each projection is a
packed GGUF weight of its own type (gguf.mix.q4_k_m_layer_types); the dispatch is by type,
per matrix.  Projections that read the same input and have the same GGUF type (q/k, and v too
when it is not the Q6_K one; gate/up) are fused once at construction: their packed rows are
copied end to end into one device buffer (the bytes are unchanged -- a packed row is whole
blocks), so each such set is ONE call (one activation quantization, one launch, the split-K
plan of the taller matrix) whose (N, sum M) output is returned as per-projection column views.
Sets that share an input but differ in type quantize the input once (gq_act_prepare) and run
gq_mmq_prepared per weight.  At 1..4 tokens (q8_1 activations) every call of the layer goes
into ONE grouped decode launch (gq_mmq_grouped: the chip's workgroups split over the matrices by
weight bytes, each matrix's rows bit-identical to its own call).  Measured (Q4_K_M 7B layer 0,
graph-replayed, profiles/r03/tails/grouped_q6k_weight_ab.log): 28.8 / 42.3 / 58.8 / 59.5 us at
1 / 2 / 3 / 4 tokens vs 44.2 / 54.1 / 79.9 / 80.2 for the fused sets' own launches.  grouped="auto"
and True take it at 1..4 tokens (a call the grouped launch refuses -- e.g. a long-K Q6_K item
at 3..4 tokens -- runs the sets' own launches), False never.  From 5 tokens on (q8_1) the four
inputs' activations are quantized in one launch (gq_act_prepare_grouped) and every call reads
them prepared: one act_quant launch per layer instead of four.  act="fp8" (the e4m3 variant):
the decode kernel's fp8 form at 1..2 tokens -- one grouped launch (gq_mmq_grouped_ex) at one
token, at two the projections whose 2-token x~ fits LDS grouped and the rest on their own
(40 / 62 us for the 7B layer) -- and from 3 tokens the grouped prepare and prepared calls as
q8_1 from 5 (profiles/r03/s3/fp8_decode.log).
"""
from __future__ import annotations

import torch

from . import _lib


# grouped= setting -> the most tokens LayerMix runs as one grouped decode launch
GROUPED_MAX_TOKENS = {"auto": 4, True: 4, False: 0}
# grouped= setting -> the fewest tokens LayerMix runs as one grouped streaming-GEMM launch (the
# stream-K plan: a 7B layer at 8 tokens 64.1 vs 66.3 us one call per set; profiles/r04/ab9_layer.txt)
GEMM_GROUPED_MIN_TOKENS = {"auto": 5, True: 5, False: 1 << 62}
# activation format -> the fewest tokens whose calls take prepared activations (one quantization
# per input group) instead of quantizing in the decode kernel
PREPARED_MIN_TOKENS = {"q8_1": 5, "fp8": 3}


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

    def __init__(self, linears: dict, act: str = "q8_1", fuse: bool = True, grouped="auto",
                 gemm_grouped_min: int | None = None):
        self.act = act  # "q8_1" (the reference's activation quantization) or "fp8" (e4m3 variant)
        # one gq_mmq_grouped launch for the whole layer: "auto" / True at 1..4 tokens, False never
        self.max_grouped = GROUPED_MAX_TOKENS[grouped]
        # one gq_mmq_grouped_prepared launch (the streaming GEMM) for the whole layer from this
        # many tokens ("auto" / True; False never)
        self.min_gemm_grouped = GEMM_GROUPED_MIN_TOKENS[grouped] if gemm_grouped_min is None else gemm_grouped_min
        self.lin = {}     # name -> GGUFLinear (unfused projections)
        self.parts = {}   # name -> (fused key, first column, rows)
        # per input group: the calls to make, each (key, GGUFLinear); fused keys join names by "+"
        self.calls = []
        for group in self.GROUPS:
            by_type = {}
            for n in group:
                by_type.setdefault(linears[n].type_name, []).append(n)
            calls = []
            for names in by_type.values():
                if fuse and len(names) > 1:
                    L0 = linears[names[0]]
                    A = torch.cat([linears[n].A.reshape(-1) for n in names])  # rows end to end
                    M = sum(linears[n].M for n in names)
                    key = "+".join(names)
                    col = 0
                    for n in names:
                        self.parts[n] = (key, col, linears[n].M)
                        col += linears[n].M
                    calls.append((key, GGUFLinear(L0.type_name, A, M, L0.K)))
                else:
                    for n in names:
                        self.lin[n] = linears[n]
                        calls.append((n, linears[n]))
            self.calls.append(calls)
        self._fused_out = {}

    @classmethod
    def from_gguf(cls, tensors: dict, layer: int, device="cuda", act: str = "q8_1", fuse: bool = True,
                  grouped="auto"):
        """From read_gguf() tensors named blk.<layer>.<proj>.weight."""
        lins = {}
        for group in cls.GROUPS:
            for name in group:
                t = tensors[f"blk.{layer}.{name}.weight"]
                M, K = t.shape
                lins[name] = GGUFLinear(t.type_name, t.to_device(device), M, K)
        return cls(lins, act, fuse, grouped)

    def _out(self, key, L, N, dev, out):
        """Output buffer of one call: the caller's for an unfused projection, else ours."""
        if "+" not in key:
            return None if out is None else out[key]
        buf = self._fused_out.get(key)
        if buf is None or buf.shape[0] != N or buf.device != dev:
            buf = torch.empty((N, L.M), dtype=torch.float16, device=dev)
            self._fused_out[key] = buf
        return buf

    def forward(self, x: torch.Tensor, h: torch.Tensor, *, attn: torch.Tensor | None = None,
                x_ffn: torch.Tensor | None = None, out: dict | None = None) -> dict:
        """{name: (N, M) fp16}.  Fused projections are computed as column ranges of their set's
        (N, sum M) output (kept by the layer and rewritten by the next forward) and returned as
        views of it -- or copied into out[name] when `out` supplies that name's buffer; unfused
        ones are written into out[name] directly when given."""
        res = {}
        inputs = (x, x if attn is None else attn, x if x_ffn is None else x_ffn, h)
        done = False
        if (x.shape[0] <= (self.max_grouped if self.act == "q8_1" else min(2, self.max_grouped))
                and all(inp.shape[0] == x.shape[0] for inp in inputs)):
            N = x.shape[0]
            keys, items = [], []
            for calls, inp in zip(self.calls, inputs):
                for key, L in calls:
                    keys.append(key)
                    items.append((L.gtype, L.A, inp, L.M, inp.shape[1], self._out(key, L, N, inp.device, out)))
            outs = _lib.mmq_grouped(items, N, act=self.act)
            if outs is not None:
                res.update(zip(keys, outs))
                done = True
            elif self.act == "fp8" and N == 2:
                # the fp8 decode form holds 2 tokens' fp16 x~ in LDS: rows of K > 8192 (ffn_down's
                # 11008) do not fit beside the ring -- group the rest, run those on their own
                sub = [i for i, it in enumerate(items) if it[4] <= 8192]
                o = _lib.mmq_grouped([items[i] for i in sub], N, act=self.act) if 0 < len(sub) < len(items) else None
                if o is not None:
                    res.update(zip([keys[i] for i in sub], o))
                    for i, (g, A, inp, M, K, buf) in enumerate(items):
                        if i not in sub:
                            res[keys[i]] = _lib.mmq(g, A, inp, M, N, K, out=buf, act=self.act)
                    done = True
        if not done and all(inp.shape[0] == x.shape[0] for inp in inputs) and x.shape[0] >= PREPARED_MIN_TOKENS[self.act]:
            # every input group's activations quantized in ONE launch (gq_act_prepare_grouped),
            # then every call prepared -- bit-identical to each call quantizing its own input
            N = x.shape[0]
            preps, wss = [], []
            for calls, inp in zip(self.calls, inputs):
                ws_bytes = max(L.workspace_bytes(N, self.act) for _, L in calls)
                ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=inp.device)
                preps.append((inp, N, inp.shape[1], ws))
                wss.append(ws)
            _lib.act_prepare_grouped(preps, act=self.act)
            outs = None
            if N >= self.min_gemm_grouped:
                # every call in ONE grouped streaming-GEMM launch (+ one split-K reduce launch)
                keys, items = [], []
                for calls, inp, ws in zip(self.calls, inputs, wss):
                    for key, L in calls:
                        keys.append(key)
                        items.append((L.gtype, L.A, ws, L.M, inp.shape[1], self._out(key, L, N, inp.device, out)))
                outs = _lib.mmq_grouped_prepared(items, N, act=self.act)
                if outs is not None:
                    res.update(zip(keys, outs))
            if outs is None:
                for calls, inp, ws in zip(self.calls, inputs, wss):
                    for key, L in calls:
                        res[key] = _lib.mmq_prepared(L.gtype, L.A, ws, L.M, N, inp.shape[1],
                                                     self._out(key, L, N, inp.device, out), act=self.act)
            done = True
        if not done:
            for calls, inp in zip(self.calls, inputs):
                N, K = inp.shape
                if N < PREPARED_MIN_TOKENS[self.act] or len(calls) == 1:
                    # decode (each call quantizes its tokens in-kernel), or a single call
                    for key, L in calls:
                        res[key] = _lib.mmq(L.gtype, L.A, inp, L.M, N, K, out=self._out(key, L, N, inp.device, out),
                                            act=self.act)
                else:
                    ws_bytes = max(L.workspace_bytes(N, self.act) for _, L in calls)
                    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=inp.device)
                    _lib.act_prepare(inp, N, K, ws, act=self.act)
                    for key, L in calls:
                        res[key] = _lib.mmq_prepared(L.gtype, L.A, ws, L.M, N, K,
                                                     self._out(key, L, N, inp.device, out), act=self.act)
        for n, (key, col, rows) in self.parts.items():
            view = res[key][:, col:col + rows]
            if out is not None and n in out:
                out[n].copy_(view)
                view = out[n]
            res[n] = view
        for key in [k for k in res if "+" in k]:
            del res[key]
        return res
