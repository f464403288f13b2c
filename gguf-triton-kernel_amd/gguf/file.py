"""Minimal GGUF (v2/v3) reader and writer for the block formats this library multiplies.

Not part of the reference ("GGUF tensor reader + Q4_K_M layer dispatcher,
not in reference"): it lets real llama.cpp checkpoints feed kernels.mmq_* without copies.
Layout (GGUF spec, little endian): magic "GGUF", u32 version, u64 n_tensors, u64 n_kv, then
n_kv metadata entries (string key, u32 type, value), n_tensors tensor infos (string name,
u32 n_dims, u64 dims[n_dims] (innermost first), u32 ggml type, u64 offset), padding to
`general.alignment` (default 32), and the tensor data.  A GGUF 2-D weight has dims
(K, M): K elements per row, M rows -- exactly the packed row layout kernels.mmq_* take.

Tensors are returned as numpy memory maps (no copy); `.to_device()` makes the int8 tensor the
drop-in API expects.  Only built-in value types are handled (no pickles, nothing executed).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

GGUF_MAGIC = b"GGUF"
# ggml type id -> (name, block elements, block bytes)
GGML_TYPES = {0: ("f32", 1, 4), 1: ("f16", 1, 2), 8: ("q8_0", 32, 34), 12: ("q4_k", 256, 144),
              14: ("q6_k", 256, 210)}
TYPE_IDS = {v[0]: k for k, v in GGML_TYPES.items()}

# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f", _BOOL: "<?",
           _U64: "<Q", _I64: "<q", _F64: "<d"}


@dataclass
class GGUFTensor:
    name: str
    type_name: str   # "q4_k", "q6_k", "q8_0", "f16", "f32"
    dims: tuple      # GGUF order: innermost (K) first
    offset: int      # from the start of the data section
    data: np.ndarray  # raw bytes (uint8 memmap)

    @property
    def shape(self):
        """(M, K): rows x elements per row (reverse of the GGUF dims)."""
        return tuple(reversed(self.dims))

    def to_device(self, device="cuda"):
        import torch
        return torch.from_numpy(np.array(self.data, dtype=np.uint8).view(np.int8)).to(device)  # host copy: memmaps are read-only


class _Reader:
    def __init__(self, buf):
        self.b, self.o = buf, 0

    def take(self, fmt):
        v = struct.unpack_from(fmt, self.b, self.o)[0]
        self.o += struct.calcsize(fmt)
        return v

    def string(self):
        n = self.take("<Q")
        s = bytes(self.b[self.o:self.o + n]).decode("utf-8")
        self.o += n
        return s

    def value(self, t):
        if t in _SCALAR:
            return self.take(_SCALAR[t])
        if t == _STR:
            return self.string()
        if t == _ARR:
            et, n = self.take("<I"), self.take("<Q")
            return [self.value(et) for _ in range(n)]
        raise ValueError(f"unknown GGUF metadata type {t}")


def read_gguf(path):
    """(metadata dict, {name: GGUFTensor}) of a GGUF file, tensors memory-mapped."""
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    r = _Reader(memoryview(mm))
    if bytes(mm[:4]) != GGUF_MAGIC:
        raise ValueError(f"{path}: not a GGUF file")
    r.o = 4
    version = r.take("<I")
    if version not in (2, 3):
        raise ValueError(f"{path}: unsupported GGUF version {version}")
    n_tensors, n_kv = r.take("<Q"), r.take("<Q")
    meta = {}
    for _ in range(n_kv):
        k = r.string()
        meta[k] = r.value(r.take("<I"))
    infos = []
    for _ in range(n_tensors):
        name = r.string()
        nd = r.take("<I")
        dims = tuple(r.take("<Q") for _ in range(nd))
        t = r.take("<I")
        off = r.take("<Q")
        infos.append((name, dims, t, off))
    align = int(meta.get("general.alignment", 32))
    data0 = (r.o + align - 1) // align * align
    tensors = {}
    for name, dims, t, off in infos:
        if t not in GGML_TYPES:
            raise ValueError(f"tensor {name}: ggml type {t} not supported")
        tname, qk, bb = GGML_TYPES[t]
        n = int(np.prod(dims))
        if dims[0] % qk:
            raise ValueError(f"tensor {name}: row of {dims[0]} not a multiple of {qk}")
        nbytes = n // qk * bb
        start = data0 + off
        tensors[name] = GGUFTensor(name, tname, dims, off, mm[start:start + nbytes])
    return meta, tensors


def _w_str(f, s):
    b = s.encode("utf-8")
    f.write(struct.pack("<Q", len(b)))
    f.write(b)


def _w_val(f, v):
    if isinstance(v, bool):
        f.write(struct.pack("<I?", _BOOL, v))
    elif isinstance(v, int):
        f.write(struct.pack("<Iq", _I64, v))
    elif isinstance(v, float):
        f.write(struct.pack("<If", _F32, v))
    elif isinstance(v, str):
        f.write(struct.pack("<I", _STR))
        _w_str(f, v)
    else:
        raise TypeError(f"metadata value {v!r}")


def write_gguf(path, tensors, metadata=None, alignment=32):
    """Write a GGUF v3 file.  tensors: {name: (type_name, (M, K), raw bytes ndarray)}."""
    metadata = dict(metadata or {})
    metadata.setdefault("general.alignment", alignment)
    with open(path, "wb") as f:
        f.write(GGUF_MAGIC)
        f.write(struct.pack("<IQQ", 3, len(tensors), len(metadata)))
        for k, v in metadata.items():
            _w_str(f, k)
            _w_val(f, v)
        off = 0
        blobs = []
        for name, (tname, (M, K), raw) in tensors.items():
            _, qk, bb = GGML_TYPES[TYPE_IDS[tname]]
            raw = np.ascontiguousarray(raw).view(np.uint8).reshape(-1)
            assert raw.size == M * K // qk * bb, f"{name}: {raw.size} bytes for {tname} {M}x{K}"
            _w_str(f, name)
            f.write(struct.pack("<I", 2))
            f.write(struct.pack("<QQ", K, M))
            f.write(struct.pack("<IQ", TYPE_IDS[tname], off))
            blobs.append((off, raw))
            off = (off + raw.size + alignment - 1) // alignment * alignment
        pos = f.tell()
        data0 = (pos + alignment - 1) // alignment * alignment
        f.write(b"\0" * (data0 - pos))
        for o, raw in blobs:
            cur = f.tell() - data0
            f.write(b"\0" * (o - cur))
            f.write(raw.tobytes())
