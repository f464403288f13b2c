"""Loader and thin torch front end for libgguf_mmq.so (the C ABI in include/gguf_mmq.h).

The library is built in-tree (`make -C gguf-triton-kernel_amd`, or __graft_entry__.build()).
There is no fallback: if the HIP library is missing or no ROCm device is present, the
MMQ entry points raise.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libgguf_mmq.so")

GQ_Q8_0, GQ_Q4_K, GQ_Q6_K = 0, 1, 2
GQ_ACT_Q8_1, GQ_ACT_FP8_E4M3 = 0, 1
ACTS = {"q8_1": GQ_ACT_Q8_1, "fp8": GQ_ACT_FP8_E4M3}
TYPES = {"q8_0": GQ_Q8_0, "q4_k": GQ_Q4_K, "q6_k": GQ_Q6_K}
BLOCK_ELEMS = {GQ_Q8_0: 32, GQ_Q4_K: 256, GQ_Q6_K: 256}
BLOCK_BYTES = {GQ_Q8_0: 34, GQ_Q4_K: 144, GQ_Q6_K: 210}

# symbol -> (argtypes, restype); mirrors include/gguf_mmq.h
_P, _I64, _I, _SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_size_t
GQ_OK, GQ_EINVAL, GQ_EHIP, GQ_EUNSUPPORTED = 0, 1, 2, 3


class GroupItem(ctypes.Structure):
    """gq_group_item (include/gguf_mmq.h)."""
    _fields_ = [("type", ctypes.c_int), ("A", _P), ("B", _P), ("ldb", _I64), ("C", _P), ("ldc", _I64),
                ("M", _I64), ("K", _I64)]


class PrepItem(ctypes.Structure):
    """gq_prep_item (include/gguf_mmq.h)."""
    _fields_ = [("B", _P), ("N", _I64), ("K", _I64), ("ldb", _I64), ("workspace", _P), ("workspace_bytes", _SZ)]


class GemmItem(ctypes.Structure):
    """gq_gemm_item (include/gguf_mmq.h)."""
    _fields_ = [("type", ctypes.c_int), ("A", _P), ("ws", _P), ("C", _P), ("ldc", _I64), ("M", _I64), ("K", _I64)]


SIGNATURES = {
    "gq_block_elems": ([_I], _I),
    "gq_block_bytes": ([_I], _I),
    "gq_mmq_workspace_size": ([_I, _I64, _I64, _I64], _SZ),
    "gq_mmq": ([_I, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P], _I),
    "gq_act_prepare": ([_P, _I64, _I64, _I64, _P, _SZ, _P], _I),
    "gq_mmq_prepared": ([_I, _P, _P, _SZ, _P, _I64, _I64, _I64, _I64, _P], _I),
    "gq_quantize_q8_1": ([_P, _P, _I64, _I64, _I64, _P], _I),
    "gq_dequantize": ([_I, _P, _P, _I64, _I64, _I64, _P], _I),
    "gq_mmq_workspace_size_ex": ([_I, _I, _I64, _I64, _I64], _SZ),
    "gq_mmq_call_workspace_size": ([_I, _I, _I64, _I64, _I64], _SZ),
    "gq_mmq_ex": ([_I, _I, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _P, _SZ, _P], _I),
    "gq_act_prepare_ex": ([_I, _P, _I64, _I64, _I64, _P, _SZ, _P], _I),
    "gq_mmq_prepared_ex": ([_I, _I, _P, _P, _SZ, _P, _I64, _I64, _I64, _I64, _P], _I),
    "gq_quantize_fp8": ([_P, _P, _P, _I64, _I64, _I64, _P], _I),
    "gq_quantize_weights": ([_I, _P, _P, _I64, _P], _I),
    "gq_shard_rows": ([_I64, _I, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                       ctypes.POINTER(ctypes.c_int64)], _I),
    "gq_assemble_shards": ([_P, _P, _I, _I64, _I64, _I64, _I64, _P], _I),
    "gq_mmq_sharded_workspace_size": ([_I, _I64, _I64, _I64, _I], _SZ),
    "gq_mmq_sharded": ([_I, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I, _I, _P, _P, _SZ, _P], _I),
    "gq_mmq_grouped": ([ctypes.POINTER(GroupItem), _I, _I64, _P], _I),
    "gq_mmq_grouped_ex": ([_I, ctypes.POINTER(GroupItem), _I, _I64, _P], _I),
    "gq_act_prepare_grouped": ([_I, ctypes.POINTER(PrepItem), _I, _P], _I),
    "gq_debug_route": ([_I, _I, _I64, _I64, _I64, _I], ctypes.c_char_p),
    "gq_mmq_grouped_prepared_workspace_size": ([_I, ctypes.POINTER(GemmItem), _I, _I64], _SZ),
    "gq_mmq_grouped_prepared": ([_I, ctypes.POINTER(GemmItem), _I, _I64, _P, _SZ, _P], _I),
    "gq_last_error": ([], ctypes.c_char_p),
    "gq_version": ([], _I),
    "gq_debug_set_tuning": ([ctypes.c_char_p, ctypes.c_longlong], _I),
    "gq_debug_reset_tuning": ([], None),
    "gq_debug_sync_timeouts": ([], ctypes.c_uint),
}

_lib = None
_call_ws = {}  # (gtype, act, M, N, K) -> bytes one gq_mmq_ex call needs (0: one-launch decode)


def lib():
    """The loaded libgguf_mmq.so (raises RuntimeError when it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not found: build the HIP library first "
                "(make -C gguf-triton-kernel_amd, or python -c 'import __graft_entry__ as g; g.build()')")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (argtypes, restype) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _lib = handle
    return _lib


def _bind_mmq_ex():
    """gq_mmq_ex as the eager path calls it: through lib/_gqcall (csrc/gq_pycall.c, a METH_FASTCALL
    entry bound to the ctypes-loaded library's gq_mmq_ex -- ~0.2 us per call instead of ctypes'
    ~1.5-2 us of argument conversion), or the ctypes function when that module was not built.
    Both reach the same gq_mmq_ex in the same loaded libgguf_mmq.so."""
    import importlib.machinery
    import importlib.util
    fn = lib().gq_mmq_ex
    # only a build for THIS interpreter's ABI (lib/ may hold builds for several Pythons)
    for suffix in importlib.machinery.EXTENSION_SUFFIXES:
        path = os.path.join(LIB_DIR, "_gqcall" + suffix)
        if not os.path.exists(path):
            continue
        try:
            spec = importlib.util.spec_from_file_location("_gqcall", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
        except ImportError:
            continue
        mod.bind(ctypes.cast(fn, ctypes.c_void_p).value)
        return mod.mmq_ex
    return fn


def set_tuning(key: str, value: int):
    """Override one GQ_* tuning default by name for later calls (gq_debug_set_tuning; the
    library reads the environment once, so setting os.environ later has no effect)."""
    _call_ws.clear()  # (the workspace a shape needs depends on the tuning)
    _check(lib().gq_debug_set_tuning(key.encode(), int(value)))


def route_name(gtype: int, M: int, N: int, K: int, act: str = "q8_1", prepared: bool = False) -> str:
    """The kernel(s) the library would launch for this call (gq_debug_route)."""
    return lib().gq_debug_route(gtype, ACTS[act], M, N, K, int(prepared)).decode()


def reset_tuning():
    """Back to the tuning values the environment gave at first use."""
    _call_ws.clear()
    lib().gq_debug_reset_tuning()


class tuning:
    """Context manager: `with tuning(GQ_GEMM_SPLITS=8, GQ_RGEMM=0): ...` (values reset on exit)."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        for k, v in self.kw.items():
            set_tuning(k, v)
        return self

    def __exit__(self, *exc):
        reset_tuning()
        return False


def _check(status: int):
    if status != 0:
        msg = lib().gq_last_error().decode(errors="replace")
        raise RuntimeError(f"gguf_mmq error {status}: {msg}")


def _require_device(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a ROCm device tensor (got device {t.device}); "
                           "the MMQ kernels have no CPU path")


def workspace_size(gtype: int, M: int, N: int, K: int, act: str = "q8_1") -> int:
    return int(lib().gq_mmq_workspace_size_ex(gtype, ACTS[act], M, N, K))


def _check_weights(gtype: int, A: torch.Tensor, M: int, K: int):
    qk, bb = BLOCK_ELEMS[gtype], BLOCK_BYTES[gtype]
    _require_device(A, "A")
    if A.dtype not in (torch.int8, torch.uint8):
        raise RuntimeError(f"A must be the packed int8/uint8 block tensor, got {A.dtype}")
    if not A.is_contiguous():
        raise RuntimeError("A (packed blocks) must be contiguous")
    if A.numel() != M * (K // qk) * bb:
        raise RuntimeError(f"A has {A.numel()} bytes, expected M*K/{qk}*{bb} = {M * (K // qk) * bb}")


def _check_acts(B: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """B as the fp16 (N, K) unit-column-stride tensor the ABI reads."""
    _require_device(B, "B")
    if B.dtype != torch.float16:
        B = B.to(torch.float16)
    if B.dim() != 2 or B.shape[0] != N or B.shape[1] != K:
        if B.numel() != N * K:
            raise RuntimeError(f"B has {B.numel()} elements, expected N*K = {N * K}")
        B = B.reshape(N, K)
    if B.stride(1) != 1:
        B = B.contiguous()
    return B


def _check_out(out: torch.Tensor | None, N: int, M: int, dev) -> torch.Tensor:
    C = out if out is not None else torch.empty((N, M), dtype=torch.float16, device=dev)
    if C.dtype != torch.float16 or C.dim() != 2 or C.stride(1) != 1 or C.shape[0] != N or C.shape[1] != M:
        raise RuntimeError("out must be an fp16 (N, M) tensor with unit column stride")
    if C.device != dev:
        raise RuntimeError(f"out on {C.device}, expected {dev}")
    return C


def _check_workspace(ws: torch.Tensor, need: int, dev):
    if ws.device != dev or ws.dtype != torch.uint8 or not ws.is_contiguous():
        raise RuntimeError("workspace must be a contiguous uint8 tensor on the weights' device")
    if ws.numel() < need:
        raise RuntimeError(f"workspace has {ws.numel()} bytes, this call needs {need}")


def _stream(dev) -> int:
    """torch's current HIP stream on `dev` (the raw handle: the Stream object costs ~2 us)."""
    return torch._C._cuda_getCurrentRawStream(dev.index if dev.index is not None else torch.cuda.current_device())


_F16, _I8, _U8 = torch.float16, torch.int8, torch.uint8
_empty, _get_device, _raw_stream = torch.empty, torch._C._cuda_getDevice, torch._C._cuda_getCurrentRawStream
_mmq_ex = None  # the bound gq_mmq_ex (set on first use)


def mmq(gtype: int, A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int,
        out: torch.Tensor | None = None, workspace: torch.Tensor | None = None, act: str = "q8_1") -> torch.Tensor:
    """C = (A @ B^T)^T as fp16 (N, M) on A's device; the common body of mmq_q8_0/q4_k/q6_k.
    act="fp8": the fp8 activation variant (gq_mmq_ex, GQ_ACT_FP8_E4M3) instead of q8_1.
    The common eager form (contiguous device A, fp16 (N, K) B with unit column stride on A's
    device, no out/workspace given) takes a short path: the same checks, fewer Python calls."""
    global _mmq_ex
    if (out is None and workspace is None and A.is_cuda and B.dtype is _F16 and B.dim() == 2 and
            (A.dtype is _I8 or A.dtype is _U8)):
        ns, ks = B.shape
        if ns == N and ks == K and B.stride(1) == 1 and A.is_contiguous() and \
                A.numel() == M * (K // BLOCK_ELEMS[gtype]) * BLOCK_BYTES[gtype]:
            idx = A.get_device()  # (an int: cheaper than building A.device)
            if B.get_device() != idx:
                raise RuntimeError(f"A on {A.device} but B on {B.device}")
            if M == 0 or N == 0:
                return _empty((N, M), dtype=_F16, device=A.device)
            key = (gtype, act, M, N, K)
            need = _call_ws.get(key)
            if need is None:
                need = _call_ws[key] = int(lib().gq_mmq_call_workspace_size(gtype, ACTS[act], M, N, K))
            if _mmq_ex is None:
                _mmq_ex = _bind_mmq_ex()
            if idx == _get_device():
                C = _empty((N, M), dtype=_F16, device=idx)
                if need:
                    ws = _empty(need, dtype=_U8, device=idx)
                    rc = _mmq_ex(gtype, ACTS[act], A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, B.stride(0), M,
                                 ws.data_ptr(), need, _raw_stream(idx))
                else:
                    rc = _mmq_ex(gtype, ACTS[act], A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, B.stride(0), M,
                                 None, 0, _raw_stream(idx))
                if rc:
                    _check(rc)
                return C
    _check_weights(gtype, A, M, K)
    _require_device(B, "B")
    dev = A.device
    if B.device != dev:
        raise RuntimeError(f"A on {dev} but B on {B.device}")
    B = _check_acts(B, N, K)
    C = _check_out(out, N, M, dev)
    if M == 0 or N == 0:
        return C
    key = (gtype, act, M, N, K)
    need = _call_ws.get(key)
    if need is None:
        need = _call_ws[key] = int(lib().gq_mmq_call_workspace_size(gtype, ACTS[act], M, N, K))
    if need and (workspace is None or workspace.numel() < need):
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    wp, wn = (workspace.data_ptr(), workspace.numel()) if need else (None, 0)
    if dev.index == torch.cuda.current_device():
        rc = lib().gq_mmq_ex(gtype, ACTS[act], A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, B.stride(0),
                             C.stride(0), wp, wn, _stream(dev))
    else:
        with torch.cuda.device(dev):
            rc = lib().gq_mmq_ex(gtype, ACTS[act], A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, B.stride(0),
                                 C.stride(0), wp, wn, _stream(dev))
    _check(rc)
    return C


def mmq_grouped(items, N: int, act: str = "q8_1"):
    """One grouped launch (gq_mmq_grouped_ex) for several MMQs with the same token count N:
    items = [(gtype, A, B, M, K, out or None), ...], every B an fp16 (N, K) tensor.  1..4 tokens
    (act="fp8": 1..2): the streaming decode kernel, bit-identical to mmq() per item; 5..32 (fp8:
    3..32): the K-chunked streaming MMQ (K <= 4096, M % 16 == 0), bit-identical to each item's
    call on that kernel.  Returns the (N, M) outputs, or None when the library reports the shapes
    unsupported (N > 32, or an item that is no shape of the launch) -- nothing was launched then
    and the caller runs mmq() per item."""
    if not items:
        return []
    dev = items[0][1].device
    arr = (GroupItem * len(items))()
    outs, keep = [], []
    for i, (gtype, A, B, M, K, out) in enumerate(items):
        _check_weights(gtype, A, M, K)
        if A.device != dev or B.device != dev:
            raise RuntimeError("grouped items must share one device")
        B = _check_acts(B, N, K)
        C = _check_out(out, N, M, dev)
        keep.append(B)
        outs.append(C)
        arr[i] = GroupItem(gtype, A.data_ptr(), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0), M, K)
    with torch.cuda.device(dev):
        rc = lib().gq_mmq_grouped_ex(ACTS[act], arr, len(items), N, torch.cuda.current_stream(dev).cuda_stream)
    if rc == GQ_EUNSUPPORTED:
        return None
    _check(rc)
    return outs


def mmq_grouped_prepared(items, N: int, act: str = "q8_1"):
    """One grouped streaming-GEMM launch (gq_mmq_grouped_prepared) for several prepared MMQs with
    the same token count N: items = [(gtype, A, ws, M, K, out or None), ...], ws the workspace the
    item's input was prepared into (act_prepare / act_prepare_grouped with this N, K, act).
    Returns the (N, M) outputs, or None when the library reports the shapes unsupported (N < 5,
    K % 256 != 0, > 16 items): nothing was launched then, call mmq_prepared per item."""
    if not items:
        return []
    dev = items[0][1].device
    arr = (GemmItem * len(items))()
    outs = []
    for i, (gtype, A, ws, M, K, out) in enumerate(items):
        _check_weights(gtype, A, M, K)
        if A.device != dev or ws.device != dev:
            raise RuntimeError("grouped items must share one device")
        C = _check_out(out, N, M, dev)
        outs.append(C)
        arr[i] = GemmItem(gtype, A.data_ptr(), ws.data_ptr(), C.data_ptr(), C.stride(0), M, K)
    need = int(lib().gq_mmq_grouped_prepared_workspace_size(ACTS[act], arr, len(items), N))
    part = torch.empty(need, dtype=torch.uint8, device=dev) if need else None
    with torch.cuda.device(dev):
        rc = lib().gq_mmq_grouped_prepared(ACTS[act], arr, len(items), N, part.data_ptr() if need else None, need,
                                           torch.cuda.current_stream(dev).cuda_stream)
    if rc == GQ_EUNSUPPORTED:
        return None
    _check(rc)
    return outs


def quantize_q8_1_device(X: torch.Tensor) -> torch.Tensor:
    """Device q8_1 quantizer (bit-exact with utils/quantize/q8_1.py) -> flat int8 bytes."""
    _require_device(X, "X")
    if X.dtype != torch.float16:
        X = X.to(torch.float16)
    X2 = X.reshape(-1, X.shape[-1]) if X.dim() > 1 else X.reshape(1, -1)
    if X2.stride(-1) != 1:
        X2 = X2.contiguous()
    rows, K = X2.shape
    if K % 32 != 0:
        raise ValueError("The total number of elements must be divisible by 32.")
    Y = torch.empty(rows * (K // 32) * 36, dtype=torch.int8, device=X.device)
    with torch.cuda.device(X.device):
        stream = torch.cuda.current_stream(X.device).cuda_stream
        _check(lib().gq_quantize_q8_1(X2.data_ptr(), Y.data_ptr(), rows, K, X2.stride(0), stream))
    return Y


def dequantize_device(gtype: int, A: torch.Tensor, M: int, K: int) -> torch.Tensor:
    """fp16 (M, K) weights from packed blocks on the device (gq_dequantize)."""
    _require_device(A, "A")
    qk, bb = BLOCK_ELEMS[gtype], BLOCK_BYTES[gtype]
    if A.numel() != M * (K // qk) * bb:
        raise RuntimeError(f"A has {A.numel()} bytes, expected {M * (K // qk) * bb}")
    W = torch.empty((M, K), dtype=torch.float16, device=A.device)
    with torch.cuda.device(A.device):
        stream = torch.cuda.current_stream(A.device).cuda_stream
        _check(lib().gq_dequantize(gtype, A.data_ptr(), W.data_ptr(), M, K, K, stream))
    return W


def act_prepare(B: torch.Tensor, N: int, K: int, workspace: torch.Tensor, act: str = "q8_1"):
    """Quantize the activations once into the front of `workspace` (gq_act_prepare_ex); any
    number of mmq_prepared calls with the same (N, K, act) then reuse them."""
    B = _check_acts(B, N, K)
    _check_workspace(workspace, 0, B.device)
    with torch.cuda.device(B.device):
        stream = torch.cuda.current_stream(B.device).cuda_stream
        _check(lib().gq_act_prepare_ex(ACTS[act], B.data_ptr(), N, K, B.stride(0), workspace.data_ptr(),
                                       workspace.numel(), stream))


def act_prepare_grouped(items, act: str = "q8_1"):
    """Several act_prepare calls in as few launches as possible (gq_act_prepare_grouped):
    items = [(B, N, K, workspace), ...] -- each workspace gets exactly what act_prepare would
    write; one launch per 8 items whose form is the GEMM paths' fp16 x~ (q8_1 at N >= 5; the fp8
    variant's widened codes at every N)."""
    if not items:
        return
    dev = items[0][0].device
    arr = (PrepItem * len(items))()
    keep = []
    for i, (B, N, K, ws) in enumerate(items):
        B = _check_acts(B, N, K)
        _check_workspace(ws, 0, B.device)
        if B.device != dev:
            raise RuntimeError("grouped items must share one device")
        keep.append(B)
        arr[i] = PrepItem(B.data_ptr(), N, K, B.stride(0), ws.data_ptr(), ws.numel())
    with torch.cuda.device(dev):
        _check(lib().gq_act_prepare_grouped(ACTS[act], arr, len(items), torch.cuda.current_stream(dev).cuda_stream))


def mmq_prepared(gtype: int, A: torch.Tensor, workspace: torch.Tensor, M: int, N: int, K: int,
                 out: torch.Tensor | None = None, act: str = "q8_1") -> torch.Tensor:
    """C (N, M) fp16 from packed A and the activations act_prepare left in `workspace`."""
    _check_weights(gtype, A, M, K)
    _check_workspace(workspace, workspace_size(gtype, M, N, K, act), A.device)
    C = _check_out(out, N, M, A.device)
    if M == 0 or N == 0:
        return C
    with torch.cuda.device(A.device):
        stream = torch.cuda.current_stream(A.device).cuda_stream
        _check(lib().gq_mmq_prepared_ex(gtype, ACTS[act], A.data_ptr(), workspace.data_ptr(), workspace.numel(),
                                        C.data_ptr(), M, N, K, C.stride(0), stream))
    return C


def quantize_weights_device(fmt: str, X: torch.Tensor) -> torch.Tensor:
    """GGUF weight quantization on the device (gq_quantize_weights): the bytes of
    utils.quantize.quantize_to_<fmt> (int8, flat), from an fp16 (q8_0) or fp32 (q4_k, q6_k)
    device tensor read as flat blocks."""
    want = torch.float16 if fmt == "q8_0" else torch.float32
    if not X.is_cuda or X.dtype != want:
        raise RuntimeError(f"quantize_weights_device({fmt}) needs a {want} device tensor")
    X = X.contiguous().reshape(-1)
    qk, nbytes = (32, 34) if fmt == "q8_0" else (256, 144 if fmt == "q4_k" else 210)
    if X.numel() % qk:
        raise RuntimeError(f"{X.numel()} elements are not whole {fmt} blocks")
    out = torch.empty(X.numel() // qk * nbytes, dtype=torch.int8, device=X.device)
    with torch.cuda.device(X.device):
        _check(lib().gq_quantize_weights(TYPES[fmt], X.data_ptr(), out.data_ptr(), X.numel(),
                                         torch.cuda.current_stream(X.device).cuda_stream))
    return out


def quantize_fp8_device(X: torch.Tensor):
    """The fp8 variant's activation quantizer (gq_quantize_fp8) -> (codes uint8 (rows, K) in the
    (0,2,1,3) group order, scales float32 (K/32, (rows+3)&~3))."""
    _require_device(X, "X")
    X2 = X.to(torch.float16).reshape(-1, X.shape[-1]).contiguous()
    rows, K = X2.shape
    codes = torch.empty((rows, K), dtype=torch.uint8, device=X.device)
    scales = torch.empty((K // 32, (rows + 3) & ~3), dtype=torch.float32, device=X.device)
    with torch.cuda.device(X.device):
        stream = torch.cuda.current_stream(X.device).cuda_stream
        _check(lib().gq_quantize_fp8(X2.data_ptr(), codes.data_ptr(), scales.data_ptr(), rows, K, X2.stride(0),
                                     stream))
    return codes, scales


def shard_rows(M: int, world: int, rank: int):
    """(row0, rows, R) of rank `rank` (gq_shard_rows; the rule of dist/row_shard.shard_rows)."""
    r0, rows, R = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _check(lib().gq_shard_rows(M, world, rank, ctypes.byref(r0), ctypes.byref(rows), ctypes.byref(R)))
    return r0.value, rows.value, R.value


def assemble_shards(gathered: torch.Tensor, M: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """(world, N, R) fp16 slabs -> (N, M) on the device (gq_assemble_shards)."""
    _require_device(gathered, "gathered")
    if gathered.dtype != torch.float16 or gathered.dim() != 3 or not gathered.is_contiguous():
        raise RuntimeError("gathered must be a contiguous (world, N, R) fp16 tensor")
    W, N, R = gathered.shape
    C = _check_out(out, N, M, gathered.device)
    with torch.cuda.device(gathered.device):
        stream = torch.cuda.current_stream(gathered.device).cuda_stream
        _check(lib().gq_assemble_shards(gathered.data_ptr(), C.data_ptr(), W, N, R, M, C.stride(0), stream))
    return C


def mmq_sharded_single(gtype: int, A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int) -> torch.Tensor:
    """gq_mmq_sharded at world 1 (no communicator): the C-ABI sharded entry point end to end on
    one device (multi-rank callers pass their own RCCL communicator through the C ABI)."""
    _require_device(A, "A")
    _check_weights(gtype, A, M, K)
    B = _check_acts(B, N, K)
    C = _check_out(None, N, M, A.device)
    need = int(lib().gq_mmq_sharded_workspace_size(gtype, M, N, K, 1))
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=A.device)
    with torch.cuda.device(A.device):
        stream = torch.cuda.current_stream(A.device).cuda_stream
        _check(lib().gq_mmq_sharded(gtype, A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, B.stride(0), C.stride(0),
                                    1, 0, None, ws.data_ptr(), ws.numel(), stream))
    return C

