"""ctypes binding of ``libggnn.so`` (the C ABI declared in ``include/ggnn.h``).

The product path has exactly one implementation: the HIP kernels behind this
library.  If the library is missing or fails to load, every entry point
raises -- there is no CPU or PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

from .build import LIB

GGNN_USE_EDGE_BIAS = 1
GGNN_FP32_PARITY = 2
GGNN_FP16 = 4
GGNN_DENSE_CHANNELS = 8
GGNN_GENERIC = 16
GGNN_UNFUSED_FWD = 32
GGNN_SPARSE_PAIRS = 64
GGNN_SEED_DEVICE = 128
PRECISIONS = ("bf16", "fp16", "fp32")

# Every symbol include/ggnn.h declares (checked by tests/test_lib.py).
EXPORTED = (
    "ggnn_version", "ggnn_last_error", "ggnn_check_dims", "ggnn_workspace_bytes",
    "ggnn_adjacency_bytes", "ggnn_weight_pack_bytes", "ggnn_pack_weights", "ggnn_pack_weights_batch", "ggnn_set_adjacency",
    "ggnn_set_adjacency_edges",
    "ggnn_forward", "ggnn_backward", "ggnn_adam_step", "ggnn_dropout_mask", "ggnn_kernel_kind_name", "ggnn_profile_begin",
    "ggnn_profile_end", "ggnn_embed_forward", "ggnn_embed_backward", "ggnn_embed_workspace_bytes",
    "ggnn_embed_backward_ws", "ggnn_embed_lookup_rows", "ggnn_heads_workspace_bytes",
    "ggnn_heads_forward", "ggnn_heads_backward", "ggnn_dbg_gemm", "ggnn_dbg_gemm_ex",
    "ggnn_adam_step_dev", "ggnn_heads_forward_dev", "ggnn_heads_backward_dev",
)
NUM_KERNEL_KINDS = 11


class GGNNDims(ctypes.Structure):
    _fields_ = [("b", ctypes.c_int32), ("v", ctypes.c_int32), ("h", ctypes.c_int32),
                ("C", ctypes.c_int32), ("T", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("edge_keep", ctypes.c_float), ("state_keep", ctypes.c_float), ("seed", ctypes.c_uint64)]

    def __repr__(self):
        return "GGNNDims(b=%d, v=%d, h=%d, C=%d, T=%d, flags=%d, edge_keep=%g, state_keep=%g, seed=%d)" % (
            self.b, self.v, self.h, self.C, self.T, self.flags, self.edge_keep, self.state_keep, self.seed)


class GGNNError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I = ctypes.c_int
_DP = ctypes.POINTER(GGNNDims)


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libggnn.so (once).  Raises GGNNError if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = path or os.environ.get("GGNN_LIB", LIB)
        if not os.path.exists(path):
            raise GGNNError("libggnn.so not found at %s: run `python -m ggnn_amd.build` "
                            "(or __graft_entry__.build()) first" % path)
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        lib.ggnn_version.restype = _I
        lib.ggnn_version.argtypes = []
        lib.ggnn_last_error.restype = ctypes.c_char_p
        lib.ggnn_last_error.argtypes = []
        lib.ggnn_check_dims.restype = _I
        lib.ggnn_check_dims.argtypes = [_DP]
        lib.ggnn_workspace_bytes.restype = _I
        lib.ggnn_workspace_bytes.argtypes = [_DP, _I, ctypes.POINTER(ctypes.c_size_t)]
        lib.ggnn_adjacency_bytes.restype = _I
        lib.ggnn_adjacency_bytes.argtypes = [_DP, ctypes.POINTER(ctypes.c_size_t)]
        lib.ggnn_weight_pack_bytes.restype = _I
        lib.ggnn_weight_pack_bytes.argtypes = [_DP, ctypes.POINTER(ctypes.c_size_t)]
        lib.ggnn_pack_weights.restype = _I
        lib.ggnn_pack_weights.argtypes = [_DP, _P, _P, _P, _P, _P, _P, _P, _P]
        if hasattr(lib, "ggnn_pack_weights_batch"):   # (absent from builds before round 4: A/B runs)
            lib.ggnn_pack_weights_batch.restype = _I
            lib.ggnn_pack_weights_batch.argtypes = [_DP, _P, _P, _P, _P, _P, _P, _P, _P, _P]
        lib.ggnn_set_adjacency.restype = _I
        lib.ggnn_set_adjacency.argtypes = [_DP, _P, _P, _P]
        lib.ggnn_set_adjacency_edges.restype = _I
        lib.ggnn_set_adjacency_edges.argtypes = [_DP, _P, _P, _P, ctypes.c_int64, _I, _P]
        lib.ggnn_forward.restype = _I
        lib.ggnn_forward.argtypes = [_DP, _P, _P, _P, _I, _P, _P, _P]
        lib.ggnn_backward.restype = _I
        lib.ggnn_backward.argtypes = [_DP, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]
        lib.ggnn_adam_step.restype = _I
        lib.ggnn_adam_step.argtypes = [_P, _I, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                       ctypes.c_float, ctypes.c_int64, ctypes.c_float, _P, _P]
        lib.ggnn_adam_step_dev.restype = _I
        lib.ggnn_adam_step_dev.argtypes = [_P, _I, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, _P, ctypes.c_float, _P, _P]
        lib.ggnn_dropout_mask.restype = _I
        lib.ggnn_dropout_mask.argtypes = [_DP, _I, _I, _P, _P]
        U64, F = ctypes.c_uint64, ctypes.c_float
        lib.ggnn_embed_forward.restype = _I
        lib.ggnn_embed_forward.argtypes = [_DP, _P, _I, _P, _I, F, U64, _P, _P]
        lib.ggnn_embed_backward.restype = _I
        lib.ggnn_embed_backward.argtypes = [_DP, _P, _I, _P, _I, F, U64, _P, _P, _P, _P]
        if hasattr(lib, "ggnn_embed_backward_ws"):   # (absent from builds before round 5: A/B runs)
            lib.ggnn_embed_workspace_bytes.restype = _I
            lib.ggnn_embed_workspace_bytes.argtypes = [_P, _I, ctypes.POINTER(ctypes.c_size_t)]
            lib.ggnn_embed_backward_ws.restype = _I
            lib.ggnn_embed_backward_ws.argtypes = [_DP, _P, _I, _P, _I, F, U64, _P, _P, _P, _P, _P]
            lib.ggnn_embed_lookup_rows.restype = _I
            lib.ggnn_embed_lookup_rows.argtypes = [_DP, _P, _I, _I, _P, _I, F, U64, _P, _P, _P, _P,
                                                   ctypes.c_int64, _P]
        lib.ggnn_heads_workspace_bytes.restype = _I
        lib.ggnn_heads_workspace_bytes.argtypes = [_DP, _P, _I, ctypes.POINTER(ctypes.c_size_t)]
        lib.ggnn_heads_forward.restype = _I
        lib.ggnn_heads_forward.argtypes = [_DP, _P, _I, _P, _P, F, U64, F, _P, _P, _P]
        lib.ggnn_heads_backward.restype = _I
        lib.ggnn_heads_backward.argtypes = [_DP, _P, _I, _P, _P, F, _P, _P, _P, _P, _P]
        lib.ggnn_heads_forward_dev.restype = _I
        lib.ggnn_heads_forward_dev.argtypes = [_DP, _P, _I, _P, _P, F, U64, _P, _P, _P, _P]
        lib.ggnn_heads_backward_dev.restype = _I
        lib.ggnn_heads_backward_dev.argtypes = [_DP, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P]
        lib.ggnn_dbg_gemm.restype = _I
        lib.ggnn_dbg_gemm.argtypes = [_DP, _I, _I, _I, _P, _P, _P, _P]
        lib.ggnn_dbg_gemm_ex.restype = _I
        lib.ggnn_dbg_gemm_ex.argtypes = [_DP, _I, _I, _I, _P, _I, _P, _I, _P, _I, _P]
        lib.ggnn_kernel_kind_name.restype = ctypes.c_char_p
        lib.ggnn_kernel_kind_name.argtypes = [_I]
        lib.ggnn_profile_begin.restype = _I
        lib.ggnn_profile_begin.argtypes = [_I]
        lib.ggnn_profile_end.restype = _I
        lib.ggnn_profile_end.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().ggnn_last_error().decode(errors="replace")
        raise GGNNError("%s failed (%d): %s" % (what, rc, msg))


def dims(b: int, v: int, h: int, C: int, T: int, use_edge_bias: bool = True, precision: str = "fp32",
         edge_keep: float = 1.0, state_keep: float = 1.0, seed: int = 0,
         skip_empty_channels: bool = True, force_generic: bool = False,
         unfused_forward: bool = False, sparse_pairs: bool = False, seed_device: bool = False) -> GGNNDims:
    """seed_device: ``seed`` is the address of a device uint64 the kernels read
    (GGNN_SEED_DEVICE, for hipGraph capture)."""
    if precision not in PRECISIONS:
        raise ValueError("precision must be one of %s" % (PRECISIONS,))
    flags = (GGNN_USE_EDGE_BIAS if use_edge_bias else 0) | {"bf16": 0, "fp16": GGNN_FP16, "fp32": GGNN_FP32_PARITY}[precision]
    if not skip_empty_channels:
        flags |= GGNN_DENSE_CHANNELS
    if force_generic:
        flags |= GGNN_GENERIC
    if unfused_forward:
        flags |= GGNN_UNFUSED_FWD
    if sparse_pairs:
        flags |= GGNN_SPARSE_PAIRS
    if seed_device:
        flags |= GGNN_SEED_DEVICE
    return GGNNDims(int(b), int(v), int(h), int(C), int(T), flags, float(edge_keep), float(state_keep),
                    int(seed) & 0xFFFFFFFFFFFFFFFF)


def check_dims(d: GGNNDims) -> None:
    check(load().ggnn_check_dims(ctypes.byref(d)), "ggnn_check_dims(%r)" % (d,))


def workspace_bytes(d: GGNNDims, training: bool) -> int:
    n = ctypes.c_size_t(0)
    check(load().ggnn_workspace_bytes(ctypes.byref(d), int(bool(training)), ctypes.byref(n)),
          "ggnn_workspace_bytes")
    return int(n.value)


def adjacency_bytes(d: GGNNDims) -> int:
    n = ctypes.c_size_t(0)
    check(load().ggnn_adjacency_bytes(ctypes.byref(d), ctypes.byref(n)), "ggnn_adjacency_bytes")
    return int(n.value)


def weight_pack_bytes(d: GGNNDims) -> int:
    n = ctypes.c_size_t(0)
    check(load().ggnn_weight_pack_bytes(ctypes.byref(d), ctypes.byref(n)), "ggnn_weight_pack_bytes")
    return int(n.value)


class KernelTimer:
    """Context manager: HIP-event time of every libggnn launch, per kernel kind."""

    def __init__(self, max_launches: int = 100000):
        self.max_launches = max_launches
        self.total_ms = {}
        self.launches = {}

    def __enter__(self):
        check(load().ggnn_profile_begin(self.max_launches), "ggnn_profile_begin")
        return self

    def __exit__(self, *exc):
        ms = (ctypes.c_double * NUM_KERNEL_KINDS)()
        n = (ctypes.c_int * NUM_KERNEL_KINDS)()
        check(load().ggnn_profile_end(ms, n), "ggnn_profile_end")
        for k in range(NUM_KERNEL_KINDS):
            name = load().ggnn_kernel_kind_name(k).decode()
            self.total_ms[name] = ms[k]
            self.launches[name] = n[k]
        return False
