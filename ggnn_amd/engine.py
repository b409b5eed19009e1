"""Host-side driver of the HIP propagation engine.

``PropagationEngine`` owns the device buffers of one batch shape and calls
the C ABI (``include/ggnn.h``) on PyTorch's current HIP stream.  PyTorch is
used only to hold device memory and to name the stream; every arithmetic op
of the hot path runs in ``libggnn.so``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from .upload import Uploader

WEIGHT_NAMES = ("edge_weights", "edge_biases", "gates_kernel", "gates_bias",
                "candidate_kernel", "candidate_bias")


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _require(t: torch.Tensor, shape, name: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor on the GPU, got %r" % (name, type(t)))
    if t.device.type != "cuda":
        raise ValueError("%s must live on a HIP device (got %s)" % (name, t.device))
    if t.dtype != torch.float32:
        raise TypeError("%s must be float32 (got %s)" % (name, t.dtype))
    if tuple(t.shape) != tuple(shape):
        raise ValueError("%s: expected shape %s, got %s" % (name, tuple(shape), tuple(t.shape)))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % name)


@dataclass
class WeightPack:
    """MFMA-fragment copy of one weight set (see ggnn_pack_weights).  Under
    edge-weight dropout (edge_keep < 1) it holds one masked copy per timestep
    of a T-step pass keyed by `seed`."""
    buf: torch.Tensor
    hidden: int
    channels: int
    use_edge_bias: bool
    T: int = 1
    edge_keep: float = 1.0
    seed: int = 0
    seed_device: bool = False   # seed is the address of a device uint64 (GGNN_SEED_DEVICE)
    batch_gen: int | None = None  # made for the staged batch of this generation (pack_weights(batch=True))


class PropagationEngine:
    """Runs ``compute_final_node_representations`` (chem_tensorflow_dense.py:312-340)
    and its backward for batches of shape [b, C, v, v] / [b, v, h]."""

    def __init__(self, hidden: int, channels: int, use_edge_bias: bool = True, device=None,
                 precision: str = "fp32", skip_empty_channels: bool = True, force_generic: bool = False,
                 unfused_forward: bool = False, sparse_pairs="auto"):
        """precision: "fp32" (GGNN_FP32_PARITY, the default: every non-exact MFMA
        operand of the propagation as an f16 hi/lo limb pair, fp32 accumulation,
        matches the reference's fp32 math to <= 1e-3), "fp16" or "bf16" (single
        16-bit MFMA operands, fp32 accumulation; reduced precision, opt-in).
        skip_empty_channels: run the message passing only over each graph's
        non-empty adjacency channels (bit-identical; False = GGNN_DENSE_CHANNELS).
        force_generic: run the general path (k_gemm products) even where the
        specialised kernels apply (hidden 128 / 256, v <= 128); other shapes
        always take it (GGNN_GENERIC).  unfused_forward: per-timestep
        k_prop_fwd + k_gru_fwd launches instead of the one-launch fused forward
        at hidden 256, v <= 128 (GGNN_UNFUSED_FWD; A/B and tests).
        sparse_pairs: the general path's sparse message passing
        (GGNN_SPARSE_PAIRS: the message transform over the (node, channel)
        pairs with an incoming edge instead of every row of every non-empty
        tile) for batches staged from edge lists: "auto" = whenever such a
        batch runs the general path anyway (hidden not 128 / 256, v > 128 or
        force_generic) and qualifies (hidden % 4 == 0, edges <= b*v); True =
        for every qualifying edge-list batch (also hidden 128 / 256: pair mode
        implies the general path); False = never."""
        self.h = int(hidden)
        self.C = int(channels)
        self.use_edge_bias = bool(use_edge_bias)
        self._up_edges, self._up_offs = Uploader(), Uploader()
        if precision not in _lib.PRECISIONS:
            raise ValueError("precision must be one of %s" % (_lib.PRECISIONS,))
        self.precision = precision
        self.skip_empty_channels = bool(skip_empty_channels)
        self.force_generic = bool(force_generic)
        self.unfused_forward = bool(unfused_forward)
        if sparse_pairs not in ("auto", True, False):
            raise ValueError("sparse_pairs must be 'auto', True or False")
        self.sparse_pairs = sparse_pairs
        self._sparse = False        # the staged batch runs pair mode
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._lib = _lib.load()
        self._adj = None            # staged adjacency buffer
        self._batch = None          # (b, v) of the staged adjacency
        self._ws = {}               # (b, v, T, training) -> workspace
        self._trained = None        # (b, v, T, pack, ws) of the last training forward
        self._adj_gen = 0           # bumped by every staging (set_adjacency*)
        self.generation = 0         # bumped by every forward (autograd staleness check)

    # ------------------------------------------------------------------ utils
    def dims(self, b: int, v: int, T: int, edge_keep: float = 1.0, state_keep: float = 1.0,
             seed: int = 0, seed_device: bool = False) -> _lib.GGNNDims:
        d = _lib.dims(b, v, self.h, self.C, T, self.use_edge_bias, self.precision, edge_keep, state_keep, seed,
                      self.skip_empty_channels, self.force_generic, self.unfused_forward, self._sparse,
                      seed_device)
        _lib.check_dims(d)
        return d

    def workspace(self, b: int, v: int, T: int, training: bool, edge_dropout: bool = False) -> torch.Tensor:
        key = (b, v, T, bool(training), bool(edge_dropout), self._sparse)
        ws = self._ws.get(key)
        if ws is None:
            if len(self._ws) >= 4:      # keep a handful of shapes (bucketed batches)
                self._ws.clear()
            d = self.dims(b, v, T, edge_keep=0.5 if edge_dropout else 1.0)
            ws = torch.empty(_lib.workspace_bytes(d, training), dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    # ---------------------------------------------------------------- weights
    def pack_weights(self, weights: dict, T: int = 1, edge_keep: float = 1.0, seed: int = 0,
                     seed_device: bool = False, batch: bool = False, out: torch.Tensor | None = None) -> WeightPack:
        """weights: dict of fp32 device tensors with the reference's shapes:
        edge_weights [C,h,h], edge_biases [C,1,h] (or [C,h]), gates_kernel [2h,2h],
        gates_bias [2h], candidate_kernel [2h,h], candidate_bias [h].
        edge_keep < 1: edge-weight dropout (chem_tensorflow_dense.py:397-403),
        one fresh mask per timestep of a T-step pass, keyed by seed.
        seed_device: seed is the address of a device uint64 holding the seed
        (read when the kernels run: hipGraph capture, ggnn_amd/graphs.py).
        batch: pack for the batch staged now (ggnn_pack_weights_batch): under
        edge dropout on the general path only the channels the batch uses get
        their masked copies; the pack then serves that staged batch only.
        out: a caller-owned uint8 device buffer of at least
        ggnn_weight_pack_bytes to pack into (else one is allocated)."""
        h, C = self.h, self.C
        _require(weights["edge_weights"], (C, h, h), "edge_weights")
        eb = weights.get("edge_biases") if self.use_edge_bias else None
        if self.use_edge_bias:
            if eb is None:
                raise ValueError("use_edge_bias=True but no edge_biases given")
            _require(eb, (C, 1, h) if eb.dim() == 3 else (C, h), "edge_biases")
        _require(weights["gates_kernel"], (2 * h, 2 * h), "gates_kernel")
        _require(weights["gates_bias"], (2 * h,), "gates_bias")
        _require(weights["candidate_kernel"], (2 * h, h), "candidate_kernel")
        _require(weights["candidate_bias"], (h,), "candidate_bias")
        T = int(T) if edge_keep < 1.0 else 1
        # (a library built before round 4 has no ggnn_pack_weights_batch: the
        # whole-set pack is still correct there, only slower)
        for_batch = (bool(batch) and self._batch is not None and edge_keep < 1.0
                     and hasattr(self._lib, "ggnn_pack_weights_batch"))
        b, v = self._batch if for_batch else (1, 1)
        d = self.dims(b, v, T, edge_keep=edge_keep, seed=seed, seed_device=seed_device)
        nbytes = _lib.weight_pack_bytes(d)
        if out is None:
            buf = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        else:
            if out.dtype != torch.uint8 or out.device.type != "cuda" or out.numel() < nbytes or not out.is_contiguous():
                raise ValueError("out must be a contiguous uint8 device buffer of >= %d bytes" % nbytes)
            buf = out
        wp = (_ptr(weights["edge_weights"]), _ptr(eb), _ptr(weights["gates_kernel"]), _ptr(weights["gates_bias"]),
              _ptr(weights["candidate_kernel"]), _ptr(weights["candidate_bias"]), _stream())
        if for_batch:
            _lib.check(self._lib.ggnn_pack_weights_batch(ctypes.byref(d), _ptr(buf), _ptr(self._adj), *wp),
                       "ggnn_pack_weights_batch")
        else:
            _lib.check(self._lib.ggnn_pack_weights(ctypes.byref(d), _ptr(buf), *wp), "ggnn_pack_weights")
        return WeightPack(buf, h, C, self.use_edge_bias, T, float(edge_keep), int(seed), bool(seed_device),
                          self._adj_gen if for_batch else None)

    # -------------------------------------------------------------- adjacency
    def set_adjacency(self, adjacency: torch.Tensor) -> None:
        """adjacency: [b, C, v, v] fp32 0/1 on the device (the reference's feed,
        chem_tensorflow_dense.py:192-195)."""
        if adjacency.dim() != 4 or adjacency.shape[1] != self.C or adjacency.shape[2] != adjacency.shape[3]:
            raise ValueError("adjacency must be [b, %d, v, v], got %s" % (self.C, tuple(adjacency.shape)))
        b, _, v, _ = adjacency.shape
        _require(adjacency, (b, self.C, v, v), "adjacency")
        self._sparse = False          # (pair mode is staged from edge lists only)
        d = self.dims(b, v, 1)
        nbytes = _lib.adjacency_bytes(d)
        if self._adj is None or self._adj.numel() < nbytes:
            self._adj = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        _lib.check(self._lib.ggnn_set_adjacency(ctypes.byref(d), _ptr(self._adj), _ptr(adjacency), _stream()),
                   "ggnn_set_adjacency")
        self._batch = (int(b), int(v))
        self._trained = None
        self._adj_gen += 1

    def set_adjacency_edges(self, graphs, v: int, num_edge_types: int) -> None:
        """Stage a batch from the reference's edge lists (each graph a list of
        (src, label, dest) triples, chem_tensorflow_dense.py:65-83) without
        building the dense [b, 2E, v, v] feed: only the edge rows (12 B each)
        cross PCIe.  ``graphs`` is a list of per-graph edge lists, or a tuple
        (edges int32 [n, 3], graph_offsets int32 [b + 1]) already on the
        device.  Raises IndexError for edges the reference would index out of
        range."""
        import numpy as np
        E = int(num_edge_types)
        if 2 * E != self.C:
            raise ValueError("num_edge_types=%d does not match C=%d channels" % (E, self.C))
        if isinstance(graphs, tuple):
            edges, offs = graphs
            b = int(offs.numel()) - 1
            n = int(edges.shape[0])
        else:
            b = len(graphs)
            sizes = [len(g) for g in graphs]
            offs_np = np.zeros(b + 1, np.int32)
            offs_np[1:] = np.cumsum(sizes)
            n = int(offs_np[-1])
            e_np = (np.concatenate([np.asarray(g, np.int32).reshape(-1, 3) for g in graphs if len(g)])
                    if n else np.zeros((0, 3), np.int32))
            if n:
                src, lab, dst = e_np[:, 0], e_np[:, 1], e_np[:, 2]
                if lab.min() < 1 or lab.max() > E:
                    raise IndexError("edge label outside 1..%d" % E)
                if min(src.min(), dst.min()) < 0 or max(src.max(), dst.max()) >= v:
                    raise IndexError("edge node index outside 0..%d" % (v - 1))
            edges = self._up_edges(e_np, self.device)
            offs = self._up_offs(offs_np, self.device)
        self._sparse = self._use_pairs(b, v, n)
        d = self.dims(b, v, 1)
        nbytes = _lib.adjacency_bytes(d)
        if self._adj is None or self._adj.numel() < nbytes:
            self._adj = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        _lib.check(self._lib.ggnn_set_adjacency_edges(ctypes.byref(d), _ptr(self._adj), _ptr(edges), _ptr(offs),
                                                      n, E, _stream()), "ggnn_set_adjacency_edges")
        self._batch = (int(b), int(v))
        self._trained = None
        self._adj_gen += 1

    def _use_pairs(self, b: int, v: int, n_edges: int) -> bool:
        """Pair mode for this edge-list batch (see __init__'s sparse_pairs)."""
        if self.sparse_pairs is False or self.h % 4 or n_edges > b * v:
            return False
        if self.sparse_pairs is True:
            return True
        return self.force_generic or self.h not in (128, 256) or v > 128

    @property
    def sparse(self) -> bool:
        """Whether the staged batch runs the general path's pair mode."""
        return self._sparse

    @property
    def batch_shape(self):
        return self._batch

    # ---------------------------------------------------------------- compute
    def forward(self, h0: torch.Tensor, pack: WeightPack, T: int, training: bool = False,
                out: torch.Tensor | None = None, state_keep: float = 1.0) -> torch.Tensor:
        """state_keep < 1: GRU state dropout (DropoutWrapper, chem_tensorflow_dense.py:239-240),
        keyed by the pack's seed; edge-weight dropout comes with the pack."""
        if self._batch is None:
            raise RuntimeError("set_adjacency() must be called before forward()")
        if not isinstance(pack, WeightPack):
            raise RuntimeError("forward() needs a WeightPack from pack_weights()")
        b, v = self._batch
        _require(h0, (b, v, self.h), "initial_node_representations")
        if pack.edge_keep < 1.0 and pack.T != T:
            raise ValueError("the pack holds edge-dropout masks for T=%d, forward asked for T=%d" % (pack.T, T))
        if pack.batch_gen is not None and pack.batch_gen != self._adj_gen:
            raise RuntimeError("this pack was made for another staged batch (pack_weights(batch=True)): "
                               "pack again after staging the batch")
        ws = self.workspace(b, v, T, training, pack.edge_keep < 1.0)
        d = self.dims(b, v, T, pack.edge_keep, state_keep, pack.seed, pack.seed_device)
        if out is None:
            out = torch.empty((b, v, self.h), dtype=torch.float32, device=self.device)
        _require(out, (b, v, self.h), "out")
        _lib.check(self._lib.ggnn_forward(ctypes.byref(d), _ptr(pack.buf), _ptr(self._adj), _ptr(ws),
                                          int(bool(training)), _ptr(h0), _ptr(out), _stream()), "ggnn_forward")
        self._trained = (b, v, T, pack, ws, float(state_keep)) if training else None
        self.generation += 1
        return out

    def alloc_grads(self, b: int, v: int) -> dict:
        h, C, dev = self.h, self.C, self.device
        return {
            "h0": torch.empty((b, v, h), dtype=torch.float32, device=dev),
            "edge_weights": torch.empty((C, h, h), dtype=torch.float32, device=dev),
            "edge_biases": torch.empty((C, 1, h), dtype=torch.float32, device=dev) if self.use_edge_bias else None,
            "gates_kernel": torch.empty((2 * h, 2 * h), dtype=torch.float32, device=dev),
            "gates_bias": torch.empty((2 * h,), dtype=torch.float32, device=dev),
            "candidate_kernel": torch.empty((2 * h, h), dtype=torch.float32, device=dev),
            "candidate_bias": torch.empty((h,), dtype=torch.float32, device=dev),
        }

    def backward(self, dhT: torch.Tensor, grads: dict | None = None) -> dict:
        """Backward of the last training forward.  Returns a dict with 'h0' and
        the six weight gradients (reference shapes, fp32)."""
        if self._trained is None:
            raise RuntimeError("backward() needs a preceding forward(..., training=True) on this batch")
        b, v, T, pack, ws, state_keep = self._trained
        _require(dhT, (b, v, self.h), "dL/dh_T")
        if grads is None:
            grads = self.alloc_grads(b, v)
        d = self.dims(b, v, T, pack.edge_keep, state_keep, pack.seed, pack.seed_device)
        _lib.check(self._lib.ggnn_backward(
            ctypes.byref(d), _ptr(pack.buf), _ptr(self._adj), _ptr(ws), _ptr(dhT), _ptr(grads["h0"]),
            _ptr(grads["edge_weights"]), _ptr(grads.get("edge_biases")), _ptr(grads["gates_kernel"]),
            _ptr(grads["gates_bias"]), _ptr(grads["candidate_kernel"]), _ptr(grads["candidate_bias"]),
            _stream()), "ggnn_backward")
        return grads

    def dropout_mask(self, kind: str, b: int, v: int, T: int, t: int, keep: float, seed: int) -> torch.Tensor:
        """The keep-mask (uint8, 1 = kept) the kernels apply: kind "edge" ->
        [C, h, h] of timestep t; kind "state" -> [b, v, h] of timestep t."""
        k = {"edge": 0, "state": 1}[kind]
        d = self.dims(b, v, T, keep if k == 0 else 1.0, keep if k == 1 else 1.0, seed)
        shape = (self.C, self.h, self.h) if k == 0 else (b, v, self.h)
        m = torch.empty(shape, dtype=torch.uint8, device=self.device)
        _lib.check(self._lib.ggnn_dropout_mask(ctypes.byref(d), k, int(t), _ptr(m), _stream()), "ggnn_dropout_mask")
        return m
