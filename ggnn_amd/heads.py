"""The callers either side of the propagation path, btb task.

* ``EmbeddingFrontEnd`` -- ``get_initial_node_representation``
  (chem_tensorflow_dense.py:264-306): embedding lookups of the ``word_inputs``
  columns, embedding dropout, concat, zero pad to ``hidden_size``.
* ``OutputHeads`` -- ``gated_regression`` for ``--pr btb``
  (chem_tensorflow_dense.py:439-516) with ``MLP(2h, o, [], keep)``
  (utils.py:40-84) and the btb cross-entropy (chem_tensorflow.py:349-403).

Both run in libggnn.so (``ggnn_embed_*``, ``ggnn_heads_*``; kernels in
``csrc/k_head.h``); torch tensors only hold device memory.  The autograd
Functions ``EmbedFunction`` / ``HeadsFunction`` let the drop-in model train with
``loss.backward()``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .upload import Uploader

from . import _lib

SMALL_NUMBER = 1e-7   # utils.py


class EmbedSegment(ctypes.Structure):          # include/ggnn.h: ggnn_embed_segment
    _fields_ = [("table", ctypes.c_void_p), ("d_table", ctypes.c_void_p), ("rows", ctypes.c_int64),
                ("width", ctypes.c_int32), ("column", ctypes.c_int32)]


class OutputHead(ctypes.Structure):            # include/ggnn.h: ggnn_output_head
    _fields_ = [("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("o", ctypes.c_int32),
                ("labels", ctypes.c_void_p), ("probs", ctypes.c_void_p), ("d_weight", ctypes.c_void_p),
                ("d_bias", ctypes.c_void_p)]


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _f32(t, device):
    if not isinstance(t, torch.Tensor):
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(t, dtype=np.float32)))
    return t.to(device=device, dtype=torch.float32).contiguous()


_WI_UPLOAD = Uploader()


def word_inputs_tensor(word_inputs, device, table_rows=None) -> torch.Tensor:
    """The feed's ``word_inputs`` [b, v, ncols] (float64 in the reference's feed)
    as int32 on the device.  ``table_rows``: {column: rows} to validate (the
    reference's CPU ``embedding_lookup`` raises for an index out of range)."""
    wi = np.asarray(word_inputs)
    wi_i = wi.astype(np.int64)
    if table_rows:
        for col, rows in table_rows.items():
            c = wi_i[..., col]
            if c.size and (c.min() < 0 or c.max() >= rows):
                raise IndexError("word_inputs[..., %d] holds index %d outside [0, %d)"
                                 % (col, int(c.max() if c.max() >= rows else c.min()), rows))
    return _WI_UPLOAD(wi_i.astype(np.int32), device)


class EmbeddingFrontEnd:
    """segments: list of (table tensor [rows, width], word_inputs column), in
    concat order.  btb: [(loc_embeddings, 0), (pos_embeddings, 1),
    (word_embeddings, 2), (loc_embeddings, 3)] (:268-299)."""

    def __init__(self, hidden: int, deterministic: bool = True):
        """deterministic: the table gradients through ggnn_embed_backward_ws
        (fixed-point accumulation: the same bits run to run); False: the fp32
        atomics of ggnn_embed_backward."""
        self.hidden = int(hidden)
        self._lib = _lib.load()
        self.deterministic = bool(deterministic) and hasattr(self._lib, "ggnn_embed_backward_ws")
        self._ws = {}    # table set -> zero-filled workspace (each call leaves it zero-filled)

    def workspace(self, segments, device):
        """The deterministic backward's workspace for this table set: allocated
        (zero-filled) once and kept, so a captured step's pointer stays valid."""
        key = tuple((t.data_ptr(), tuple(t.shape)) for t, _ in segments)
        ws = self._ws.get(key)
        if ws is None:
            n = ctypes.c_size_t(0)
            _lib.check(self._lib.ggnn_embed_workspace_bytes(self._segs(segments), len(segments), ctypes.byref(n)),
                       "ggnn_embed_workspace_bytes")
            ws = torch.zeros(max(int(n.value), 1), dtype=torch.uint8, device=device)
            self._ws[key] = ws
        return ws

    def _segs(self, segments, dtables=None):
        arr = (EmbedSegment * len(segments))()
        for i, (t, col) in enumerate(segments):
            dt = None if dtables is None or dtables[i] is None else dtables[i].data_ptr()
            arr[i] = EmbedSegment(t.data_ptr(), dt, t.shape[0], t.shape[1], int(col))
        return arr

    def lookup_rows(self, segments, seg, wi, dh0, keep, seed, rows, ids, dh0_add=None, seed_device=False):
        """Segment ``seg``'s gradient as IndexedSlices: rows [cap, width] (the
        per-lookup gradient rows, embedding dropout applied) and ids [cap]
        (int32, -1 past the batch) -- ggnn_embed_lookup_rows."""
        b, v, ncols = wi.shape
        d = _lib.dims(b, v, self.hidden, 1, 1, True, "fp32", seed_device=seed_device)
        _lib.check(self._lib.ggnn_embed_lookup_rows(ctypes.byref(d), self._segs(segments), len(segments), int(seg),
                                                    _ptr(wi), ncols, float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                    _ptr(dh0.contiguous()),
                                                    _ptr(None if dh0_add is None else dh0_add.contiguous()),
                                                    _ptr(rows), _ptr(ids), int(rows.shape[0]), _stream()),
                   "ggnn_embed_lookup_rows")

    def union_backward(self, table, dtable, rows, ids, sq_out):
        """The gradient of ``table`` from IndexedSlices (rows [n, width], ids
        [n]; -1 = none): dtable = the sum of the rows per id in 64-bit fixed
        point (exact, whatever order -- the same bits on every rank that holds
        the same slices), sq_out[0] = the sum of the squared rows
        (ggnn_embed_backward_ws over one segment, keep 1)."""
        n, w = rows.shape
        segs = [(table, 0)]
        d = _lib.dims(int(n), 1, int(w), 1, 1, True, "fp32")
        _lib.check(self._lib.ggnn_embed_backward_ws(ctypes.byref(d), self._segs(segs, [dtable]), 1,
                                                    _ptr(ids.contiguous()), 1, 1.0, 0, _ptr(rows.contiguous()),
                                                    None, _ptr(sq_out), _ptr(self.workspace(segs, rows.device)),
                                                    _stream()), "ggnn_embed_backward_ws")

    def forward(self, segments, wi: torch.Tensor, keep: float = 1.0, seed: int = 0, seed_device: bool = False,
                out=None) -> torch.Tensor:
        """seed_device: seed is the address of a device uint64 (GGNN_SEED_DEVICE)."""
        b, v, ncols = wi.shape
        h0 = out if out is not None else torch.empty(b, v, self.hidden, dtype=torch.float32, device=wi.device)
        d = _lib.dims(b, v, self.hidden, 1, 1, True, "fp32", seed_device=seed_device)
        _lib.check(self._lib.ggnn_embed_forward(ctypes.byref(d), self._segs(segments), len(segments), _ptr(wi), ncols,
                                                float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(h0), _stream()),
                   "ggnn_embed_forward")
        return h0

    def backward(self, segments, wi, dh0, keep=1.0, seed=0, dh0_add=None, dtables=None, sq_out=None,
                 seed_device=False):
        """Returns (per-segment dense table gradients, lookup sqnorm device
        vector [nseg]).  dtables: optional per-segment gradient buffers;
        segments that share a table may share one buffer (the kernel adds both
        segments' lookups into it, and the table's squared lookup norm goes to
        the first such segment's slot).  sq_out: optional [nseg] fp32 output
        (e.g. a view into a flat all-reduce buffer)."""
        b, v, ncols = wi.shape
        dts = dtables if dtables is not None else [torch.empty_like(t) for t, _ in segments]
        sq = sq_out if sq_out is not None else torch.empty(len(segments), dtype=torch.float32, device=wi.device)
        d = _lib.dims(b, v, self.hidden, 1, 1, True, "fp32", seed_device=seed_device)
        args = (ctypes.byref(d), self._segs(segments, dts), len(segments), _ptr(wi), ncols, float(keep),
                int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(dh0.contiguous()),
                _ptr(None if dh0_add is None else dh0_add.contiguous()), _ptr(sq))
        if self.deterministic:
            _lib.check(self._lib.ggnn_embed_backward_ws(*args, _ptr(self.workspace(segments, wi.device)), _stream()),
                       "ggnn_embed_backward_ws")
        else:
            _lib.check(self._lib.ggnn_embed_backward(*args, _stream()), "ggnn_embed_backward")
        return dts, sq


class OutputHeads:
    """heads: list of (W [2h, o], b [o]) tensors; labels per head [b, v, o]."""

    def __init__(self, hidden: int):
        self.hidden = int(hidden)
        self._lib = _lib.load()
        self._ws = None
        self._saved = None

    def _table(self, heads, labels, probs, dws=None, dbs=None):
        arr = (OutputHead * len(heads))()
        for i, (W, bias) in enumerate(heads):
            arr[i] = OutputHead(W.data_ptr(), bias.data_ptr(), W.shape[1],
                                None if labels is None or labels[i] is None else labels[i].data_ptr(),
                                probs[i].data_ptr(), None if dws is None else dws[i].data_ptr(),
                                None if dbs is None else dbs[i].data_ptr())
        return arr

    def forward(self, hT, h0, heads, labels=None, keep=1.0, seed=0, target_num=1.0, loss_out=None, probs_out=None,
                seed_device=False):
        """Returns (probs list [b, v, o], loss tensor [nheads] or None).
        loss_out / probs_out: optional output buffers (loss [nheads] fp32).
        target_num: a number, or a device fp32 tensor of one element
        (ggnn_heads_forward_dev); seed_device: seed is the address of a
        device uint64 (GGNN_SEED_DEVICE)."""
        b, v, h = hT.shape
        dev = hT.device
        probs = probs_out if probs_out is not None else [torch.empty(b, v, W.shape[1], dtype=torch.float32, device=dev)
                                                          for W, _ in heads]
        d = _lib.dims(b, v, h, 1, 1, True, "fp32", seed_device=seed_device)
        tab = self._table(heads, labels, probs)
        n = ctypes.c_size_t(0)
        _lib.check(self._lib.ggnn_heads_workspace_bytes(ctypes.byref(d), tab, len(heads), ctypes.byref(n)),
                   "ggnn_heads_workspace_bytes")
        if self._ws is None or self._ws.numel() < n.value:
            self._ws = torch.empty(max(int(n.value), 1), dtype=torch.uint8, device=dev)
        loss = None
        if labels is not None:
            loss = loss_out if loss_out is not None else torch.empty(len(heads), dtype=torch.float32, device=dev)
        if isinstance(target_num, torch.Tensor):
            _lib.check(self._lib.ggnn_heads_forward_dev(ctypes.byref(d), tab, len(heads), _ptr(hT.contiguous()),
                                                        _ptr(h0.contiguous()), float(keep),
                                                        int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(target_num), _ptr(loss),
                                                        _ptr(self._ws), _stream()),
                       "ggnn_heads_forward_dev")
        else:
            _lib.check(self._lib.ggnn_heads_forward(ctypes.byref(d), tab, len(heads), _ptr(hT.contiguous()),
                                                    _ptr(h0.contiguous()), float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                    float(target_num), _ptr(loss), _ptr(self._ws), _stream()),
                       "ggnn_heads_forward")
        self._saved = (b, v, h)
        return probs, loss

    def backward(self, hT, h0, heads, labels, probs, target_num=1.0, d_loss=None, dws=None, dbs=None, dhT=None,
                 dh0=None):
        """Gradients of sum(loss) (times d_loss, a device scalar): dW, db per
        head and (dhT, dh0).  Uses the workspace of the last forward.  dws, dbs,
        dhT, dh0: optional output buffers (overwritten)."""
        b, v, h = hT.shape
        if self._saved != (b, v, h):
            raise RuntimeError("heads backward without a matching forward")
        dws = dws if dws is not None else [torch.empty_like(W) for W, _ in heads]
        dbs = dbs if dbs is not None else [torch.empty_like(bb) for _, bb in heads]
        dhT = dhT if dhT is not None else torch.empty_like(hT)
        dh0 = dh0 if dh0 is not None else torch.empty_like(h0)
        d = _lib.dims(b, v, h, 1, 1, True, "fp32")
        tab = self._table(heads, labels, probs, dws, dbs)
        if isinstance(target_num, torch.Tensor):     # device target_num (ggnn_heads_backward_dev)
            _lib.check(self._lib.ggnn_heads_backward_dev(ctypes.byref(d), tab, len(heads), _ptr(hT.contiguous()),
                                                         _ptr(h0.contiguous()), _ptr(target_num), _ptr(d_loss),
                                                         _ptr(self._ws), _ptr(dhT), _ptr(dh0), _stream()),
                       "ggnn_heads_backward_dev")
        else:
            _lib.check(self._lib.ggnn_heads_backward(ctypes.byref(d), tab, len(heads), _ptr(hT.contiguous()),
                                                     _ptr(h0.contiguous()), float(target_num), _ptr(d_loss),
                                                     _ptr(self._ws), _ptr(dhT), _ptr(dh0), _stream()),
                       "ggnn_heads_backward")
        return dws, dbs, dhT, dh0


class EmbedFunction(torch.autograd.Function):
    """h0 = front-end(tables); backward gives the dense table gradients and
    stashes the per-lookup squared norms on ``owner.lookup_sqnorm`` (for
    ClipAdam's IndexedSlices clip)."""

    @staticmethod
    def forward(ctx, fe, owner, wi, keep, seed, cols, *tables):
        segs = list(zip(tables, cols))
        ctx.fe, ctx.owner, ctx.wi, ctx.keep, ctx.seed, ctx.cols = fe, owner, wi, keep, seed, cols
        ctx.tables = tables
        return fe.forward(segs, wi, keep, seed)

    @staticmethod
    def backward(ctx, dh0):
        segs = list(zip(ctx.tables, ctx.cols))
        # segments sharing a table (btb: loc_embeddings for the location and
        # the head location) share one gradient buffer
        first = [next(j for j, u in enumerate(ctx.tables) if u is t) for t in ctx.tables]
        bufs = {}
        for i, t in enumerate(ctx.tables):
            if first[i] == i:
                bufs[i] = torch.empty_like(t)
        dts, sq = ctx.fe.backward(segs, ctx.wi, dh0, ctx.keep, ctx.seed, dtables=[bufs[f] for f in first])
        # (a table's squared lookup norm is in its first segment's slot)
        ctx.owner.lookup_sqnorm = {id(t): sq[first[i]:first[i] + 1] for i, t in enumerate(ctx.tables)}
        out = tuple(bufs[i] if first[i] == i else None for i in range(len(ctx.tables)))
        return (None, None, None, None, None, None) + out


class HeadsFunction(torch.autograd.Function):
    """loss = sum over heads of the btb cross-entropy; also returns the probs
    (computed_values)."""

    @staticmethod
    def forward(ctx, oh, labels, keep, seed, target_num, hT, h0, *wb):
        heads = [(wb[2 * i], wb[2 * i + 1]) for i in range(len(wb) // 2)]
        probs, loss = oh.forward(hT, h0, heads, labels, keep, seed, target_num)
        ctx.oh, ctx.labels, ctx.target_num = oh, labels, target_num
        ctx.save_for_backward(hT, h0, *wb)
        ctx.probs = probs
        ctx.mark_non_differentiable(*probs)
        return (loss.sum(),) + tuple(probs)

    @staticmethod
    def backward(ctx, d_loss, *unused):
        hT, h0, *wb = ctx.saved_tensors
        heads = [(wb[2 * i], wb[2 * i + 1]) for i in range(len(wb) // 2)]
        dws, dbs, dhT, dh0 = ctx.oh.backward(hT, h0, heads, ctx.labels, ctx.probs, ctx.target_num,
                                             d_loss.reshape(1).contiguous())
        grads = []
        for dw, db in zip(dws, dbs):
            grads += [dw, db]
        return (None, None, None, None, None, dhT, dh0) + tuple(grads)
