"""Data-parallel plumbing: one process per GPU, gradients all-reduced over RCCL.

Two flat buffers: ``FlatGradients`` (the path's six weight gradients, the
propagation-only step of bench.py) and ``FlatTrainBuffer`` (every trainable
variable of the btb model plus the IndexedSlices norms and the losses, the
whole training step of ``DenseGGNNChemModel.train_step``).

The propagation path shards naturally by graph (chem_tensorflow_dense.py:414-428
contracts only inside graph g); the only cross-graph coupling is the batch sum
of the weight gradients (TF autodiff, chem_tensorflow.py:496).  Each rank runs
its own batch through the engine, then ONE all-reduce of a flat fp32 gradient
buffer per step (3.68 MB at h=256, C=8) sums them.  The per-tensor
clip_by_norm of the reference (chem_tensorflow.py:498-503) must see the
reduced gradient, so it runs after this reduction (optimizer, next row).

``torch.distributed`` with backend "nccl" is RCCL on ROCm; "gloo" is used by
the CPU tests.

A collective normally runs only when the group has more than one rank.  An
explicit backend passed to ``init_from_env`` at WORLD_SIZE 1 (bench.py
``--dist-backend nccl`` under a one-rank torchrun) still creates the process
group and turns the collectives on (``collectives_at_world_one``), so the
RCCL path that an N-GPU run takes can be executed on a one-GPU box: the sum
over one rank leaves every value unchanged.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as tdist

_ALWAYS = False   # collectives at world size 1 (init_from_env with an explicit backend)


def collectives_at_world_one(on: bool | None = None) -> bool:
    """Whether FlatGradients.all_reduce / all_reduce_sum issue their collective
    in a one-rank group (set by init_from_env with an explicit backend at
    WORLD_SIZE 1; ``on`` overrides).  Returns the setting."""
    global _ALWAYS
    if on is not None:
        _ALWAYS = bool(on)
    return _ALWAYS


def _reducing(group) -> bool:
    if not (tdist.is_available() and tdist.is_initialized()):
        return False
    return tdist.get_world_size(group) > 1 or _ALWAYS


GRAD_ORDER = ("edge_weights", "edge_biases", "gates_kernel", "gates_bias",
              "candidate_kernel", "candidate_bias")


def grad_shapes(hidden: int, channels: int, use_edge_bias: bool = True):
    h, C = hidden, channels
    shapes = {
        "edge_weights": (C, h, h),
        "edge_biases": (C, 1, h),
        "gates_kernel": (2 * h, 2 * h),
        "gates_bias": (2 * h,),
        "candidate_kernel": (2 * h, h),
        "candidate_bias": (h,),
    }
    if not use_edge_bias:
        shapes.pop("edge_biases")
    return shapes


class FlatGradients:
    """One contiguous fp32 buffer holding every weight gradient of the path;
    ``views`` are the per-tensor views the engine writes into, so the
    all-reduce is a single collective with no packing copy."""

    def __init__(self, hidden: int, channels: int, use_edge_bias: bool = True, device=None):
        self.shapes = grad_shapes(hidden, channels, use_edge_bias)
        total = sum(int(torch.Size(s).numel()) for s in self.shapes.values())
        self.flat = torch.zeros(total, dtype=torch.float32, device=device)
        self.views = {}
        off = 0
        for name in GRAD_ORDER:
            if name not in self.shapes:
                continue
            n = int(torch.Size(self.shapes[name]).numel())
            self.views[name] = self.flat[off:off + n].view(self.shapes[name])
            off += n

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def all_reduce(self, group=None) -> None:
        """Sum the gradients over all ranks (RCCL on GPUs, gloo on CPU)."""
        if _reducing(group):
            tdist.all_reduce(self.flat, op=tdist.ReduceOp.SUM, group=group)


class FlatTrainBuffer:
    """ONE contiguous fp32 buffer for a whole btb training step of the model
    (``DenseGGNNChemModel.train_step``): the gradient of every trainable
    variable (the path's six tensors, the loc/pos/word embedding tables and
    both output heads' W, b), then the tables' squared lookup norms (the
    IndexedSlices norms ``tf.clip_by_norm`` takes, chem_tensorflow.py:498-500)
    and the per-head losses.  Every producer writes straight into its views
    (ggnn_backward, ggnn_heads_backward, ggnn_embed_backward, heads forward),
    so a data-parallel step is a single all-reduce of ``flat`` with no packing
    copy, and it sums the gradients, the lookup norms and the losses at once.

    Each view starts on a 64-float (256-byte) boundary (the library's
    16-byte vector paths and the MFMA epilogues' stores).

    Layout (round 5): the ``first`` variables (the output heads, whose
    gradients are final before the propagation backward starts) and the
    losses, then the other dense variables and the lookup norms, then the
    ``sparse`` variables (the word embedding table: reduced as IndexedSlices,
    not all-reduced densely).  ``buckets`` = [(heads + losses), (the rest of
    the dense part)] as flat slices; ``dense`` = both."""

    ALIGN = 64

    def __init__(self, params, n_sq: int, n_loss: int, device=None, first=(), sparse=()):
        n = len(params)
        first, sparse = [i for i in first if i not in sparse], list(sparse)
        rest = [i for i in range(n) if i not in first and i not in sparse]
        al = lambda k: -(-k // self.ALIGN) * self.ALIGN  # noqa: E731
        offs, off = [None] * n, 0
        for i in first:
            offs[i] = off
            off += al(int(params[i].numel()))
        loss_off = off
        off += al(int(n_loss))
        self._b0 = off
        for i in rest:
            offs[i] = off
            off += al(int(params[i].numel()))
        sq_off = off
        off += al(int(n_sq))
        self._dense_end = off
        for i in sparse:
            offs[i] = off
            off += al(int(params[i].numel()))
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.grads = [self.flat[o:o + p.numel()].view(p.shape) for o, p in zip(offs, params)]
        self.sq = self.flat[sq_off:sq_off + n_sq]
        self.loss = self.flat[loss_off:loss_off + n_loss]
        self.sparse = tuple(sparse)

    @property
    def dense(self) -> torch.Tensor:
        """Everything the all-reduce sums (all but the sparse variables)."""
        return self.flat[:self._dense_end]

    @property
    def buckets(self):
        """(heads + losses, the rest of the dense part): the first is final
        after the heads' backward, so its reduction can start while the
        propagation backward runs."""
        return self.flat[:self._b0], self.flat[self._b0:self._dense_end]

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * 4

    def zero_(self) -> None:
        """A rank without a batch in this global step contributes zeros."""
        self.flat.zero_()


class Reducer:
    """Sums tensors over the ranks of a group (RCCL on GPUs, gloo on CPU).
    Called as ``r(t)``: a blocking in-place all-reduce.  ``start(t)`` issues
    it asynchronously (RCCL runs it on its own stream after the work queued
    so far on the current stream) and returns a handle; ``wait(h)`` makes the
    current stream wait for it.  ``gather(t)``: all ranks' ``t`` stacked in
    rank order (all_gather_into_tensor)."""

    def __init__(self, group=None):
        self.group = group
        self.world = tdist.get_world_size(group)

    def __call__(self, t):
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group)

    def start(self, t):
        return tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group, async_op=True)

    @staticmethod
    def wait(h):
        if h is not None:
            h.wait()

    def gather(self, t):
        t = t.contiguous()
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        tdist.all_gather_into_tensor(out, t, group=self.group)
        return out.view((self.world,) + tuple(t.shape))


def all_reduce_sum(group=None):
    """A Reducer summing a tensor over the ranks of `group` (RCCL on GPUs,
    gloo on CPU), or None outside a multi-rank job (a one-rank group counts
    as multi-rank when collectives_at_world_one() is on)."""
    if not _reducing(group):
        return None
    return Reducer(group)


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, local_rank).

    backend None: a group only when WORLD_SIZE > 1 (nccl = RCCL on a GPU, else
    gloo).  An explicit backend at WORLD_SIZE 1 also creates the (one-rank)
    group, needs MASTER_ADDR / MASTER_PORT, and turns the collectives on
    (collectives_at_world_one): the rehearsal of the N-rank RCCL path on one
    GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or backend is not None) and not tdist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            tdist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        if world == 1:
            collectives_at_world_one(True)
    return rank, world, local
