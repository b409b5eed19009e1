"""hipGraph capture of run_epoch's per-batch step.

The reference runs one ``sess.run`` per minibatch (chem_tensorflow.py:595);
here the eager step is ~85 library launches (front-end, adjacency staging,
weight pack, T-step forward, heads, the backward of each, clip + Adam), and at
the reference's batch_size 20 the host's launch work is close to the GPU time.
A captured step replaces them with one H2D copy of the batch's inputs and one
graph launch.  A shape's first batch runs the same body eagerly (one-off
shapes never pay for a capture); its second batch is captured and replayed.

What stays fixed across replays of one graph (its key: batch shape (b, v),
the word_inputs width, the dropout keep probabilities, train / eval): every
device pointer (the step owns its engine -- adjacency, workspaces -- and its
heads workspace; the variables, their Adam slots and the flat gradient buffer
belong to the model), every launch shape and every host scalar the library
bakes into a launch.  What changes per batch lives in one device buffer
(``StepInputs``) that the graph reads: word_inputs, the edge list and graph
offsets (capacity b*v rows; the kernels read only rows [off[0], off[b])), both
heads' labels, and the step scalars -- the three dropout seeds
(GGNN_SEED_DEVICE), the loss normaliser target_num (ggnn_heads_*_dev) and the
Adam step count (ggnn_adam_step_dev).  Results equal the eager step's on the
same inputs and seeds (tests/test_gpu_graphs.py).

Staging: the host writes a batch into one of two page-locked buffers
(alternating; each reused only after its previous copy completed, an event),
then one ``copy_`` moves it into the step's device buffer on the stream, ahead
of the replay.
"""
from __future__ import annotations

import numpy as np
import torch

_ALIGN = 256


def _al(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class StepLayout:
    """Byte layout of one batch shape's inputs (the same on the host staging
    buffer and the device buffer).  Scalars: seeds uint64[3] at 0 (front-end,
    path, heads), the Adam step int64 at 24, target_num fp32 at 32."""
    SCALARS = 64

    def __init__(self, b: int, v: int, ncols: int, o: int, oe: int):
        self.b, self.v, self.ncols, self.o, self.oe = int(b), int(v), int(ncols), int(o), int(oe)
        n = self.b * self.v
        off = self.SCALARS
        self.wi = off
        off = _al(off + n * self.ncols * 4)
        self.edges = off
        off = _al(off + n * 3 * 4)
        self.offs = off
        off = _al(off + (self.b + 1) * 4)
        self.yh = off
        off = _al(off + n * self.o * 4)
        self.ye = off
        off = _al(off + n * self.oe * 4)
        self.nbytes = off

    @property
    def edge_capacity(self) -> int:
        return self.b * self.v

    def fill(self, host: np.ndarray, seeds, step: int, target_num, wi, edges, offs, yh, ye) -> None:
        """Write one batch into ``host`` (a uint8 array of >= nbytes)."""
        b, v = self.b, self.v
        host[0:24].view(np.uint64)[:] = np.asarray(seeds, dtype=np.uint64)
        host[24:32].view(np.int64)[0] = int(step)
        host[32:36].view(np.float32)[0] = np.float32(target_num)
        host[self.wi:self.wi + wi.nbytes].view(np.int32)[:] = wi.reshape(-1)
        if edges.size:
            host[self.edges:self.edges + edges.nbytes].view(np.int32)[:] = edges.reshape(-1)
        host[self.offs:self.offs + (b + 1) * 4].view(np.int32)[:] = offs
        host[self.yh:self.yh + b * v * self.o * 4].view(np.float32)[:] = yh.reshape(-1)
        host[self.ye:self.ye + b * v * self.oe * 4].view(np.float32)[:] = ye.reshape(-1)


class StepInputs:
    """The device buffer one captured step reads, with typed views."""

    def __init__(self, layout: StepLayout, device):
        L = self.layout = layout
        b, v, n = L.b, L.v, L.b * L.v
        self.buf = torch.zeros(L.nbytes, dtype=torch.uint8, device=device)
        u = self.buf
        self.seeds = u[0:24].view(torch.int64)
        self.step = u[24:32].view(torch.int64)
        self.target_num = u[32:36].view(torch.float32)
        self.wi = u[L.wi:L.wi + n * L.ncols * 4].view(torch.int32).view(b, v, L.ncols)
        self.edges = u[L.edges:L.edges + n * 12].view(torch.int32).view(n, 3)
        self.offs = u[L.offs:L.offs + (b + 1) * 4].view(torch.int32)
        self.yh = u[L.yh:L.yh + n * L.o * 4].view(torch.float32).view(b, v, L.o)
        self.ye = u[L.ye:L.ye + n * L.oe * 4].view(torch.float32).view(b, v, L.oe)

    def seed_address(self, i: int) -> int:
        return self.seeds.data_ptr() + 8 * int(i)


class PinnedRing:
    """Two alternating page-locked staging buffers; a buffer is rewritten only
    after the copy that last read it has completed."""

    def __init__(self):
        self._bufs = [None, None]
        self._events = [None, None]
        self._i = 0

    def acquire(self, nbytes: int):
        i = self._i
        ev = self._events[i]
        if ev is not None:
            ev.synchronize()
        buf = self._bufs[i]
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(int(nbytes), 1 << 20), dtype=torch.uint8, pin_memory=True)
            self._bufs[i] = buf
        return i, buf[:nbytes]

    def release(self, i: int, stream) -> None:
        ev = torch.cuda.Event()
        ev.record(stream)
        self._events[i] = ev
        self._i ^= 1


class CapturedStep:
    """One batch shape's inputs, private engine / heads and (after its first,
    eager run) its graph and the graph's output tensors."""

    def __init__(self, layout: StepLayout, engine, heads, device):
        self.layout = layout
        self.inputs = StepInputs(layout, device)
        self.engine = engine
        self.heads = heads
        self.graph = None
        self.out = None
        self.runs = 0               # batches this step has run (eager first, then replays)
        self.pool_bytes = 0         # allocated in the graph's private pool during the capture

    def nbytes(self) -> int:
        """Device bytes this step holds: its input buffer, the engine's staged
        adjacency and workspaces, the heads' workspace, and what the captured
        body allocated in the graph's private pool (its activations and
        outputs: memory_allocated across the capture)."""
        n = self.inputs.buf.numel() + int(self.pool_bytes)
        eng = self.engine
        if getattr(eng, "_adj", None) is not None:
            n += eng._adj.numel()
        n += sum(w.numel() for w in getattr(eng, "_ws", {}).values())
        ws = getattr(self.heads, "_ws", None)
        if ws is not None:
            n += ws.numel()
        return int(n)

    def release(self) -> None:
        """Free the graph and every buffer it references (eviction)."""
        if self.graph is not None:
            self.graph.reset()
        self.graph = self.out = None
        self.engine = self.heads = self.inputs = None


def edge_arrays(graphs, v: int, num_edge_types: int):
    """(edges int32 [n, 3], offsets int32 [b + 1]) of a batch's per-graph edge
    lists, validated as PropagationEngine.set_adjacency_edges does (the
    reference raises IndexError for them)."""
    b = len(graphs)
    offs = np.zeros(b + 1, np.int32)
    offs[1:] = np.cumsum([len(g) for g in graphs])
    n = int(offs[-1])
    if not n:
        return np.zeros((0, 3), np.int32), offs
    e = np.concatenate([np.asarray(g, np.int32).reshape(-1, 3) for g in graphs if len(g)])
    src, lab, dst = e[:, 0], e[:, 1], e[:, 2]
    if lab.min() < 1 or lab.max() > num_edge_types:
        raise IndexError("edge label outside 1..%d" % num_edge_types)
    if min(src.min(), dst.min()) < 0 or max(src.max(), dst.max()) >= v:
        raise IndexError("edge node index outside 0..%d" % (v - 1))
    return e, offs
