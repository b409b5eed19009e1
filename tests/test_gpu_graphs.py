"""hipGraph-captured steps (ggnn_amd/graphs.py) against the eager path.

The captured step reads its batch and its step scalars (dropout seeds,
target_num, Adam step) from device memory and replays the same launches; on
the same inputs and seeds it must give the eager step's results.  Since
round 5 every reduction of the library is order-fixed (split-K slabs summed
in z order, bias partials summed in row order, fixed-point embedding
accumulators: no fp32 atomics), so the two paths agree BIT FOR BIT at every
step, through Adam at the reference's epsilon 1e-8 (round 4 compared the
first step at 1e-5 and later steps within the drift fp32 atomics left).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _model(graphs, lr=None):
    from ggnn_amd.batching import wsj_model_sizes
    from ggnn_amd.model import DenseGGNNChemModel
    params = {"compact_adjacency": True, "hip_graphs": graphs}
    if lr is not None:
        params["learning_rate"] = lr
    return DenseGGNNChemModel(params=params, seed=0, **wsj_model_sizes())


def _feeds(m, restrict, training):
    from ggnn_amd.batching import TRAIN_WITH_DEV
    np.random.seed(0)
    data = m.load_data(TRAIN_WITH_DEV["train_file"], training, restrict=restrict)
    return list(m.make_minibatch_iterator(data, training))


def _shape_sequence(feeds):
    """A batch, the same batch again (new seeds, new weights), a batch of
    another shape, the first again, the second again: eager first run,
    capture + replay, eager first run, replay, capture + replay."""
    a = feeds[0]
    other = next(f for f in feeds if (f["num_graphs"], f["num_vertices"]) != (a["num_graphs"], a["num_vertices"]))
    return [a, a, other, a, other]


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def test_captured_train_steps_match_eager():
    torch = _torch()
    ea, gr = _model(False), _model(True)
    seq = _shape_sequence(_feeds(ea, 100, True))
    for k, f in enumerate(seq):
        w0 = [p.detach().clone() for p in gr.trainable_variables()]
        la = float(ea.train_step(dict(f)))
        pa = ea.ops["computed_values"].clone()
        lb = float(gr.train_step(dict(f)))
        torch.cuda.synchronize()
        # same weights, inputs and seeds: the same bits everywhere, every step
        assert la == lb, (k, la, lb)
        assert torch.equal(pa, gr.ops["computed_values"]), k
        assert torch.equal(gr.train_buffer().flat, ea.train_buffer().flat), (k, _rel(gr.train_buffer().flat,
                                                                                    ea.train_buffer().flat))
        for ma, mb in zip(ea.optimizer.m + ea.optimizer.v, gr.optimizer.m + gr.optimizer.v):
            assert torch.equal(ma, mb), k
        for pe, pg in zip(ea.trainable_variables(), gr.trainable_variables()):
            assert torch.equal(pe.detach(), pg.detach()), k
        assert ea.optimizer.t == gr.optimizer.t == k + 1
    st = gr.graph_stats
    assert st["captured"] == 2 and st["replayed"] == 3 and st["uncaptured"] == 2 and st["eager"] == 0, st
    assert ea.graph_stats["eager"] == len(seq)


def test_captured_eval_matches_eager():
    torch = _torch()
    ea, gr = _model(False), _model(True)
    from ggnn_amd.batching import TRAIN_WITH_DEV
    valid = ea.load_data(TRAIN_WITH_DEV["valid_file"], False, restrict=150)
    ra = ea.run_epoch("valid", valid, False)
    for _ in range(3):               # first pass eager, second captures, third replays
        rb = gr.run_epoch("valid", valid, False)
        torch.cuda.synchronize()
        assert abs(ra[0] - rb[0]) <= 1e-6 * abs(ra[0])
        assert ra[5] == rb[5] and ra[6] == rb[6] and ra[16] == rb[16]
        for xa, xb in zip(ra[8], rb[8]):
            assert np.array_equal(xa, xb)            # computed_values: forward only, deterministic
    assert gr.graph_stats["replayed"] > 0


def test_captured_run_epoch_trains_like_eager():
    """Two training epochs through captured steps equal the eager run: the
    same epoch loss and LAS / UAS (every step bit-identical, see above)."""
    _torch()
    from ggnn_amd.batching import TRAIN_WITH_DEV
    ea, gr = _model(False), _model(True)
    # (one copy of the data per model: run_epoch shuffles its buckets in place)
    np.random.seed(0)
    train_a = ea.load_data(TRAIN_WITH_DEV["train_file"], True, restrict=200)
    np.random.seed(0)
    train_b = gr.load_data(TRAIN_WITH_DEV["train_file"], True, restrict=200)
    for epoch in range(2):
        np.random.seed(epoch + 1)
        ra = ea.run_epoch("e", train_a, True)
        np.random.seed(epoch + 1)
        rb = gr.run_epoch("g", train_b, True)
        assert ra[0] == rb[0] and ra[5] == rb[5] and ra[6] == rb[6] and ra[16] == rb[16], (epoch, ra[0], rb[0])
    st = gr.graph_stats
    assert st["replayed"] > 0 and st["eager"] == 0


def test_profiler_sees_no_capture():
    """The kernel timer skips records while a stream is capturing (a timed
    epoch with graphs on still completes and times its eager launches)."""
    torch = _torch()
    from ggnn_amd import _lib
    gr = _model(True)
    feeds = _feeds(gr, 60, True)
    with _lib.KernelTimer(max_launches=100000) as t:
        for f in feeds[:3]:
            gr.train_step(dict(f))
        torch.cuda.synchronize()
    assert sum(t.launches.values()) > 0
