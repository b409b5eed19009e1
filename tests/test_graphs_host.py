"""Host side of the hipGraph-captured steps (ggnn_amd/graphs.py): the staging
layout one H2D copy fills, and the edge-list validation it shares with
PropagationEngine.set_adjacency_edges.  No GPU."""
import numpy as np
import pytest

from ggnn_amd.graphs import StepLayout, edge_arrays


def test_step_layout_fill_places_every_input():
    b, v, ncols, o, oe = 3, 7, 6, 150, 12
    L = StepLayout(b, v, ncols, o, oe)
    for off in (L.wi, L.edges, L.offs, L.yh, L.ye):
        assert off % 64 == 0 and off >= StepLayout.SCALARS
    assert L.wi < L.edges < L.offs < L.yh < L.ye < L.nbytes
    assert L.edge_capacity == b * v
    rng = np.random.default_rng(0)
    wi = rng.integers(0, 100, (b, v, ncols)).astype(np.int32)
    edges = rng.integers(0, 5, (9, 3)).astype(np.int32)
    offs = np.array([0, 3, 7, 9], np.int32)
    yh = rng.random((b, v, o)).astype(np.float32)
    ye = rng.random((b, v, oe)).astype(np.float32)
    host = np.zeros(L.nbytes, np.uint8)
    seeds = [2 ** 63 - 5, 17, 2 ** 40 + 3]
    L.fill(host, seeds, 12345, 61.0000001, wi, edges, offs, yh, ye)
    assert list(host[0:24].view(np.uint64)) == seeds
    assert host[24:32].view(np.int64)[0] == 12345
    assert host[32:36].view(np.float32)[0] == np.float32(61.0000001)
    assert np.array_equal(host[L.wi:L.wi + wi.nbytes].view(np.int32).reshape(wi.shape), wi)
    assert np.array_equal(host[L.edges:L.edges + edges.nbytes].view(np.int32).reshape(edges.shape), edges)
    assert np.array_equal(host[L.offs:L.offs + offs.nbytes].view(np.int32), offs)
    assert np.array_equal(host[L.yh:L.yh + yh.nbytes].view(np.float32).reshape(yh.shape), yh)
    assert np.array_equal(host[L.ye:L.ye + ye.nbytes].view(np.float32).reshape(ye.shape), ye)


def test_edge_arrays_concatenate_and_validate():
    graphs = [[[0, 1, 1], [1, 2, 2]], [], [[2, 3, 0]]]
    e, offs = edge_arrays(graphs, 4, 3)
    assert offs.tolist() == [0, 2, 2, 3]
    assert e.tolist() == [[0, 1, 1], [1, 2, 2], [2, 3, 0]]
    e0, o0 = edge_arrays([[], []], 4, 3)
    assert e0.shape == (0, 3) and o0.tolist() == [0, 0, 0]
    with pytest.raises(IndexError):
        edge_arrays([[[0, 4, 1]]], 4, 3)        # label outside 1..E (the reference indexes out of range)
    with pytest.raises(IndexError):
        edge_arrays([[[0, 1, 4]]], 4, 3)        # node outside 0..v-1


def test_captured_step_cache_evicts_least_recently_used():
    """model._evict_graphs: while the captured steps hold more than
    params['hip_graph_cache_mb'], the least recently used one is released
    (never the step that just ran)."""
    from collections import OrderedDict
    from test_dist import _golden_model

    class Fake:
        def __init__(self, mb):
            self.mb, self.released = mb, False

        def nbytes(self):
            return self.mb * 2 ** 20

        def release(self):
            self.released = True

    m, _ = _golden_model()
    m.params["hip_graph_cache_mb"] = 10
    steps = {k: Fake(4) for k in "abcd"}
    m._graphs = OrderedDict(steps)
    m._graphs.move_to_end("a")            # "a" ran most recently but one
    m._graphs.move_to_end("d")
    m._evict_graphs(keep="d")
    assert list(m._graphs) == ["a", "d"] and steps["b"].released and steps["c"].released
    assert m.graph_stats["evicted"] == 2 and m.graph_stats["cache_bytes"] == 8 * 2 ** 20
    m.params["hip_graph_cache_mb"] = 1
    m._evict_graphs(keep="a")             # one step always stays: the one that ran
    assert list(m._graphs) == ["a"] and not steps["a"].released
