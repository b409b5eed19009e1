"""Our btb batching (ggnn_amd.batching) against golden fixtures produced by the
REFERENCE's own numpy helpers (tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest

from ggnn_amd.batching import BtbBatching, graph_to_adj_mat_bd

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "batching_golden.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD, allow_pickle=False)


class _M(BtbBatching):
    def __init__(self, g):
        self.num_edge_types = int(g["num_edge_types"])
        self.output_size_edges = int(g["output_size_edges"])
        self.pos_size = int(g["pos_size"])
        self.bucket_max_nodes = int(g["bucket_max_nodes"])
        self.params = {"batch_size": 8, "output_size": 150, "task_ids": [0], "task_sample_ratios": {},
                       "tie_fwd_bkwd": True, "hidden_size": 400, "graph_state_dropout_keep_prob": 0.9,
                       "emb_dropout_keep_prob": 0.55}


def test_graph_to_adj_mat_bd_matches_reference(gold):
    data = json.loads(str(gold["raw_json"]))
    E = int(gold["num_edge_types"])
    for i in range(6):
        exp = gold["adj_%d" % i]
        got = graph_to_adj_mat_bd(data[i]["graph"], exp.shape[1], E)
        assert got.shape == exp.shape and got.dtype == np.float64
        assert np.array_equal(got.astype(np.uint8), exp)


def test_eval_minibatches_match_reference(gold):
    m = _M(gold)
    data = json.loads(str(gold["raw_json"]))
    feeds = list(m.make_minibatch_iterator(m.process_raw_graphs(data, False), False))
    assert len(feeds) == int(gold["n_eval_batches"])
    for bi, fd in enumerate(feeds):
        p = "eval%d_" % bi
        assert np.array_equal(np.asarray(fd["adjacency_matrix"]).astype(np.uint8), gold[p + "adjacency"])
        assert np.array_equal(fd["word_inputs"].astype(np.int32), gold[p + "word_inputs"])
        for k in ("node_mask", "node_mask_edges", "target_values_head", "target_values_edges",
                  "target_mask", "target_pos"):
            assert np.array_equal(np.asarray(fd[k]).astype(np.float32), gold[p + k]), k
        sc = gold[p + "scalars"]
        assert (fd["num_graphs"], fd["num_vertices"]) == (int(sc[0]), int(sc[1]))
        assert fd["graph_state_keep_prob"] == sc[2] and fd["emb_dropout_keep_prob"] == sc[3]
        assert list(fd["sentences_id"]) == list(gold[p + "ids"])


def test_training_order_matches_reference_rng(gold):
    m = _M(gold)
    data = json.loads(str(gold["raw_json"]))
    np.random.seed(0)
    feeds = list(m.make_minibatch_iterator(m.process_raw_graphs(data, True), True))
    assert len(feeds) == int(gold["n_train_batches"])
    for bi, fd in enumerate(feeds):
        assert list(fd["sentences_id"]) == list(gold["train%d_ids" % bi])
        sc = gold["train%d_scalars" % bi]
        assert fd["graph_state_keep_prob"] == sc[2] and fd["emb_dropout_keep_prob"] == sc[3]


def test_empty_graph_is_skipped_and_buckets():
    m = _M({"num_edge_types": 3, "output_size_edges": 2, "pos_size": 5, "bucket_max_nodes": 10})
    raw = [{"graph": [], "node_features": [0], "words_index": [0], "targets": [], "node_features_target": [0]},
           {"graph": [[0, 1, 1], [1, 2, 2]], "node_features": [0, 1, 2], "words_index": [0, 5, 6],
            "targets": [[0, 1], [1, 2]], "node_features_target": [0, 1, 2], "id": "x"}]
    bucketed, sizes, steps = m.process_raw_graphs(raw, False)
    assert steps == [0] and sizes[0] == 4            # max node id 2 -> bucket 4
    fd = next(m.make_minibatch_iterator((bucketed, sizes, steps), False))
    assert fd["adjacency_matrix"][0].shape == (6, 4, 4) and fd["num_graphs"] == 1


def test_threaded_iterator_and_synthetic_treebank():
    """ThreadedIterator (utils.py:17-37) preserves order and surfaces producer
    errors; the synthetic treebank (bench / e2e tests) goes through the
    reference's batching unchanged."""
    from ggnn_amd.batching import ThreadedIterator, synthetic_treebank
    assert list(ThreadedIterator(iter(range(50)), max_queue_size=3)) == list(range(50))

    def bad():
        yield 1
        raise KeyError("boom")
    with pytest.raises(KeyError):
        list(ThreadedIterator(bad()))
    raw = synthetic_treebank(60, seed=3)
    assert all(len(d["graph"]) == len(d["node_features"]) - 1 == len(d["targets"]) for d in raw)
    assert all(0 <= e[0] < len(d["node_features"]) and 1 <= e[1] < 46 for d in raw for e in d["graph"])

    class M(BtbBatching):
        params = {"batch_size": 8, "output_size": 150, "task_ids": [0], "task_sample_ratios": {},
                  "tie_fwd_bkwd": True, "graph_state_dropout_keep_prob": 0.9, "emb_dropout_keep_prob": 0.55,
                  "out_layer_dropout_keep_prob": 0.85, "compact_adjacency": True}
        num_edge_types, output_size_edges, pos_size, bucket_max_nodes = 46, 12, 46, 120
    m = M()
    data = m.process_raw_graphs(raw, False)
    feeds = list(m.make_minibatch_iterator(data, False))
    assert sum(f["num_graphs"] for f in feeds) == 60
    for f in feeds:
        assert f["adjacency_matrix"] is None and len(f["adjacency_edges"]) == f["num_graphs"]
        assert f["word_inputs"].shape == (f["num_graphs"], f["num_vertices"], 6)
