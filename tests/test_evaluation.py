"""Host LAS/UAS scoring and the checkpoint format.

The adj_mat_to_target / get_las_uas vectors are the reference's own unit tests
(tests_chem.py:9-27, 50-88), restated as data.
"""
import os
import pickle

import numpy as np
import pytest
import torch

from ggnn_amd import evaluation as E
from ggnn_amd import checkpoint as K
from ggnn_amd.model import DenseGGNNChemModel


def test_adj_mat_to_target_reference_vector():
    # tests_chem.py:9-27
    adj = np.array([[[0., 0., 0., 0., 0.], [0., 0., 0., 1., 0.], [0., 0., 0., 1., 0.], [0., 0., 0., 0., 0.]],
                    [[0., 0., 0., 0., 0.], [0., 0., 0., 0., 0.], [0., 0., 0., 0., 0.], [1., 0., 0., 0., 0.]]])
    assert E.adj_mat_to_target(adj_mat=adj) == [[3, 1], [3, 1], [0, 2]]


@pytest.mark.parametrize("result,expected", [
    ([[1, 1], [2, 0], [2, 2]], (1, 1)),        # tests_chem.py:50-58
    ([[1, 1], [2, 1], [2, 2]], (2 / 3, 1)),    # :60-68
    ([[1, 0], [2, 1], [2, 1]], (0, 1)),        # :70-78
    ([[2, 1], [1, 0], [3, 2]], (0, 0)),        # :80-88
])
def test_get_las_uas_reference_vectors(result, expected):
    target = [[1, 1], [2, 0], [2, 2]]
    assert E.get_las_uas(target_graph=target, result_graph=result) == expected
    assert DenseGGNNChemModel.get_las_uas(target, result) == expected


def test_adj_mat_to_target_probability_first_maximum():
    rng = np.random.default_rng(0)
    a = rng.random((3, 6, 6))
    a[1, 2, 4] = a[2, 2, 0] = 5.0          # tie: (e=1, src=4) comes first in (e, src) order
    g = E.adj_mat_to_target(a, is_probability=True)
    assert g[1] == [4, 2]
    for node, edge in zip(range(1, 6), g):
        e, src = np.unravel_index(np.argmax(a[:, node, :]), a[:, node, :].shape)
        assert edge == [int(src), int(e) + 1]


def test_batch_las_uas_perfect_and_wrong_predictions():
    b, v, o, e = 3, 5, 7, 4
    rng = np.random.default_rng(1)
    heads = np.zeros((b, v, o), np.float32)
    labs = np.zeros((b, v, e), np.float32)
    for g in range(b):
        for node in range(1, v):
            heads[g, node, rng.integers(0, v)] = 1
            labs[g, node, rng.integers(0, e)] = 1
    mask = np.ones((b, v * o), np.float32)
    mask_e = np.ones((b, v * e), np.float32)
    las, uas, le = E.batch_las_uas(heads.reshape(b, -1), heads.reshape(b, -1), v, mask,
                                   labs.reshape(b, -1), labs.reshape(b, -1), mask_e, o, e)
    assert (las, uas, le) == (1.0, 1.0, 1.0)
    wrong = np.roll(labs, 1, axis=2)  # every label wrong, heads right
    las, uas, le = E.batch_las_uas(heads.reshape(b, -1), heads.reshape(b, -1), v, mask,
                                   labs.reshape(b, -1), wrong.reshape(b, -1), mask_e, o, e)
    assert las == 0.0 and uas == 1.0 and le == 0.0


def _cpu_model(seed):
    return DenseGGNNChemModel(params={"hidden_size": 64, "num_timesteps": 2}, num_edge_types=3, device="cpu",
                              seed=seed, precision="fp32", vocab_size=50, embedding_sizes=dict(loc=16, pos=8, word=24,
                                                                                                  edge=16))


def test_checkpoint_names_follow_the_tf_graph():
    names = K.variable_names(_cpu_model(0))
    assert "graph_model/Variable:0" in names and "graph_model/Variable_3:0" in names
    assert tuple(names["graph_model/Variable:0"].shape) == (6, 64, 64)          # edge_weights [2E, h, h]
    assert tuple(names["graph_model/Variable_1:0"].shape) == (6, 1, 64)         # edge_biases
    assert tuple(names["graph_model/gru_scope/gru_cell/gates/kernel:0"].shape) == (128, 128)
    assert "out_layer_task0/regression_gate/MLP_W_layer0_1:0" in names
    assert "graph_model/word_embedding:0" in names


class _FakeAdam:  # ClipAdam's state attributes (the real one needs a GPU)
    def __init__(self, params):
        self.params = params
        self.m = [torch.full_like(p, 0.25) for p in params]
        self.v = [torch.full_like(p, 0.5) for p in params]
        self.b1, self.b2, self.t = 0.9, 0.999, 7


def test_checkpoint_round_trip(tmp_path):
    a, b = _cpu_model(0), _cpu_model(1)
    a.optimizer = _FakeAdam(a.trainable_variables())
    b.optimizer = _FakeAdam(b.trainable_variables())
    for m in b.optimizer.m:
        m.zero_()
    b.optimizer.t = 0
    path = os.path.join(tmp_path, "model.pickle")
    a.save_progress(path, train_step=11, valid_step=4)
    with open(path, "rb") as f:
        data = pickle.load(f)  # our own file
    # the reference's four keys (chem_tensorflow.py:800-806) plus the integer Adam step
    assert set(data) == {"params", "weights", "train_step", "valid_step", "adam_step"}
    assert data["params"]["hidden_size"] == 64
    assert "graph_model/Variable/Adam:0" in data["weights"] and "beta1_power:0" in data["weights"]
    logs = []
    assert K.restore_progress(b, path, log=logs.append) == (11, 4)
    for n, t in K.variable_names(a).items():
        assert torch.equal(t, K.variable_names(b)[n]), n
    assert all(torch.all(m == 0.25) for m in b.optimizer.m) and b.optimizer.t == 7
    assert not logs


def test_checkpoint_restore_tolerates_missing_and_reports_unused(tmp_path):
    a = _cpu_model(0)
    path = os.path.join(tmp_path, "m.pickle")
    a.save_progress(path, 1, 2)
    with open(path, "rb") as f:
        data = pickle.load(f)
    del data["weights"]["graph_model/word_embedding:0"]
    data["weights"]["graph_model/att_weights_extra:0"] = np.zeros(3, np.float32)
    with open(path, "wb") as f:
        pickle.dump(data, f)
    b = _cpu_model(5)
    before = b.weights["word_embeddings"].detach().clone()
    logs = []
    K.restore_progress(b, path, log=logs.append)
    assert torch.equal(b.weights["word_embeddings"], before)
    assert any("Freshly initializing graph_model/word_embedding:0" in s for s in logs)
    assert any("att_weights_extra" in s for s in logs)
    data["weights"]["graph_model/Variable:0"] = np.zeros((2, 2), np.float32)
    with open(path, "wb") as f:
        pickle.dump(data, f)
    with pytest.raises(ValueError):
        K.restore_progress(b, path, log=logs.append)


def test_adam_step_count_survives_float32_underflow():
    """checkpoint._adam_step_count: the stored integer wins; without it the
    float32 beta2 power (0.999**t) recovers t long after 0.9**t has underflowed."""
    from types import SimpleNamespace
    from ggnn_amd.checkpoint import _adam_step_count
    opt = SimpleNamespace(b1=0.9, b2=0.999)
    for t in (1, 25, 983, 1000, 5000, 40000):
        w = {"beta1_power:0": np.float32(0.9 ** t), "beta2_power:0": np.float32(0.999 ** t)}
        assert _adam_step_count({"weights": w}, opt) == t, t
        assert _adam_step_count({"weights": w, "adam_step": t}, opt) == t
    assert _adam_step_count({"weights": {}}, opt) is None


def _adj_mat_to_target_loop(adj_mat, is_probability=False):
    """The per-node loop of chem_tensorflow_dense.py:106-131, restated as is."""
    a = np.asarray(adj_mat)
    ne, nv, no = a.shape
    g = []
    for node in range(1, nv):
        sl = a[:, node, :]
        mx = np.amax(sl)
        if mx == 0:
            continue
        hits = np.flatnonzero(sl.reshape(-1) == (mx if is_probability else 1))
        if hits.size == 0:
            continue
        e, src = divmod(int(hits[0]), no)
        g.append([src, e + 1])
    return g


def test_adj_mat_to_target_vectorised_matches_loop():
    """The vectorised adj_mat_to_target against the reference's per-node loop:
    0/1 targets, probabilities with ties and zeros, negatives, NaN rows."""
    from ggnn_amd import evaluation as E
    rng = np.random.default_rng(0)
    for trial in range(600):
        ne, nv, no = int(rng.integers(1, 5)), int(rng.integers(1, 12)), int(rng.integers(1, 12))
        kind = trial % 4
        if kind == 0:
            a = (rng.random((ne, nv, no)) < 0.1).astype(np.float32)
        elif kind == 1:
            a = (rng.random((ne, nv, no)) * (rng.random((ne, nv, no)) < 0.5)).astype(np.float32)
        elif kind == 2:
            a = rng.integers(0, 3, (ne, nv, no)).astype(np.float32)
            a[rng.random(a.shape) < 0.05] = -1
        else:
            a = np.round(rng.random((ne, nv, no)), 1).astype(np.float32)
        if trial % 50 == 0:
            a[0, min(1, nv - 1), 0] = np.nan
        for p in (False, True):
            assert E.adj_mat_to_target(a, p) == _adj_mat_to_target_loop(a, p), (trial, p)


def test_las_uas_equal_the_reference_on_real_dev_batches():
    """Host LAS/UAS (evaluation.py) against fixtures written by the
    reference's OWN adj_mat_to_target, get_las_uas and
    humanize_batch_results_btb (chem_tensorflow_dense.py:106-131, 1160-1215,
    1304-1319; tests/golden/make_golden.py) on real WSJ dev batches with
    seeded head / label probabilities (ties included): bit-exact, per batch
    and per graph."""
    import json
    here = os.path.join(os.path.dirname(__file__), "golden")
    ev = np.load(os.path.join(here, "eval_golden.npz"))
    g = np.load(os.path.join(here, "batching_golden.npz"))
    o, oe = int(ev["output_size"]), int(ev["output_size_edges"])
    for k in range(int(ev["n_batches"])):
        pre = "b%d_" % k
        bi = int(ev[pre + "batch"])
        b, v = (int(x) for x in g["eval%d_scalars" % bi][:2])
        lv = np.float32(int(ev[pre + "levels"]))
        cv = ev[pre + "probs_head"].astype(np.float32) / lv
        cv_e = ev[pre + "probs_edges"].astype(np.float32) / lv
        labels, labels_e = g["eval%d_target_values_head" % bi], g["eval%d_target_values_edges" % bi]
        mask, mask_e = g["eval%d_node_mask" % bi], g["eval%d_node_mask_edges" % bi]
        got = E.batch_las_uas(labels, cv, v, mask, labels_e, cv_e, mask_e, o, oe)
        assert tuple(got) == tuple(ev[pre + "las_uas_uase"]), (k, got, ev[pre + "las_uas_uase"])
        _, res, tgt = E.results_reshaped_btb(labels, cv, mask, v, o, oe)
        _, res_e, tgt_e = E.results_reshaped_btb(labels_e, cv_e, mask_e, v, o, oe, is_edge=True)
        for i, ref in enumerate(json.loads(str(ev[pre + "graphs"]))):
            tg = E.merge_head_and_edge_graph(E.adj_mat_to_target(tgt[i]), E.adj_mat_to_target(tgt_e[i]))
            rg_e = E.adj_mat_to_target(res_e[i], is_probability=True)
            rg = E.merge_head_and_edge_graph(E.adj_mat_to_target(res[i], is_probability=True), rg_e)
            assert tg == ref["target"] and rg == ref["result"] and rg_e == ref["result_e"], (k, i)
            assert E.get_las_uas(tg, rg) == (ref["las"], ref["uas"])
    assert int(ev["n_batches"]) >= 6


def test_batch_las_uas_vectorised_matches_lists():
    """The vectorised batch scoring against the reference's per-graph list
    path on random batches with ties, all-zero probability rows (skipped
    nodes: lists shift by position) and padded nodes -- exact equality."""
    rng = np.random.default_rng(5)
    for trial in range(300):
        b, v, o, e = int(rng.integers(1, 6)), int(rng.integers(2, 12)), 12, int(rng.integers(1, 5))
        o = max(o, v)
        heads = np.zeros((b, v, o), np.float32)
        labs = np.zeros((b, v, e), np.float32)
        mask = np.zeros((b, v, o), np.float32)
        mask_e = np.zeros((b, v, e), np.float32)
        for g in range(b):
            n = int(rng.integers(1, v + 1))
            for node in range(1, n):
                heads[g, node, rng.integers(0, n)] = 1
                labs[g, node, rng.integers(0, e)] = 1
            mask[g, :n, :n] = 1
            mask_e[g, :n, :] = 1
        lv = [2, 5, 255][trial % 3]
        ph = (rng.integers(0, lv + 1, heads.shape) / lv).astype(np.float32)
        pe = (rng.integers(0, lv + 1, labs.shape) / lv).astype(np.float32)
        if trial % 4 == 0:                     # some real nodes with an all-zero row
            ph[rng.random((b, v)) < 0.2] = 0
        if trial % 5 == 0:
            pe[rng.random((b, v)) < 0.2] = 0
        args = (heads.reshape(b, -1), ph.reshape(b, -1), v, mask.reshape(b, -1), labs.reshape(b, -1),
                pe.reshape(b, -1), mask_e.reshape(b, -1), o, e)
        _, res, tgt = E.results_reshaped_btb(args[0], args[1], args[3], v, o, e)
        _, res_e, tgt_e = E.results_reshaped_btb(args[4], args[5], args[6], v, o, e, is_edge=True)
        try:
            ref = E._batch_las_uas_lists(res, tgt, res_e, tgt_e)
        except ZeroDivisionError:
            with pytest.raises(ZeroDivisionError):
                E.batch_las_uas(*args)
            continue
        assert E.batch_las_uas(*args) == ref, trial
