"""Bit-reproducible training (round 5).

Every cross-workgroup reduction of the library is order-fixed: the weight
gradients' split-K partials are stored to slabs and summed in z order
(k_wgrad_reduce, k_slab_reduce), the bias gradients' partial rows in row
order (k_sum_rows), and the embedding tables accumulate in 64-bit fixed
point, whose integer sums do not depend on the order the additions land in
(ggnn_embed_backward_ws).  So two identical models fed the same batches
reach the same bits after any number of steps -- through Adam at the
reference's epsilon 1e-8 (chem_tensorflow.py:494), where g / (sqrt(v) + eps)
would otherwise turn last-bit differences of near-zero gradients into
O(learning rate) weight differences (round 4's 4.0e-5 drift in 3 steps).
"""
import json
import os

import numpy as np
import pytest

import ggnn_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    return torch


def _golden_model(hidden, compact, graphs=False, T=3):
    from ggnn_amd.model import DenseGGNNChemModel
    g = np.load(os.path.join(ROOT, "tests", "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)
    params = {"hidden_size": hidden, "num_timesteps": T, "batch_size": 8, "compact_adjacency": compact,
              "hip_graphs": graphs}
    m = DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                           output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                           bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                           embedding_sizes=dict(loc=16, pos=8, word=16, edge=8), seed=5)
    return m, data


@pytest.mark.parametrize("hidden,compact", [
    (128, False),   # the specialised path (k_wgrad, k_gru_bwd) from the dense feed
    (128, True),    # the same from edge lists
    (400, True),    # the general path in pair mode (the reference's hidden size)
    (400, False),   # the general path's dense (graph, channel) tiles
])
def test_two_identical_models_stay_bit_identical(hidden, compact):
    """Two btb models, same seed, same three training batches (the
    reference's training-feed dropout on, Adam epsilon 1e-8): every variable,
    every Adam slot and the flat gradient buffer equal bit for bit after each
    step."""
    torch = _torch()
    m1, data = _golden_model(hidden, compact)
    m2, _ = _golden_model(hidden, compact)
    bucketed, sizes, _ = m1.process_raw_graphs(data, True)
    bidx = max(bucketed, key=lambda k: len(bucketed[k]))
    feed = m1._make_feed(bucketed[bidx][:6], int(sizes[bidx]), True)
    for step in range(3):
        l1 = float(m1.train_step(dict(feed)))
        l2 = float(m2.train_step(dict(feed)))
        torch.cuda.synchronize()
        assert m1.optimizer.eps == 1e-8 and m2.optimizer.eps == 1e-8
        assert l1 == l2, (step, l1, l2)
        assert torch.equal(m1.train_buffer().flat, m2.train_buffer().flat), step
        for a, b in zip(m1.trainable_variables(), m2.trainable_variables()):
            assert torch.equal(a.detach(), b.detach()), step
        for a, b in zip(m1.optimizer.m + m1.optimizer.v, m2.optimizer.m + m2.optimizer.v):
            assert torch.equal(a, b), step


@pytest.mark.parametrize("sparse,generic,keep", [
    ("auto", False, 0.9),   # pair mode (hidden 400: the general path), edge + state dropout
    (False, True, 1.0),     # dense tiles, dW over chunks of each channel's graphs (slabs)
    (False, True, 0.8),     # the same under edge dropout (per-timestep GW)
])
def test_general_path_backward_is_deterministic(sparse, generic, keep):
    """The general path's backward twice on one batch of b = 40 trees (hidden
    400, C = 92): every gradient equal bit for bit (GRU weight gradients and
    dW_c through split-K slabs, pair dW over multi-chunk channels, bias
    partials summed in row order)."""
    torch = _torch()
    from ggnn_amd.engine import PropagationEngine
    b, v, h, T, E = 40, 30, 400, 3, 46
    rng = np.random.default_rng(21)
    pz = 1.0 / np.arange(1, E + 1)
    pz /= pz.sum()
    graphs = []
    for _ in range(b):
        n = int(rng.integers(v // 2, v + 1))
        graphs.append([(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)])
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=8)
    dhT = rng.standard_normal((b, v, h)).astype(np.float32)
    res = []
    for _ in range(2):
        eng = PropagationEngine(h, 2 * E, sparse_pairs=sparse, force_generic=generic)
        dev = eng.device
        wd = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
        eng.set_adjacency_edges(graphs, v, E)
        pack = eng.pack_weights(wd, T=T, edge_keep=keep, seed=99, batch=True)
        eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=True, state_keep=keep)
        g = eng.backward(torch.from_numpy(dhT).to(dev))
        res.append({k: x.cpu().numpy() for k, x in g.items() if x is not None})
        assert eng.sparse == (sparse == "auto")
    for k in res[0]:
        assert np.array_equal(res[0][k], res[1][k]), k


def test_heads_and_embedding_backward_are_deterministic():
    """The heads' dW (split-K slab) and bias (block partial rows) and the
    embedding tables (fixed-point accumulators), twice on inputs with many
    repeated ids: equal bit for bit, and equal to the float64 oracle at the
    fp32 bar; the embedding workspace is zero again after each call."""
    torch = _torch()
    from ggnn_amd.heads import EmbeddingFrontEnd, OutputHeads
    dev = torch.device("cuda")
    rng = np.random.default_rng(5)
    b, v, h = 16, 40, 128
    loc = rng.normal(size=(40, 16)).astype(np.float32)
    word = rng.normal(size=(7, 32)).astype(np.float32)      # 7 ids over 640 lookups: heavy repeats
    wi = np.stack([rng.integers(0, 40, (b, v)), rng.integers(0, 7, (b, v)), rng.integers(0, 40, (b, v))], 2)
    segs_np = [(loc, 0), (word, 1), (loc, 2)]
    T_ = {id(a): torch.from_numpy(a).to(dev) for a in (loc, word)}
    segs = [(T_[id(a)], c) for a, c in segs_np]
    wi_t = torch.from_numpy(wi.astype(np.int32)).to(dev)
    G = torch.from_numpy(rng.normal(size=(b, v, h)).astype(np.float32)).to(dev)
    fe = EmbeddingFrontEnd(h)
    assert fe.deterministic
    outs = []
    for _ in range(2):
        shared = torch.empty_like(T_[id(loc)])
        dts, sq = fe.backward(segs, wi_t, G, 0.7, 1234, dtables=[shared, torch.empty_like(T_[id(word)]), shared])
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in (dts[0], dts[1], sq)])
        ws = fe.workspace(segs, dev)
        assert int(torch.count_nonzero(ws)) == 0
    for a, c in zip(*outs):
        assert np.array_equal(a, c)
    rd, rsq = O.embed_backward(segs_np, wi, h, G.cpu().numpy().astype(np.float64), 0.7, 1234)
    assert np.abs(outs[0][0] - (rd[0] + rd[2])).max() <= 1e-5 * np.abs(rd[0] + rd[2]).max()
    assert np.abs(outs[0][1] - rd[1]).max() <= 1e-5 * np.abs(rd[1]).max()
    assert abs(outs[0][2][0] - rsq[0] - rsq[2]) <= 1e-5 * (rsq[0] + rsq[2]) and outs[0][2][2] == 0
    # heads
    oh = OutputHeads(h)
    mk = lambda *s_: torch.from_numpy(rng.uniform(-0.1, 0.1, s_).astype(np.float32)).to(dev)  # noqa: E731
    hT, h0 = mk(b, v, h), mk(b, v, h)
    heads = [(mk(2 * h, 150), mk(150)), (mk(2 * h, 46), mk(46))]
    labels = []
    for o in (150, 46):
        y = np.zeros((b, v, o), np.float32)
        y[np.arange(b)[:, None], np.arange(v)[None, :], rng.integers(0, o, (b, v))] = 1
        labels.append(torch.from_numpy(y).to(dev))
    got = []
    for _ in range(2):
        probs, _ = oh.forward(hT, h0, heads, labels, 0.85, 3, float(b * v))
        dws, dbs, dhT, dh0 = oh.backward(hT, h0, heads, labels, probs, float(b * v))
        torch.cuda.synchronize()
        got.append([x.cpu().numpy().copy() for x in list(dws) + list(dbs) + [dhT, dh0]])
    for a, c in zip(*got):
        assert np.array_equal(a, c)
