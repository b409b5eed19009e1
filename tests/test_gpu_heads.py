"""GPU parity of the callers either side of the path:
embedding front-end, output heads + btb loss, and a whole btb training step
of the drop-in model, each against the float64 oracle on the same inputs and
the same Philox masks.  fp32 arithmetic: tolerance 1e-3 (north_star), the
kernels land near 1e-6."""
import json
import os

import numpy as np
import pytest

import ggnn_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-3


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    return torch


def _nmax(x, ref):
    return float(np.abs(np.asarray(x, np.float64) - ref).max() / max(np.abs(ref).max(), 1e-30))


@pytest.mark.parametrize("keep", [1.0, 0.55])
def test_embed_forward_backward_parity(keep):
    torch = _torch()
    from ggnn_amd.heads import EmbeddingFrontEnd
    rng = np.random.default_rng(3)
    b, v, h = 5, 23, 64
    loc = rng.normal(size=(30, 16)).astype(np.float32)
    pos = rng.normal(size=(12, 8)).astype(np.float32)
    word = rng.normal(size=(50, 24)).astype(np.float32)
    wi = np.stack([rng.integers(0, 30, (b, v)), rng.integers(0, 12, (b, v)), rng.integers(0, 50, (b, v)),
                   rng.integers(0, 30, (b, v)), rng.integers(0, 12, (b, v)), rng.integers(0, 5, (b, v))], axis=2)
    segs_np = [(loc, 0), (pos, 1), (word, 2), (loc, 3)]
    dev = torch.device("cuda")
    T = {id(a): torch.from_numpy(a).to(dev) for a in (loc, pos, word)}
    segs = [(T[id(a)], c) for a, c in segs_np]
    wi_t = torch.from_numpy(wi.astype(np.int32)).to(dev)
    fe = EmbeddingFrontEnd(h)
    seed = 0xABCDEF12345
    h0 = fe.forward(segs, wi_t, keep, seed)
    ref = O.embed_forward(segs_np, wi, h, keep, seed)
    assert np.abs(h0.cpu().numpy() - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())
    G = rng.normal(size=(b, v, h)).astype(np.float32)
    G2 = rng.normal(size=(b, v, h)).astype(np.float32)
    shared = torch.empty_like(T[id(loc)])
    dts, sq = fe.backward(segs, wi_t, torch.from_numpy(G).to(dev), keep, seed, dh0_add=torch.from_numpy(G2).to(dev),
                          dtables=[shared, torch.empty_like(T[id(pos)]), torch.empty_like(T[id(word)]), shared])
    rd, rsq = O.embed_backward(segs_np, wi, h, G.astype(np.float64) + G2, keep, seed)
    assert _nmax(dts[0].cpu().numpy(), rd[0] + rd[3]) <= 1e-5
    assert _nmax(dts[1].cpu().numpy(), rd[1]) <= 1e-5
    assert _nmax(dts[2].cpu().numpy(), rd[2]) <= 1e-5
    # one squared lookup norm per TABLE, in its first segment's slot: loc's two
    # lookups (columns 0 and 3) share one gradient, as the reference's two
    # IndexedSlices of one variable are concatenated into one
    np.testing.assert_allclose(sq.cpu().numpy(), [rsq[0] + rsq[3], rsq[1], rsq[2], 0.0], rtol=1e-5)


@pytest.mark.parametrize("b,v,h,os_,keep", [(4, 20, 64, (150, 12), 1.0), (3, 37, 128, (150, 46), 0.85),
                                            (2, 128, 256, (150, 46), 0.85)])
def test_heads_forward_backward_parity(b, v, h, os_, keep):
    torch = _torch()
    from ggnn_amd.heads import OutputHeads
    rng = np.random.default_rng(b * v)
    dev = torch.device("cuda")
    hT = rng.uniform(-1, 1, (b, v, h)).astype(np.float32)
    h0 = rng.uniform(-0.5, 0.5, (b, v, h)).astype(np.float32)
    heads_np, heads_t, labels = [], [], []
    for o in os_:
        W = (np.sqrt(6.0 / (2 * h + o)) * (2 * rng.random((2 * h, o)) - 1)).astype(np.float32)
        bb = rng.normal(size=o).astype(np.float32) * 0.1
        y = np.zeros((b, v, o), np.float32)
        y[np.arange(b)[:, None], np.arange(v)[None, :], rng.integers(0, min(o, v), (b, v))] = 1
        y[:, v - 3:] = 0                                    # padded nodes
        heads_np.append(dict(W=W, b=bb, labels=y))
        heads_t.append((torch.from_numpy(W).to(dev), torch.from_numpy(bb).to(dev)))
        labels.append(torch.from_numpy(y).to(dev))
    tn = float(b) + O.SMALL_NUMBER
    seed = 99
    oh = OutputHeads(h)
    hT_t, h0_t = torch.from_numpy(hT).to(dev), torch.from_numpy(h0).to(dev)
    probs, loss = oh.forward(hT_t, h0_t, heads_t, labels, keep, seed, tn)
    rp, rl = O.heads_forward(hT, h0, heads_np, keep, seed, tn)
    for i in range(len(os_)):
        assert np.abs(probs[i].cpu().numpy() - rp[i]).max() <= 1e-5
        assert abs(float(loss[i]) - rl[i]) <= 1e-5 * abs(rl[i]) + 1e-6
    dws, dbs, dhT, dh0 = oh.backward(hT_t, h0_t, heads_t, labels, probs, tn)
    rw, rb, rhT, rh0 = O.heads_backward(hT, h0, heads_np, [p.cpu().numpy() for p in probs], keep, seed, tn)
    for i in range(len(os_)):
        assert _nmax(dws[i].cpu().numpy(), rw[i]) <= 1e-5
        assert _nmax(dbs[i].cpu().numpy(), rb[i]) <= 1e-5
    assert _nmax(dhT.cpu().numpy(), rhT) <= 1e-5
    assert _nmax(dh0.cpu().numpy(), rh0) <= 1e-5


def _dev_model(torch, keep_all, hidden=128, batch_size=6, emb=None, big_batch=False):
    from ggnn_amd.model import DenseGGNNChemModel
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)
    params = {"hidden_size": hidden, "num_timesteps": 2, "batch_size": batch_size, "learning_rate": 0.003}
    if keep_all:
        params.update(graph_state_dropout_keep_prob=1.0, emb_dropout_keep_prob=1.0, out_layer_dropout_keep_prob=1.0)
    m = DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                           output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                           bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                           embedding_sizes=emb or dict(loc=16, pos=8, word=16, edge=8))
    if big_batch:
        # one full batch of real dev sentences: the sentences of the most
        # populated bucket, repeated until batch_size graphs share that bucket
        sizes = m.get_bucket_sizes()
        bucket = [int(np.argmax(sizes > max(max(e[0], e[2]) for e in d["graph"]))) for d in data]
        top = max(set(bucket), key=bucket.count)
        pool = [d for d, k in zip(data, bucket) if k == top]
        data = [pool[i % len(pool)] for i in range(batch_size)]
        feeds = list(m.make_minibatch_iterator(m.process_raw_graphs(data, True), True))
        assert feeds[0]["num_graphs"] == batch_size
        return m, feeds
    feeds = list(m.make_minibatch_iterator(m.process_raw_graphs(data[:30], True), True))
    return m, feeds


def _check_train_step(m, fd):
    """One whole btb training step of the drop-in model against the oracle
    composed the same way, including the IndexedSlices clip norm of the
    embeddings and every dropout mask (replayed from the seeds the model
    drew)."""
    params = m.trainable_variables()
    before = [p.detach().cpu().numpy().astype(np.float64) for p in params]
    loss = m.train_step(fd)
    after = [p.detach().cpu().numpy() for p in params]
    # ---- oracle
    W = m.weights
    nm = {id(p): i for i, p in enumerate(params)}
    P = lambda t: before[nm[id(t)]]
    h = m.params["hidden_size"]
    wi = np.asarray(fd["word_inputs"]).astype(np.int64)
    segs = [(P(W["loc_embeddings"]), 0), (P(W["pos_embeddings"]), 1), (P(W["word_embeddings"]), 2),
            (P(W["loc_embeddings"]), 3)]
    e = m.last_embed
    h0 = O.embed_forward(segs, wi, h, e["keep"], e["seed"])
    w64 = {"edge_weights": P(W["edge_weights"]), "edge_biases": P(W["edge_biases"])}
    w64.update({k: P(t) for k, t in W["node_gru"].items()})
    A = np.asarray(fd["adjacency_matrix"], np.float64)
    dr = m.last_dropout
    hT, caches = O.forward(A, h0, w64, m.params["num_timesteps"],
                           dropout=dict(edge_keep=dr["edge_keep"], state_keep=dr["state_keep"], seed=dr["seed"]))
    b, v = fd["num_graphs"], fd["num_vertices"]
    o, oe = m.params["output_size"], m.output_size_edges
    g0, ge = W["regression_gate_task0"], W["regression_gate_task_edges0"]
    heads = [dict(W=P(g0["weights"][0]), b=P(g0["biases"][0]),
                  labels=np.asarray(fd["target_values_head"], np.float64).reshape(b, v, o)),
             dict(W=P(ge["weights"][0]), b=P(ge["biases"][0]),
                  labels=np.asarray(fd["target_values_edges"], np.float64).reshape(b, v, oe))]
    hd = m.last_heads
    probs, losses = O.heads_forward(hT, h0, heads, hd["keep"], hd["seed"], hd["target_num"])
    assert abs(float(loss.detach()) - sum(losses)) <= TOL * abs(sum(losses))
    dWs, dbs, dhT, dh0_heads = O.heads_backward(hT, h0, heads, probs, hd["keep"], hd["seed"], hd["target_num"])
    gp = O.backward(A, dhT, caches, w64)
    dts, sq = O.embed_backward(segs, wi, h, dh0_heads + gp["h0"], e["keep"], e["seed"])
    grads = [gp["edge_weights"], gp["edge_biases"]] + [gp[k] for k in ("gates_kernel", "gates_bias", "candidate_kernel",
                                                                      "candidate_bias")]
    grads += [dts[0] + dts[3], dts[1], dts[2], dWs[0], dbs[0], dWs[1], dbs[1]]
    sqn = [None] * 6 + [sq[0] + sq[3], sq[1], sq[2]] + [None] * 4
    # TF1 Adam step 1 with clip_by_norm (IndexedSlices norm for the tables)
    lr, clip = m.params["learning_rate"], m.params["clamp_gradient_norm"]
    lr_t = lr * np.sqrt(1 - 0.999) / (1 - 0.9)
    for i, (p0, g) in enumerate(zip(before, grads)):
        assert _nmax(params[i].grad.cpu().numpy(), g) <= TOL, (i, _nmax(params[i].grad.cpu().numpy(), g))
        if sqn[i] is not None:
            got = m.lookup_sqnorm[id(params[i])]
            assert abs(float(got) - sqn[i]) <= 1e-4 * sqn[i], i
        n = np.sqrt(sqn[i]) if sqn[i] is not None else np.sqrt(np.sum(g * g))
        gc = g * clip / max(n, clip)
        mm, vv = 0.1 * gc, 0.001 * gc * gc
        ref = p0 - lr_t * mm / (np.sqrt(vv) + 1e-8)
        # Adam's first step is ~lr * sign(g): compare it where the gradient is
        # not at rounding level (there a 1e-6 error may flip the sign)
        sig = np.abs(gc) > 1e-3 * max(np.abs(gc).max(), 1e-30)
        assert np.abs(after[i] - ref)[sig].max(initial=0.0) <= lr * 1e-2, i
        assert np.abs(after[i] - ref).max() <= 2.01 * lr, i
    return gp


@pytest.mark.parametrize("dropout", [False, True])
def test_model_train_step_matches_oracle(dropout):
    """One whole btb training step of the drop-in model on real dev batches
    (front-end -> propagation -> heads -> loss -> backward -> clip + Adam)
    against the oracle."""
    torch = _torch()
    m, feeds = _dev_model(torch, keep_all=not dropout)
    fd = feeds[0]
    if dropout:
        fd = dict(fd, edge_weight_dropout_keep_prob=0.9, graph_state_keep_prob=0.9)
    _check_train_step(m, fd)


def test_model_train_step_full_batch_hidden256():
    """The same whole training step at a real batch size: 64 WSJ dev graphs in
    one bucket, hidden 256, C = 92 channels, the training feed's dropouts.  The
    loss is divided by ~64 * n targets, so dL/dh_T is at the btb loss's real
    magnitude (chem_tensorflow.py:360,399-403), where the backward's gradient
    scale matters."""
    torch = _torch()
    m, feeds = _dev_model(torch, keep_all=False, hidden=256, batch_size=64,
                          emb=dict(loc=64, pos=32, word=96, edge=32), big_batch=True)
    fd = feeds[0]
    gp = _check_train_step(m, fd)
    assert np.abs(gp["h0"]).max() < 2.0 ** -5   # at the loss scale (~1/b), not O(1)


def test_model_trains_on_dev_batches():
    """Loss goes down over a few steps on real dev batches (sanity of the
    whole btb training loop on the GPU)."""
    torch = _torch()
    m, feeds = _dev_model(torch, keep_all=True)
    fd = feeds[0]
    losses = [float(m.train_step(fd).detach()) for _ in range(8)]
    assert np.isfinite(losses).all()
    assert losses[-1] < 0.9 * losses[0]


@pytest.mark.gpu
def test_evaluate_batch_las_uas_and_checkpoint_resume(tmp_path):
    """Host LAS/UAS of the drop-in model on real dev batches
    (chem_tensorflow_dense.py:1160-1215) improves when the model fits a batch,
    and a checkpoint written mid-training resumes to the same next step
    (chem_tensorflow.py:796-855)."""
    torch = _torch()
    m, feeds = _dev_model(torch, keep_all=True)
    fd = feeds[0]
    las0, uas0, le0 = m.evaluate_batch(fd)
    assert 0.0 <= las0 <= uas0 <= 1.0 and 0.0 <= le0 <= 1.0
    for _ in range(25):
        m.train_step(fd)
    las1, uas1, le1 = m.evaluate_batch(fd)
    assert uas1 > uas0 and las1 >= las0
    path = str(tmp_path / "model.pickle")
    m.save_progress(path, train_step=25, valid_step=0)
    m2, _ = _dev_model(torch, keep_all=True)   # fresh model: no optimizer yet, restore creates it
    assert m2.optimizer is None
    assert m2.restore_progress(path) == (25, 0)
    assert m2.optimizer is not None and m2.optimizer.t == m.optimizer.t == 25
    for _ in range(2):  # the second loss sees one Adam update from the restored state
        l_a = float(m.train_step(fd).detach())
        l_b = float(m2.train_step(fd).detach())
        assert abs(l_a - l_b) <= 1e-5 * max(1.0, abs(l_a))


def test_checkpoint_restores_adam_step_past_float32_underflow(tmp_path):
    """beta1_power = 0.9**t underflows float32 near t = 1000; the Adam step
    count must survive a save/restore well past it (checkpoint.py)."""
    torch = _torch()
    m, feeds = _dev_model(torch, keep_all=True)
    m.train_step(feeds[0])
    m.optimizer.t = 4321
    path = str(tmp_path / "late.pickle")
    m.save_progress(path, train_step=4321, valid_step=7)
    m2, _ = _dev_model(torch, keep_all=True)
    assert m2.restore_progress(path) == (4321, 7)
    assert m2.optimizer.t == 4321
    for a, b in zip(m.optimizer.m, m2.optimizer.m):
        assert torch.equal(a, b)


def test_run_epoch_end_to_end_reference_defaults():
    """run_epoch (chem_tensorflow.py:528-667) with the reference's default
    params (hidden_size 400, num_timesteps 4, batch_size 20, the 80/50/100/80
    embedding widths, output_size 150 -- config 1's model; hidden 400 runs the
    general path) on a synthetic treebank: the reference's return tuple, the
    training loss falls over epochs, LAS/UAS are fractions, instances/sec > 0."""
    _torch()
    from ggnn_amd.batching import synthetic_treebank
    from ggnn_amd.model import DenseGGNNChemModel
    raw = synthetic_treebank(120, seed=1, max_nodes=60)
    m = DenseGGNNChemModel(num_edge_types=46, output_size_edges=12, pos_size=46, vocab_size=39549,
                           params={"compact_adjacency": True}, seed=0)
    assert m.params["hidden_size"] == 400 and m.params["num_timesteps"] == 4 and m.params["batch_size"] == 20
    train = m.process_raw_graphs(raw[:100], True)
    valid = m.process_raw_graphs(raw[100:], False)
    losses = []
    for epoch in range(3):
        r = m.run_epoch("epoch %d (train)" % epoch, train, True)
        assert len(r) == 17
        loss, acc, err, ips, steps, las, uas = r[:7]
        assert np.isfinite(loss) and ips > 0 and steps >= 5 and 0 <= las <= uas <= 1
        assert np.allclose(acc, [loss]) and np.allclose(err, acc / m.CHEMICAL_ACCURACIES[0])
        losses.append(loss)
    assert losses[-1] < losses[0]
    v = m.run_epoch("valid", valid, False)
    assert np.isfinite(v[0]) and 0 <= v[5] <= v[6] <= 1 and 0 <= v[16] <= 1
    assert sum(x.shape[0] for x in v[8]) == 20      # all_computed_values cover the split


def test_run_epoch_train_with_dev_restrict_100():
    """run_epoch on the reference's OWN sentences in its --train_with_dev mode
    (chem_tensorflow.py:36-45: train = std dev, valid = std test) with
    --restrict_data 100 (:248-255; the README's sample run) and the
    reference's default params: the training loss falls over three epochs and
    the scores are fractions."""
    _torch()
    from ggnn_amd.batching import TRAIN_WITH_DEV, wsj_model_sizes
    from ggnn_amd.model import DenseGGNNChemModel
    np.random.seed(0)
    m = DenseGGNNChemModel(params={"compact_adjacency": True}, seed=0, **wsj_model_sizes())
    assert m.num_channels == 92 and m.output_size_edges == 12 and m.bucket_max_nodes == 120
    train = m.load_data(TRAIN_WITH_DEV["train_file"], True, restrict=100)
    valid = m.load_data(TRAIN_WITH_DEV["valid_file"], False, restrict=100)
    losses = []
    for epoch in range(3):
        r = m.run_epoch("epoch %d" % epoch, train, True)
        assert np.isfinite(r[0]) and 0 <= r[5] <= r[6] <= 1
        losses.append(r[0])
    assert losses[-1] < losses[0]
    va = m.run_epoch("valid", valid, False)
    assert np.isfinite(va[0]) and 0 <= va[5] <= va[6] <= 1 and 0 <= va[16] <= 1
    assert sum(x.shape[0] for x in va[8]) == 100
