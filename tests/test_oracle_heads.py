"""CPU checks of the oracle's front-end / heads restatement
and of the C-ABI argument validation of the new entry points (no GPU needed).

The reference computes these with TensorFlow (absent here): the oracle follows
chem_tensorflow_dense.py:264-306 (front-end), :439-516 + utils.py:40-84 (heads)
and chem_tensorflow.py:349-403 (btb loss).  Pinned by finite differences and
hand-checkable cases; TF outputs themselves are parity-unpinned.
"""
import ctypes

import numpy as np
import pytest

from oracle import ggnn_oracle as O


def _setup(seed=0, b=2, v=5, hd=8, o=(7, 3)):
    rng = np.random.default_rng(seed)
    hT = rng.normal(size=(b, v, hd))
    h0 = rng.normal(size=(b, v, hd))
    heads = []
    for oo in o:
        y = np.zeros((b, v, oo))
        y[np.arange(b)[:, None], np.arange(v)[None, :], rng.integers(0, oo, size=(b, v))] = 1.0
        y[:, -1] = 0.0                       # a padded node: no target
        heads.append(dict(W=rng.normal(size=(2 * hd, oo)) * 0.3, b=rng.normal(size=oo) * 0.1, labels=y))
    return hT, h0, heads


def test_heads_known_answer():
    """One node, hd=1, o=2: z = [hT, h0] @ W + b by hand."""
    hT, h0 = np.array([[[0.5]]]), np.array([[[-1.0]]])
    W, b = np.array([[1.0, -2.0], [0.5, 0.25]]), np.array([0.1, 0.0])
    y = np.array([[[0.0, 1.0]]])
    z = np.array([0.5 * 1.0 - 1.0 * 0.5 + 0.1, 0.5 * -2.0 - 1.0 * 0.25])
    p = np.exp(z) / np.exp(z).sum()
    probs, loss = O.heads_forward(hT, h0, [dict(W=W, b=b, labels=y)], target_num=2.0)
    np.testing.assert_allclose(probs[0][0, 0], p, rtol=1e-12)
    assert abs(loss[0] - (-np.log(p[1]) / 2.0)) < 1e-12


@pytest.mark.parametrize("keep", [1.0, 0.7])
def test_heads_backward_finite_differences(keep):
    hT, h0, heads = _setup()
    tn = 9.0 + O.SMALL_NUMBER

    def L(hT_, h0_, hs):
        return sum(O.heads_forward(hT_, h0_, hs, keep=keep, seed=5, target_num=tn)[1])

    probs, _ = O.heads_forward(hT, h0, heads, keep=keep, seed=5, target_num=tn)
    dWs, dbs, dhT, dh0 = O.heads_backward(hT, h0, heads, probs, keep=keep, seed=5, target_num=tn)
    eps = 1e-6
    rng = np.random.default_rng(1)
    for _ in range(6):
        i = rng.integers(0, 2)
        r, c = rng.integers(0, heads[i]["W"].shape[0]), rng.integers(0, heads[i]["W"].shape[1])
        hp = [dict(h) for h in heads]
        hp[i]["W"] = heads[i]["W"].copy(); hp[i]["W"][r, c] += eps
        hm = [dict(h) for h in heads]
        hm[i]["W"] = heads[i]["W"].copy(); hm[i]["W"][r, c] -= eps
        assert abs((L(hT, h0, hp) - L(hT, h0, hm)) / (2 * eps) - dWs[i][r, c]) < 1e-6
        hp = [dict(h) for h in heads]
        hp[i]["b"] = heads[i]["b"].copy(); hp[i]["b"][c] += eps
        hm = [dict(h) for h in heads]
        hm[i]["b"] = heads[i]["b"].copy(); hm[i]["b"][c] -= eps
        assert abs((L(hT, h0, hp) - L(hT, h0, hm)) / (2 * eps) - dbs[i][c]) < 1e-6
    for arr, g in ((hT, dhT), (h0, dh0)):
        for _ in range(4):
            idx = tuple(rng.integers(0, s) for s in arr.shape)
            a = arr.copy(); a[idx] += eps
            m = arr.copy(); m[idx] -= eps
            fd = ((L(a, h0, heads) - L(m, h0, heads)) if arr is hT else (L(hT, a, heads) - L(hT, m, heads))) / (2 * eps)
            assert abs(fd - g[idx]) < 1e-6


def test_embed_forward_layout_and_pad():
    """btb concat: loc (col 0), pos (1), word (2), loc again (3), zero pad."""
    rng = np.random.default_rng(0)
    loc, pos, word = rng.normal(size=(6, 3)), rng.normal(size=(4, 2)), rng.normal(size=(9, 4))
    wi = np.array([[[0, 1, 2, 3, 0, 0], [5, 3, 8, 0, 1, 1]]])
    h0 = O.embed_forward([(loc, 0), (pos, 1), (word, 2), (loc, 3)], wi, 16)
    np.testing.assert_array_equal(h0[0, 1, :3], loc[5])
    np.testing.assert_array_equal(h0[0, 1, 3:5], pos[3])
    np.testing.assert_array_equal(h0[0, 1, 5:9], word[8])
    np.testing.assert_array_equal(h0[0, 1, 9:12], loc[0])
    assert not h0[:, :, 12:].any()
    with pytest.raises(ValueError, match="non-negative"):
        O.embed_forward([(loc, 0), (pos, 1), (word, 2), (loc, 3)], wi, 11)


@pytest.mark.parametrize("keep", [1.0, 0.6])
def test_embed_backward_is_the_adjoint(keep):
    """<embed(T), G> is linear in the tables: its gradient is embed_backward(G);
    the lookup norm sums squares per lookup row (duplicates not merged)."""
    rng = np.random.default_rng(2)
    loc, pos = rng.normal(size=(5, 3)), rng.normal(size=(4, 2))
    segs = [(loc, 0), (pos, 1), (loc, 2)]
    wi = rng.integers(0, 4, size=(2, 6, 3))
    G = rng.normal(size=(2, 6, 10))
    dts, sq = O.embed_backward(segs, wi, 10, G, keep=keep, seed=11)
    eps = 1e-6
    for ti, tab in enumerate((loc, pos)):
        for _ in range(5):
            idx = tuple(rng.integers(0, s) for s in tab.shape)
            tp, tm = tab.copy(), tab.copy()
            tp[idx] += eps
            tm[idx] -= eps
            mk = lambda t: [(t, 0), (pos, 1), (t, 2)] if ti == 0 else [(loc, 0), (t, 1), (loc, 2)]
            fd = (np.sum(O.embed_forward(mk(tp), wi, 10, keep, 11) * G)
                  - np.sum(O.embed_forward(mk(tm), wi, 10, keep, 11) * G)) / (2 * eps)
            got = dts[0][idx] + dts[2][idx] if ti == 0 else dts[1][idx]
            assert abs(fd - got) < 1e-6
    g = G.copy()
    if keep < 1:
        mask = O.emb_keep_mask(12, 10, keep, 11).reshape(2, 6, 10)
        g = np.where(mask, g / np.float64(np.float32(keep)), 0.0)
    assert abs(sq[1] - np.sum(g[:, :, 3:5] ** 2)) < 1e-9


def test_dropout_masks_of_the_callers_are_independent_streams():
    e = O.emb_keep_mask(64, 32, 0.5, 7)
    h = O.head_keep_mask(64, 32, 0, 0.5, 7)
    h1 = O.head_keep_mask(64, 32, 1, 0.5, 7)
    for m in (e, h, h1):
        assert 0.4 < m.mean() < 0.6
    assert (e != h).mean() > 0.3 and (h != h1).mean() > 0.3


def test_callers_abi_validation_without_gpu(lib):
    """Argument errors are reported before any launch (no GPU needed)."""
    from ggnn_amd import _lib
    from ggnn_amd.heads import EmbedSegment, OutputHead
    d = _lib.dims(2, 4, 16, 1, 1)
    seg = (EmbedSegment * 2)(EmbedSegment(1, 0, 10, 10, 0), EmbedSegment(1, 0, 10, 10, 1))
    rc = lib.ggnn_embed_forward(ctypes.byref(d), seg, 2, ctypes.c_void_p(1), 2, 1.0, 0, ctypes.c_void_p(1), None)
    assert rc == -1 and b"negative pad" in lib.ggnn_last_error()
    rc = lib.ggnn_embed_forward(ctypes.byref(d), seg, 1, ctypes.c_void_p(1), 2, 0.0, 0, ctypes.c_void_p(1), None)
    assert rc == -1 and b"keep" in lib.ggnn_last_error()
    heads = (OutputHead * 1)(OutputHead(1, 1, 5, 0, 0, 0, 0))
    n = ctypes.c_size_t(0)
    assert lib.ggnn_heads_workspace_bytes(ctypes.byref(d), heads, 1, ctypes.byref(n)) == 0
    assert n.value >= (2 * 16 * 5 * 2 + 8 * 5) * 4
    rc = lib.ggnn_heads_forward(ctypes.byref(d), heads, 1, None, None, 1.0, 0, 1.0, None, None, None)
    assert rc == -1 and b"NULL" in lib.ggnn_last_error()
    assert lib.ggnn_heads_forward(ctypes.byref(d), heads, 5, None, None, 1.0, 0, 1.0, None, None, None) == -1
