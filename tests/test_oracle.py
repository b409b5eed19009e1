"""Pin the CPU oracle before trusting it:
hand-computed known answers, finite-difference gradients, and agreement of the
reference's two contraction orders (fast vs --old)."""
import numpy as np
import pytest

import ggnn_oracle as O

TANH1 = np.tanh(1.0)


def kat_inputs(beta=None):
    # v=3 nodes, h=2, C=2 channels; row = receiving node
    A = np.zeros((1, 2, 3, 3))
    A[0, 0, 0, 1] = 1      # node 0 <- node 1 on channel 0
    A[0, 0, 1, 2] = 1      # node 1 <- node 2 on channel 0
    A[0, 1, 2, 0] = 1      # node 2 <- node 0 on channel 1
    h0 = np.array([[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]]])
    w = {
        "edge_weights": np.array([[[1.0, 0.0], [0.0, 1.0]], [[0.0, 1.0], [1.0, 0.0]]]),
        "edge_biases": np.zeros((2, 1, 2)) if beta is None else np.asarray(beta, float).reshape(2, 1, 2),
        "gates_kernel": np.zeros((4, 4)),          # r = u = sigmoid(0) = 1/2
        "gates_bias": np.zeros(4),
        "candidate_kernel": np.vstack([np.eye(2), np.zeros((2, 2))]),  # c = tanh(x)
        "candidate_bias": np.zeros(2),
    }
    return A, h0, w


def test_known_answer_no_bias():
    A, h0, w = kat_inputs()
    hT, _ = O.forward(A, h0, w, 1)
    # X = [M0[1], M0[2], M1[0]] = [[0,1],[1,1],[0,1]];  h' = h/2 + tanh(X)/2
    expected = np.array([[[0.5, 0.5 * TANH1], [0.5 * TANH1, 0.5 + 0.5 * TANH1], [0.5, 0.5 + 0.5 * TANH1]]])
    np.testing.assert_allclose(hT, expected, rtol=0, atol=1e-15)


def test_known_answer_edge_bias():
    A, h0, w = kat_inputs(beta=[[0.5, 0.0], [0.0, 0.0]])
    X = O.message_aggregate_fast(A, h0, w["edge_weights"], w["edge_biases"])
    np.testing.assert_allclose(X[0], [[0.5, 1.0], [1.5, 1.0], [0.0, 1.0]], atol=1e-15)
    hT, _ = O.forward(A, h0, w, 1)
    expected = 0.5 * h0 + 0.5 * np.tanh(X)
    np.testing.assert_allclose(hT, expected, atol=1e-15)
    # use_edge_bias=False drops beta
    X0 = O.message_aggregate_fast(A, h0, w["edge_weights"], None)
    np.testing.assert_allclose(X0[0], [[0.0, 1.0], [1.0, 1.0], [0.0, 1.0]], atol=1e-15)


def test_gru_is_reset_before_matmul():
    # with a non-zero candidate h-part, r multiplies h BEFORE the matmul (TF1 GRUCell)
    rng = np.random.default_rng(0)
    x, h = rng.standard_normal((4, 3)), rng.standard_normal((4, 3))
    Wg, bg = rng.standard_normal((6, 6)), rng.standard_normal(6)
    Wc, bc = rng.standard_normal((6, 3)), rng.standard_normal(3)
    hn, (_, _, r, u, c, rh) = O.gru_cell(x, h, Wg, bg, Wc, bc)
    s = 1 / (1 + np.exp(-(np.hstack([x, h]) @ Wg + bg)))
    np.testing.assert_allclose(r, s[:, :3])
    np.testing.assert_allclose(u, s[:, 3:])
    np.testing.assert_allclose(c, np.tanh(np.hstack([x, s[:, :3] * h]) @ Wc + bc))
    np.testing.assert_allclose(hn, u * h + (1 - u) * c)


def test_fast_and_old_orderings_agree():
    A, h0 = O.synthetic_batch(3, 10, 8, 6, seed=2, density=0.3, dtype=np.float64)
    w = {k: v.astype(np.float64) for k, v in O.synthetic_weights(8, 6, seed=2).items()}
    a, _ = O.forward(A, h0, w, 3, ordering="fast")
    b, _ = O.forward(A, h0, w, 3, ordering="old")
    assert np.abs(a - b).max() < 1e-12


@pytest.mark.parametrize("use_bias", [True, False])
def test_backward_matches_finite_differences(use_bias):
    A, h0 = O.synthetic_batch(2, 5, 3, 4, seed=3, density=0.4, dtype=np.float64)
    w = {k: v.astype(np.float64) for k, v in O.synthetic_weights(3, 4, seed=1).items()}
    T = 2
    hT, caches = O.forward(A, h0, w, T, use_edge_bias=use_bias)
    dhT = np.random.default_rng(0).standard_normal(hT.shape)
    g = O.backward(A, dhT, caches, w, use_edge_bias=use_bias)

    def loss(w_, h0_):
        return float((O.forward(A, h0_, w_, T, use_edge_bias=use_bias, keep_cache=False)[0] * dhT).sum())

    eps = 1e-6
    for key in ("h0", "edge_weights", "edge_biases", "gates_kernel", "gates_bias",
                "candidate_kernel", "candidate_bias"):
        base = h0 if key == "h0" else w[key]
        num = np.zeros_like(base)
        for idx in np.ndindex(base.shape):
            p, m = base.copy(), base.copy()
            p[idx] += eps
            m[idx] -= eps
            if key == "h0":
                num[idx] = (loss(w, p) - loss(w, m)) / (2 * eps)
            else:
                num[idx] = (loss({**w, key: p}, h0) - loss({**w, key: m}, h0)) / (2 * eps)
        assert np.abs(num - g[key]).max() <= 1e-7 * max(1.0, np.abs(num).max()), key


def test_adjacency_semantics_match_reference_test_vectors():
    # tests_chem.py:29-48 pins row = dest, col = src for graph [[3,1,1],[3,1,2],[0,2,3]]
    A = O.graph_to_adj_mat_bd([[3, 1, 1], [3, 1, 2], [0, 2, 3]], 4, 2)
    assert A.shape == (4, 4, 4)
    exp_in = np.zeros((2, 4, 4))
    exp_in[0, 1, 3] = exp_in[0, 2, 3] = exp_in[1, 3, 0] = 1
    # incoming channels: label e -> channel e-1, plus the previous-word channel E-1 = 1
    assert A[0, 1, 3] == 1 and A[0, 2, 3] == 1 and A[1, 3, 0] == 1
    assert A[1, 1, 0] == 1 and A[1, 2, 1] == 1 and A[1, 3, 2] == 1      # prev-word edges
    assert A[2, 3, 1] == 1 and A[2, 3, 2] == 1 and A[3, 0, 3] == 1      # outgoing (transposed)
    assert A[3, 0, 1] == 1 and A[3, 1, 2] == 1 and A[3, 2, 3] == 1      # next-word edges
    assert A.sum() == 12


# ---------------------------------------------------------------- dropout
def test_philox_known_answer_vectors():
    """Random123's published Philox4x32-10 known-answer vectors (kat_vectors)."""
    kats = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
            ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
            ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
             (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for ctr, key, exp in kats:
        assert tuple(int(x) for x in O.philox4x32_10(*ctr, key)) == exp


def test_dropout_masks_fresh_per_step_and_seeded():
    m0 = O.edge_keep_mask(4, 64, 0, 0.9, seed=7)
    m1 = O.edge_keep_mask(4, 64, 1, 0.9, seed=7)
    assert m0.shape == (4, 64, 64) and abs(m0.mean() - 0.9) < 0.01
    assert (m0 != m1).mean() > 0.1                               # fresh mask per timestep (:397-403)
    assert np.array_equal(m0, O.edge_keep_mask(4, 64, 0, 0.9, seed=7))
    assert (m0 != O.edge_keep_mask(4, 64, 0, 0.9, seed=8)).mean() > 0.1
    s = O.state_keep_mask(5, 23, 64, 3, 0.5, seed=1)
    assert s.shape == (5, 23, 64) and abs(s.mean() - 0.5) < 0.02
    # a graph's mask does not depend on the batch it sits in (counter = (i>>2, k, g, t))
    assert np.array_equal(O.state_keep_mask(7, 23, 64, 3, 0.5, seed=1)[:5], s)


def test_dropout_forward_semantics():
    """W_t = W * mask_t / keep (edge) and h = GRU(...) * mask_t / keep (state)."""
    A, h0 = O.synthetic_batch(2, 6, 8, 4, seed=2, density=0.4, dtype=np.float64)
    w = {k: v.astype(np.float64) for k, v in O.synthetic_weights(8, 4, seed=1).items()}
    dr = dict(edge_keep=0.75, state_keep=0.6, seed=99)
    hT, _ = O.forward(A, h0, w, 2, dropout=dr)
    h = h0
    for t in range(2):
        em = O.edge_keep_mask(4, 8, t, 0.75, 99)
        X = O.message_aggregate_fast(A, h, w["edge_weights"] * em / 0.75, w["edge_biases"])
        hn, _ = O.gru_cell(X.reshape(-1, 8), h.reshape(-1, 8), w["gates_kernel"], w["gates_bias"],
                           w["candidate_kernel"], w["candidate_bias"])
        h = hn.reshape(h.shape) * O.state_keep_mask(2, 6, 8, t, 0.6, 99) / 0.6
    np.testing.assert_allclose(hT, h, rtol=1e-12, atol=1e-12)


def test_dropout_backward_matches_finite_differences():
    A, h0 = O.synthetic_batch(2, 5, 4, 4, seed=3, density=0.4, dtype=np.float64)
    w = {k: v.astype(np.float64) for k, v in O.synthetic_weights(4, 4, seed=1).items()}
    dr = dict(edge_keep=0.7, state_keep=0.8, seed=12345)
    T = 2
    hT, caches = O.forward(A, h0, w, T, dropout=dr)
    dhT = np.random.default_rng(0).standard_normal(hT.shape)
    g = O.backward(A, dhT, caches, w)

    def loss(w_, h0_):
        return float((O.forward(A, h0_, w_, T, keep_cache=False, dropout=dr)[0] * dhT).sum())

    eps = 1e-6
    for key in ("h0", "edge_weights", "edge_biases", "gates_kernel", "candidate_bias"):
        base = h0 if key == "h0" else w[key]
        num = np.zeros_like(base)
        for idx in np.ndindex(base.shape):
            p, m = base.copy(), base.copy()
            p[idx] += eps
            m[idx] -= eps
            if key == "h0":
                num[idx] = (loss(w, p) - loss(w, m)) / (2 * eps)
            else:
                num[idx] = (loss({**w, key: p}, h0) - loss({**w, key: m}, h0)) / (2 * eps)
        assert np.abs(num - g[key]).max() <= 1e-7 * max(1.0, np.abs(num).max()), key


# ---------------------------------------------------------------- optimizer
def test_clip_by_norm_and_adam_known_answer():
    # clip_by_norm: ||(3, 4)|| = 5 > 1 -> (0.6, 0.8); below the clip it is the identity
    np.testing.assert_allclose(O.clip_by_norm(np.array([3.0, 4.0]), 1.0), [0.6, 0.8])
    np.testing.assert_allclose(O.clip_by_norm(np.array([0.3, 0.4]), 1.0), [0.3, 0.4])
    # TF1 Adam, first step: m = 0.1 g, v = 0.001 g^2, lr_t = lr sqrt(0.001)/0.1
    # -> p -= lr * g/|g| (1 + O(eps)) element-wise
    p, g = [np.array([1.0, -2.0])], [np.array([0.3, -0.4])]
    m, v = [np.zeros(2)], [np.zeros(2)]
    O.adam_step(p, g, m, v, 1, lr=0.01)
    np.testing.assert_allclose(p[0], [1.0 - 0.01, -2.0 + 0.01], rtol=1e-6)
    np.testing.assert_allclose(m[0], [0.03, -0.04])
    np.testing.assert_allclose(v[0], [0.3 ** 2 * 1e-3, 0.4 ** 2 * 1e-3])
