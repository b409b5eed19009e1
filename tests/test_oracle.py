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
