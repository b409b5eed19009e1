"""GPU parity of the general path (k_gemm products + k_generic.h element-wise
kernels): the shapes the specialised kernels do not take -- the reference's
default hidden_size 400 (chem_tensorflow.py:95), buckets beyond 128 nodes up to
198 (chem_tensorflow_dense.py:584-585), odd hidden sizes, hidden 64 training
-- against the float64 oracle at the fp32 bar (forward max |err| <= 1e-3,
every gradient's normalised max error <= 1e-3), with dropout, at the btb
loss's gradient scale, with empty-channel skipping and from edge lists.
"""
import numpy as np
import pytest

import ggnn_oracle as O
from test_gpu_parity import (FP32_TOL, GRADS, _case, _f64, _nmax, _nrms, _run, _run_dropout, _torch,
                             _tree_adjacency)

pytestmark = pytest.mark.gpu

GEN_SHAPES = [
    (3, 20, 400, 4, 2),     # the reference's default hidden_size
    (2, 150, 128, 4, 2),    # v > 128
    (2, 198, 64, 6, 2),     # the reference's largest bucket, hidden 64 (training)
    (3, 37, 100, 5, 3),     # odd hidden, odd v, odd C
    (4, 50, 256, 6, 2),     # a fast-path shape, forced through the general path
]


def _ref(A, h0, w, T, dhT):
    A64, w64 = A.astype(np.float64), _f64(w)
    ref, caches = O.forward(A64, h0.astype(np.float64), w64, T)
    return ref, O.backward(A64, dhT.astype(np.float64), caches, w64)


@pytest.mark.parametrize("b,v,h,C,T", GEN_SHAPES)
def test_generic_fp32_parity(b, v, h, C, T):
    A, h0, w = _case(b, v, h, C, seed=b * 11 + v)
    dhT = np.random.default_rng(2).standard_normal((b, v, h)).astype(np.float32)
    ref, gref = _ref(A, h0, w, T, dhT)
    got = _run(A, h0, w, T, "fp32", dhT=dhT, generic=True)
    assert np.abs(got["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k
    inf = _run(A, h0, w, T, "fp32", generic=True)   # inference workspace (no saves)
    assert np.abs(inf["hT"] - ref).max() <= FP32_TOL


@pytest.mark.parametrize("scale", [2.0 ** -12, 2.0 ** -16])
def test_generic_backward_at_loss_scale(scale):
    b, v, h, C, T = 2, 150, 400, 4, 3
    A, h0, w = _case(b, v, h, C, seed=31)
    dhT = (np.random.default_rng(4).standard_normal((b, v, h)) * scale).astype(np.float32)
    ref, gref = _ref(A, h0, w, T, dhT)
    got = _run(A, h0, w, T, "fp32", dhT=dhT)
    for k in GRADS:
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k


def test_generic_matches_fast_path():
    """The config-3 slice through both paths: same math, different kernels."""
    b, v, h, C, T = 2, 128, 256, 8, 3
    A, h0, w = _case(b, v, h, C, seed=77)
    dhT = np.random.default_rng(5).standard_normal((b, v, h)).astype(np.float32)
    fast = _run(A, h0, w, T, "fp32", dhT=dhT)
    gen = _run(A, h0, w, T, "fp32", dhT=dhT, generic=True)
    assert np.abs(fast["hT"] - gen["hT"]).max() <= 5e-5
    for k in GRADS:
        # (the fast path's weight-gradient GEMMs take single f16 operands: <= 3.7e-4 vs float64)
        assert _nmax(gen[k], fast[k]) <= FP32_TOL, k


@pytest.mark.parametrize("ek,sk", [(0.9, 0.9), (0.6, 1.0), (1.0, 0.7)])
def test_generic_dropout_fp32_parity(ek, sk):
    b, v, h, C, T = 3, 140, 96, 4, 3
    A, h0, w = _case(b, v, h, C, seed=9)
    dhT = np.random.default_rng(8).standard_normal((b, v, h)).astype(np.float32)
    dr = dict(edge_keep=ek, state_keep=sk, seed=1234567 + T)
    A64, w64 = A.astype(np.float64), _f64(w)
    ref, caches = O.forward(A64, h0.astype(np.float64), w64, T, dropout=dr)
    gref = O.backward(A64, dhT.astype(np.float64), caches, w64)
    got = _run_dropout(A, h0, w, T, "fp32", dr, dhT)
    assert np.abs(got["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k
    nodrop, _ = O.forward(A64, h0.astype(np.float64), w64, T, keep_cache=False)
    assert np.abs(nodrop - ref).max() > 0.05


@pytest.mark.parametrize("b,v,h,C", [(2, 40, 65, 2), (2, 36, 102, 3), (2, 20, 3, 2), (1, 12, 1, 1)])
def test_generic_edge_dropout_hidden_not_multiple_of_4(b, v, h, C):
    """The general path's masked fp32 W copies (k_pack_multi copy mode 2) at
    hidden % 4 != 0 and hidden < 4: the last row quad of every W_c is partial,
    and every row must still be written exactly once with its Philox mask."""
    T = 2
    A, h0, w = _case(b, v, h, C, seed=h * 3 + C)
    dhT = np.random.default_rng(h).standard_normal((b, v, h)).astype(np.float32)
    dr = dict(edge_keep=0.7, state_keep=1.0, seed=98765 + h)
    A64, w64 = A.astype(np.float64), _f64(w)
    ref, caches = O.forward(A64, h0.astype(np.float64), w64, T, dropout=dr)
    gref = O.backward(A64, dhT.astype(np.float64), caches, w64)
    got = _run_dropout(A, h0, w, T, "fp32", dr, dhT)
    assert np.abs(got["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        # (hidden 1: every weight gradient is one to four numbers, each a sum over
        # 24 rows x T of single-f16 operand products (the weight-gradient
        # policy) with mixed signs; their relative error is that
        # sum's cancellation, not the mask's)
        tol = 5e-3 if (h == 1 and k in ("edge_weights", "gates_kernel", "candidate_kernel")) else FP32_TOL
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= tol, k


@pytest.mark.parametrize("v,h", [(120, 400), (190, 128)])
def test_generic_empty_channel_skipping(v, h):
    """Real-data channel count (C = 92) on the general path: h_T and dL/dh0
    bit-identical with and without skipping, and fp32 parity."""
    b, E, T = 3, 46, 2
    C = 2 * E
    A = _tree_adjacency(b, v, E, seed=v)
    rng = np.random.default_rng(h)
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, C, seed=E)
    dhT = (rng.standard_normal((b, v, h)) * 2.0 ** -10).astype(np.float32)
    skip = _run(A, h0, w, T, "fp32", dhT=dhT, skip=True)
    dense = _run(A, h0, w, T, "fp32", dhT=dhT, skip=False)
    for k in ("hT", "h0"):
        assert np.array_equal(skip[k], dense[k]), k
    ref, gref = _ref(A, h0, w, T, dhT)
    assert np.abs(skip["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        assert _nmax(skip[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k


def test_generic_adjacency_from_edges():
    """Edge-list staging on the general path (v = 160 > 128) gives the same
    forward as the dense feed of graph_to_adj_mat_bd (chem_tensorflow_dense.py:65-83)."""
    torch = _torch()
    from ggnn_amd.engine import PropagationEngine
    b, v, h, E, T = 3, 160, 128, 5, 2
    rng = np.random.default_rng(3)
    graphs = []
    for _ in range(b):
        n = int(rng.integers(v // 2, v + 1))
        graphs.append([(int(rng.integers(0, i)), int(rng.integers(1, E + 1)), i) for i in range(1, n)])
    graphs[1] = graphs[1] + [(3, 2, 0)]   # dest 0: the reference's prev-word index wraps to v-1
    A = np.stack([O.graph_to_adj_mat_bd(g, v, E, dtype=np.float32) for g in graphs])
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=1)
    eng = PropagationEngine(h, 2 * E, sparse_pairs=False)    # the dense-tile general path
    dev = eng.device
    pack = eng.pack_weights({k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()})
    eng.set_adjacency_edges(graphs, v, E)
    a = eng.forward(torch.from_numpy(h0).to(dev), pack, T).cpu().numpy()
    eng.set_adjacency(torch.from_numpy(A).to(dev))
    d = eng.forward(torch.from_numpy(h0).to(dev), pack, T).cpu().numpy()
    assert np.array_equal(a, d)
    ref, _ = O.forward(A.astype(np.float64), h0.astype(np.float64), _f64(w), T, keep_cache=False)
    assert np.abs(a - ref).max() <= FP32_TOL
    # the default ("auto") stages this edge-list batch in pair mode: same
    # math in another summation order
    pe = PropagationEngine(h, 2 * E)
    pe.set_adjacency_edges(graphs, v, E)
    assert pe.sparse
    p = pe.forward(torch.from_numpy(h0).to(dev), pe.pack_weights(
        {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}), T).cpu().numpy()
    assert np.abs(p - ref).max() <= FP32_TOL and np.abs(p - a).max() <= 1e-5


def test_generic_bf16_statistical():
    b, v, h, C, T = 2, 150, 400, 4, 2
    A, h0, w = _case(b, v, h, C, seed=12)
    dhT = np.random.default_rng(6).standard_normal((b, v, h)).astype(np.float32)
    ref, gref = _ref(A, h0, w, T, dhT)
    got = _run(A, h0, w, T, "bf16", dhT=dhT)
    assert _nrms(got["hT"], ref) <= 2e-2
    for k in GRADS:
        assert _nrms(got[k].reshape(gref[k].shape), gref[k]) <= 5e-2, k


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 150, 61), (130, 129, 257), (256, 512, 96), (512, 64, 1000)])
@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_k_gemm_against_numpy(M, N, K, precision):
    """The general path's product kernel on its own (ggnn_dbg_gemm): ragged
    shapes across the 64/128-row tile variants; fp32-parity mode within 1e-6 of
    float64 relative to the accumulated magnitude, 16-bit modes within their
    operand rounding."""
    torch = _torch()
    import ctypes
    from ggnn_amd import _lib
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    dev = torch.device("cuda", 0)
    a, b = torch.from_numpy(A).to(dev), torch.from_numpy(B).to(dev)
    d = torch.full((M, N), float("nan"), device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, precision)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.load().ggnn_dbg_gemm(ctypes.byref(dims), M, N, K, ctypes.c_void_p(a.data_ptr()),
                                         ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(d.data_ptr()), s),
               "ggnn_dbg_gemm")
    got = d.cpu().numpy()
    ref = A.astype(np.float64) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
    err = float(np.max(np.abs(got - ref) / np.maximum(scale, 1e-30)))
    assert err <= {"fp32": 1e-6, "fp16": 2e-3, "bf16": 1e-2}[precision], err


def _gemm_ex(A, a_layout, B, b_layout, M, N, K, precision, kernel):
    torch = _torch()
    import ctypes
    from ggnn_amd import _lib
    dev = torch.device("cuda", 0)
    a, b = torch.from_numpy(np.ascontiguousarray(A)).to(dev), torch.from_numpy(np.ascontiguousarray(B)).to(dev)
    d = torch.full((M, N), float("nan"), device=dev)
    dims = _lib.dims(1, 1, 64, 1, 1, True, precision)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(_lib.load().ggnn_dbg_gemm_ex(ctypes.byref(dims), M, N, K, ctypes.c_void_p(a.data_ptr()), a_layout,
                                            ctypes.c_void_p(b.data_ptr()), b_layout, ctypes.c_void_p(d.data_ptr()),
                                            kernel, s), "ggnn_dbg_gemm_ex")
    return d.cpu().numpy()


# (M, N multiples of 4 and K of 8: the ring's alignment rules for every layout
# below; ragged against its 128 x 128 tiles and 32-wide K slices)
RING_SHAPES = [(4, 4, 8), (128, 128, 32), (132, 260, 40), (400, 800, 400), (28, 400, 88), (1000, 48, 1000),
               (64, 128, 8), (36, 36, 200)]


@pytest.mark.parametrize("M,N,K", RING_SHAPES)
@pytest.mark.parametrize("a_layout,b_layout", [(0, 0), (0, 1), (1, 0), (2, 0)])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_k_gemm_ring_layouts(M, N, K, a_layout, b_layout, precision):
    """k_gemm_ring (128 x 128 tiles, LDS-DMA ring) on every operand layout the
    general path uses, incl. ragged M / N / K tails and K < one slice: fp32
    mode within 1e-6 of float64 relative to the accumulated magnitude, and
    identical to k_gemm's result up to accumulation order."""
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    if a_layout == 2:   # exact 16-bit operand (the 0/1 adjacency)
        A = (rng.random((M, K)) < 0.3).astype(np.float32)
        Aop = A.astype(np.float16).view(np.uint16) if precision != "bf16" else (A.view(np.uint32) >> 16).astype(np.uint16)
    else:
        A = rng.standard_normal((M, K)).astype(np.float32)
        Aop = A if a_layout == 0 else np.ascontiguousarray(A.T)
    B = rng.standard_normal((K, N)).astype(np.float32)
    Bop = B if b_layout == 0 else np.ascontiguousarray(B.T)
    ring = _gemm_ex(Aop, a_layout, Bop, b_layout, M, N, K, precision, 2)
    old = _gemm_ex(Aop, a_layout, Bop, b_layout, M, N, K, precision, 1)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
    # (plus an absolute floor of 2^-24 per term: the f16 lo limb of an operand
    # below 2^-3 in magnitude is subnormal, in both kernels alike)
    tol = {"fp32": 1e-6, "bf16": 1e-2}[precision]
    bound = tol * scale + K * 2.0 ** -24
    for got in (ring, old):
        assert np.all(np.abs(got - ref) <= bound), float(np.max(np.abs(got - ref) / bound))
    assert np.all(np.abs(ring - old) <= 2 * bound)


@pytest.mark.parametrize("M,N,K", RING_SHAPES + [(700, 800, 800), (33, 37 * 4, 1000), (96, 32, 264)])
@pytest.mark.parametrize("b_layout", [0, 1])
@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("kernel", [3, 4, 5])
def test_k_gemm_ks_against_numpy(M, N, K, b_layout, precision, kernel):
    """k_gemm_ks (32-row tiles, the K slices split over 4 / 2 / 1 wave groups
    of 1 / 2 / 4 column blocks, partials summed in a fixed order): fp32-parity
    mode within 1e-6 of float64 relative to the accumulated magnitude, incl.
    K < 4 slices (waves without a slice), ragged M / N / K tails; deterministic
    (two runs bit-identical)."""
    rng = np.random.default_rng(M * 5 + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    Bop = B if b_layout == 0 else np.ascontiguousarray(B.T)
    ks = _gemm_ex(A, 0, Bop, b_layout, M, N, K, precision, kernel)
    again = _gemm_ex(A, 0, Bop, b_layout, M, N, K, precision, kernel)
    assert np.array_equal(ks, again)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
    tol = {"fp32": 1e-6, "fp16": 2e-3, "bf16": 1e-2}[precision]
    bound = tol * scale + K * 2.0 ** -24
    assert np.all(np.abs(ks - ref) <= bound), float(np.max(np.abs(ks - ref) / bound))


# ---------------------------------------------------------------------------
# Pair mode (GGNN_SPARSE_PAIRS, k_pairs.h): the general path's sparse message
# passing over the (node, channel) pairs with an incoming edge.

def _trees(b, v, E, seed, extra=0):
    """Dependency trees with the real label count (E labels -> C = 2E), plus
    `extra` random extra edges per graph (a head with several children of one
    label: in-degree > 1 on an outgoing channel)."""
    rng = np.random.default_rng(seed)
    pz = 1.0 / np.arange(1, E + 1)
    pz /= pz.sum()
    graphs = []
    for _ in range(b):
        n = int(rng.integers(max(2, v // 2), v + 1))
        g = [(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)]
        g += [(int(rng.integers(0, n)), int(rng.integers(1, E + 1)), int(rng.integers(1, n))) for _ in range(extra)]
        graphs.append(g)
    A = np.stack([O.graph_to_adj_mat_bd(g, v, E, dtype=np.float32) for g in graphs])
    return graphs, A


def _run_edges(graphs, v, E, h0, w, T, precision="fp32", dhT=None, sparse="auto", dr=None, force_generic=False,
               batch_pack=False, skip=True):
    torch = _torch()
    from ggnn_amd.engine import PropagationEngine
    b, h = h0.shape[0], h0.shape[-1]
    eng = PropagationEngine(h, 2 * E, precision=precision, sparse_pairs=sparse, force_generic=force_generic,
                            skip_empty_channels=skip)
    dev = eng.device
    dr = dr or dict(edge_keep=1.0, state_keep=1.0, seed=0)
    wd = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    if batch_pack:     # the model's order: stage the batch, then pack for it (ggnn_pack_weights_batch)
        eng.set_adjacency_edges(graphs, v, E)
    out = None
    if batch_pack:     # every byte a NaN sentinel: a copy the pack skips must not be read
        d = eng.dims(b, v, T, edge_keep=dr["edge_keep"], seed=dr["seed"])
        from ggnn_amd import _lib
        out = torch.full((_lib.weight_pack_bytes(d),), 0xFF, dtype=torch.uint8, device=dev)
    pack = eng.pack_weights(wd, T=T, edge_keep=dr["edge_keep"], seed=dr["seed"], batch=batch_pack, out=out)
    if not batch_pack:
        eng.set_adjacency_edges(graphs, v, E)
    out = eng.forward(torch.from_numpy(np.ascontiguousarray(h0)).to(dev), pack, T, training=dhT is not None,
                      state_keep=dr["state_keep"])
    res = {"hT": out.cpu().numpy(), "sparse": eng.sparse}
    if dhT is not None:
        g = eng.backward(torch.from_numpy(np.ascontiguousarray(dhT)).to(dev))
        res.update({k: (None if t is None else t.cpu().numpy()) for k, t in g.items()})
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("b,v,h,T,extra,sparse", [
    (6, 30, 400, 4, 0, "auto"),     # the reference's own configuration (hidden 400, T 4, C 92)
    (4, 46, 400, 3, 3, "auto"),     # several children of one label: in-degree > 1
    (3, 150, 128, 2, 0, "auto"),    # v > 128
    (5, 30, 256, 3, 1, True),       # a fast-path hidden size, forced into pair mode
    (2, 7, 20, 2, 0, "auto"),       # tiny graphs, hidden not a multiple of 32
])
def test_sparse_pairs_fp32_parity(b, v, h, T, extra, sparse):
    E = 46
    graphs, A = _trees(b, v, E, seed=v + h, extra=extra)
    rng = np.random.default_rng(h)
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=v)
    dhT = (rng.standard_normal((b, v, h)) * 2.0 ** -8).astype(np.float32)
    got = _run_edges(graphs, v, E, h0, w, T, dhT=dhT, sparse=sparse)
    assert got["sparse"]
    ref, gref = _ref(A, h0, w, T, dhT)
    assert np.abs(got["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k
    # the same batch through the dense-tile general path: same math, another order
    dense = _run_edges(graphs, v, E, h0, w, T, dhT=dhT, sparse=False, force_generic=True)
    assert not dense["sparse"]
    assert np.abs(got["hT"] - dense["hT"]).max() <= 1e-5
    for k in GRADS:
        # (dW_c takes single f16 operands in both, <= 3.7e-4 each vs float64, with
        # different rounding points: Y = sum of h rows here, h and dM there)
        tol = FP32_TOL if k in ("edge_weights", "gates_kernel", "candidate_kernel") else 1e-4
        assert _nmax(got[k], dense[k]) <= tol, k


@pytest.mark.parametrize("batch_pack", [False, True])
@pytest.mark.parametrize("ek,sk", [(0.9, 0.9), (0.6, 1.0)])
def test_sparse_pairs_dropout_fp32_parity(ek, sk, batch_pack):
    """Edge-weight dropout in pair mode: the masked weight copies in the
    products and the mask of timestep t applied in the dW product's epilogue
    (no per-timestep slab), against the oracle's Philox masks."""
    b, v, h, T, E = 4, 30, 400, 3, 46
    graphs, A = _trees(b, v, E, seed=7, extra=2)
    rng = np.random.default_rng(3)
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=5)
    dhT = rng.standard_normal((b, v, h)).astype(np.float32)
    dr = dict(edge_keep=ek, state_keep=sk, seed=424242)
    A64, w64 = A.astype(np.float64), _f64(w)
    ref, caches = O.forward(A64, h0.astype(np.float64), w64, T, dropout=dr)
    gref = O.backward(A64, dhT.astype(np.float64), caches, w64)
    got = _run_edges(graphs, v, E, h0, w, T, dhT=dhT, dr=dr, batch_pack=batch_pack)
    assert got["sparse"]
    assert np.abs(got["hT"] - ref).max() <= FP32_TOL
    for k in GRADS:
        assert _nmax(got[k].reshape(gref[k].shape), gref[k]) <= FP32_TOL, k


@pytest.mark.parametrize("mode", ["pairs", "tiles", "tiles_dense_channels"])
def test_batch_pack_masks_only_the_batch_channels(mode):
    """ggnn_pack_weights_batch (the model's pack: stage, then pack for the
    batch): under edge dropout on the general path it writes the masked W_c
    copies only for channels with an edge in the staged batch -- a sentence
    batch touches about half of the 92 -- in pair mode and on the dense-tile
    general path; with GGNN_DENSE_CHANNELS (skip_empty_channels=False) every
    tile runs, so it writes every copy.  The pack is made into a buffer of NaN
    sentinels: the step's results equal the full pack's (h_T and dL/dh0 bit
    for bit; weight gradients up to the order of their fp32 atomics), so no
    skipped copy is read; the skipped copies still hold the sentinel; and a
    pack made for one staged batch is refused for the next."""
    torch = _torch()
    from ggnn_amd import _lib
    from ggnn_amd.engine import PropagationEngine
    kw = {"pairs": dict(sparse="auto"), "tiles": dict(sparse=False, force_generic=True),
          "tiles_dense_channels": dict(sparse=False, force_generic=True, skip=False)}[mode]
    b, v, h, T, E = 3, 30, 400, 3, 46
    graphs, A = _trees(b, v, E, seed=11)
    used = A.reshape(b, 2 * E, -1).max(axis=(0, 2)) > 0
    assert 0 < used.sum() < 2 * E
    rng = np.random.default_rng(4)
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=6)
    dhT = rng.standard_normal((b, v, h)).astype(np.float32)
    dr = dict(edge_keep=0.8, state_keep=0.9, seed=777)
    full = _run_edges(graphs, v, E, h0, w, T, dhT=dhT, dr=dr, **kw)
    part = _run_edges(graphs, v, E, h0, w, T, dhT=dhT, dr=dr, batch_pack=True, **kw)
    assert part["sparse"] == (mode == "pairs")
    for k in ("hT", "h0"):
        assert np.array_equal(full[k], part[k]), k
    for k in GRADS[1:]:
        assert np.isfinite(part[k]).all() and _nmax(part[k], full[k]) <= 1e-6, k
    # the copies: occupied channels masked exactly as the full pack, the others untouched
    eng = PropagationEngine(h, 2 * E, sparse_pairs=kw["sparse"], force_generic=kw.get("force_generic", False),
                            skip_empty_channels=kw.get("skip", True))
    wd = {k: torch.from_numpy(np.ascontiguousarray(x)).to(eng.device) for k, x in w.items()}
    eng.set_adjacency_edges(graphs, v, E)
    nb = _lib.weight_pack_bytes(eng.dims(b, v, T, edge_keep=0.8, seed=777))
    pf = eng.pack_weights(wd, T=T, edge_keep=0.8, seed=777)
    pb = eng.pack_weights(wd, T=T, edge_keep=0.8, seed=777, batch=True,
                          out=torch.full((nb,), 0xFF, dtype=torch.uint8, device=eng.device))
    pb2 = eng.pack_weights(wd, T=T, edge_keep=0.8, seed=777, batch=True)
    torch.cuda.synchronize()
    if mode == "tiles_dense_channels":
        used = np.ones_like(used)
    al = lambda x: (x + 255) & ~255  # noqa: E731  (ggnn_api.hip pack_layout: beta, bg, bc, then the copies)
    C = 2 * E
    g_w = al(C * h * 4) + al(2 * h * 4) + al(h * 4)
    n = C * h * h * 4
    for t in range(T):
        o = g_w + t * al(n)
        cf = pf.buf[o:o + n].view(torch.float32).view(C, h * h)
        cb = pb.buf[o:o + n].view(torch.float32).view(C, h * h)
        u = torch.from_numpy(used).to(eng.device)
        assert torch.equal(cf[u], cb[u]), t
        raw = pb.buf[o:o + n].view(C, h * h * 4)
        assert bool((raw[~u] == 0xFF).all()), t       # skipped copies: the sentinel, unwritten
    # the keep bits the pack writes beside the copies (round 5: the pair dW
    # product's mbits), after Wg, Wc and the occupancy bytes
    w32 = (h + 31) // 32
    ob = g_w + T * al(n) + al(4 * h * h * 4) + al(2 * h * h * 4) + al(C)
    nbits = C * h * w32 * 4
    u = torch.from_numpy(used).to(eng.device)
    for t in range(T):
        bf = pf.buf[ob + t * nbits:ob + (t + 1) * nbits].view(torch.int32).view(C, h * w32)
        bb = pb.buf[ob + t * nbits:ob + (t + 1) * nbits].view(torch.int32).view(C, h * w32)
        assert torch.equal(bf[u], bb[u]), t
        assert bool((bb[~u] == -1).all()), t
        # bit (i % 32) of word (c, j, i // 32): kept iff the masked copy is nonzero where W is
        cf = pf.buf[g_w + t * al(n):g_w + t * al(n) + n].view(torch.float32).view(C, h, h).cpu().numpy()
        words = bf.cpu().numpy().astype(np.uint32).reshape(C, h, w32)
        i = np.arange(h)
        keep = (words[:, :, i // 32] >> (i % 32)[None, None, :]) & 1      # [c][j][i]
        wsrc = w["edge_weights"].reshape(C, h, h)
        nz = wsrc != 0
        assert np.array_equal((cf != 0)[nz], keep.transpose(0, 2, 1).astype(bool)[nz]), t
    eng.set_adjacency_edges(graphs[:2], v, E)
    with pytest.raises(RuntimeError):
        eng.forward(torch.zeros((2, v, h), device=eng.device), pb2, T)


@pytest.mark.parametrize("precision", ["fp16", "bf16"])
def test_sparse_pairs_16bit(precision):
    b, v, h, T, E = 4, 30, 400, 4, 46
    graphs, A = _trees(b, v, E, seed=11)
    rng = np.random.default_rng(4)
    h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    w = O.synthetic_weights(h, 2 * E, seed=6)
    dhT = rng.standard_normal((b, v, h)).astype(np.float32)
    ref, gref = _ref(A, h0, w, T, dhT)
    got = _run_edges(graphs, v, E, h0, w, T, precision=precision, dhT=dhT)
    assert got["sparse"]
    assert _nrms(got["hT"], ref) <= 1e-2
    for k in GRADS:
        assert _nrms(got[k].reshape(gref[k].shape), gref[k]) <= 1e-2, k


def test_sparse_pairs_rejected_for_dense_staging_and_too_many_edges():
    torch = _torch()
    import ctypes
    from ggnn_amd import _lib
    lib = _lib.load()
    b, v, h, C = 2, 10, 64, 4
    d = _lib.dims(b, v, h, C, 1, True, "fp32", sparse_pairs=True)
    nb = _lib.adjacency_bytes(d)
    adj = torch.empty(nb, dtype=torch.uint8, device="cuda")
    A = torch.zeros((b, C, v, v), device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = lib.ggnn_set_adjacency(ctypes.byref(d), ctypes.c_void_p(adj.data_ptr()), ctypes.c_void_p(A.data_ptr()), s)
    assert rc == -1
    edges = torch.zeros((b * v + 1, 3), dtype=torch.int32, device="cuda")
    offs = torch.tensor([0, b * v + 1, b * v + 1], dtype=torch.int32, device="cuda")
    rc = lib.ggnn_set_adjacency_edges(ctypes.byref(d), ctypes.c_void_p(adj.data_ptr()),
                                      ctypes.c_void_p(edges.data_ptr()), ctypes.c_void_p(offs.data_ptr()),
                                      b * v + 1, C // 2, s)
    assert rc == -2
    bad = _lib.dims(b, v, 66, C, 1, True, "fp32", sparse_pairs=True)
    assert lib.ggnn_check_dims(ctypes.byref(bad)) == -2     # hidden % 4 != 0


@pytest.mark.parametrize("h,keep", [(400, 0.85), (400, 1.0), (96, 0.5)])
def test_pack_general_copies_vector_form_equals_scalar_form(h, keep):
    """ggnn_pack_weights' fp32 W copies (general path, masked per timestep
    under edge dropout): the 16-byte form (aligned W, hidden % 4 == 0) writes
    the same bytes as the per-element form (a W 4 bytes off alignment)."""
    import torch
    from ggnn_amd.engine import PropagationEngine
    C, T = 5, 3
    dev = torch.device("cuda", 0)
    eng = PropagationEngine(h, C, device=dev, force_generic=True)
    g = torch.Generator().manual_seed(7)
    w = {"edge_weights": torch.randn(C, h, h, generator=g), "edge_biases": torch.randn(C, 1, h, generator=g),
         "gates_kernel": torch.randn(2 * h, 2 * h, generator=g), "gates_bias": torch.randn(2 * h, generator=g),
         "candidate_kernel": torch.randn(2 * h, h, generator=g), "candidate_bias": torch.randn(h, generator=g)}
    w = {k: v.to(dev) for k, v in w.items()}
    big = torch.empty(C * h * h + 1, device=dev)
    big[1:] = w["edge_weights"].reshape(-1)
    w_off = dict(w, edge_weights=big[1:].view(C, h, h))
    assert w_off["edge_weights"].data_ptr() % 16 == 4
    pa = eng.pack_weights(w, T=T, edge_keep=keep, seed=12345)
    pb = eng.pack_weights(w_off, T=T, edge_keep=keep, seed=12345)
    torch.cuda.synchronize()
    al = lambda x: (x + 255) & ~255  # noqa: E731  (ggnn_api.hip pack_layout)
    g_w = al(C * h * 4) + al(2 * h * 4) + al(h * 4)
    n = C * h * h * 4
    for t in range(T if keep < 1 else 1):
        o = g_w + t * al(n)
        a, b = pa.buf[o:o + n], pb.buf[o:o + n]
        assert torch.equal(a, b), "timestep %d: vector and scalar copies differ" % t
    if keep == 1.0:
        assert torch.equal(pa.buf[g_w:g_w + n].view(torch.float32), w["edge_weights"].reshape(-1))


@pytest.mark.parametrize("kernel", [3, 4, 5])
@pytest.mark.parametrize("b_layout", [0, 1])
def test_k_gemm_ks_limb_split_wait_states(kernel, b_layout):
    """The inline-asm limb split (ggnn_common.h pk_lo: v_fma_mix{lo,hi}_f16)
    feeds MFMA operands; its VALU -> MFMA wait states live inside the asm
    string (round 4: without them k_gemm_ks read the previous fragment's lo
    limbs).  Direct check on k_gemm_ks in fp32-parity mode: every A element is
    1 + j * 2^-13 (hi limb 1, a distinct lo limb j * 2^-13 per element) and B is
    one-hot, so each output is ONE A element, exact in fp32 only if its own
    lo limb entered the product; a stale or missing lo limb shows as the exact
    (m, n) it hits (tools/ks_debug.py / tools/limb_mix_test.hip)."""
    M, N, K = 96, 64, 256
    rng = np.random.default_rng(kernel * 2 + b_layout)
    j = rng.integers(1, 64, (M, K))
    A = (1.0 + j * 2.0 ** -13).astype(np.float32)
    kk = rng.permutation(K)[:N]                           # output column n reads A[:, kk[n]]
    B = np.zeros((K, N), np.float32)
    B[kk, np.arange(N)] = 1.0
    Bop = B if b_layout == 0 else np.ascontiguousarray(B.T)
    got = _gemm_ex(A, 0, Bop, b_layout, M, N, K, "fp32", kernel)
    want = A[:, kk]
    bad = np.argwhere(got != want)
    assert bad.size == 0, (len(bad), bad[:5].tolist(), got[tuple(bad[0])], want[tuple(bad[0])])
    # the same through the B side: A one-hot rows, B with distinct lo limbs
    A2 = np.zeros((M, K), np.float32)
    ka = rng.integers(0, K, M)
    A2[np.arange(M), ka] = 1.0
    B2 = (1.0 + rng.integers(1, 64, (K, N)) * 2.0 ** -13).astype(np.float32)
    B2op = B2 if b_layout == 0 else np.ascontiguousarray(B2.T)
    got2 = _gemm_ex(A2, 0, B2op, b_layout, M, N, K, "fp32", kernel)
    assert np.array_equal(got2, B2[ka, :])
