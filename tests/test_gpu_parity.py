"""GPU parity: the HIP engine (through the C ABI) against the float64 oracle.

Tolerance (north_star, bf16 MFMA mode): 1e-2.  Forward: max |h_gpu - h_ref|
<= 1e-2 (h is bounded in (-1, 1) by the GRU).  Gradients: max-abs error
normalised by the reference's max-abs value <= 1e-2 per tensor.
"""
import numpy as np
import pytest

import ggnn_oracle as O

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-2
GRAD_TOL = 1e-2


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a HIP device")
    return torch


def _case(b, v, h, C, T, seed, use_bias=True, density=0.1):
    A, h0 = O.synthetic_batch(b, v, h, C, seed=seed, density=density)
    w = O.synthetic_weights(h, C, seed=seed)
    if not use_bias:
        w["edge_biases"] = np.zeros_like(w["edge_biases"])
    return A, h0, w


def _run_gpu(A, h0, w, T, use_bias=True, training=False, dhT=None):
    torch = _torch()
    from ggnn_amd.engine import PropagationEngine
    b, C, v, _ = A.shape
    h = h0.shape[-1]
    eng = PropagationEngine(h, C, use_edge_bias=use_bias)
    dev = eng.device
    tw = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    pack = eng.pack_weights(tw)
    eng.set_adjacency(torch.from_numpy(A).to(dev))
    out = eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=training)
    res = {"hT": out.cpu().numpy()}
    if dhT is not None:
        g = eng.backward(torch.from_numpy(dhT).to(dev))
        res.update({k: (None if t is None else t.cpu().numpy()) for k, t in g.items()})
    torch.cuda.synchronize()
    return res


def _f64(w):
    return {k: x.astype(np.float64) for k, x in w.items()}


@pytest.mark.parametrize("b,v,h,C,T", [
    (3, 20, 128, 4, 2),     # ragged v -> padded to 32
    (8, 64, 128, 4, 3),     # config-2 slice (b=32 in full)
    (2, 128, 256, 8, 2),    # config-3 shape, small batch
    (5, 50, 64, 6, 1),      # h = 64, v -> 64
    (4, 100, 256, 4, 2),    # v -> 128
])
def test_forward_matches_oracle(b, v, h, C, T):
    A, h0, w = _case(b, v, h, C, T, seed=b * 7 + v)
    ref, _ = O.forward(A.astype(np.float64), h0.astype(np.float64), _f64(w), T, keep_cache=False)
    got = _run_gpu(A, h0, w, T)["hT"]
    err = np.abs(got - ref).max()
    assert err <= FWD_TOL, "max |h_gpu - h_ref| = %.3e" % err


def test_forward_no_edge_bias():
    A, h0, w = _case(3, 40, 128, 4, 2, seed=11, use_bias=False)
    ref, _ = O.forward(A.astype(np.float64), h0.astype(np.float64), _f64(w), 2,
                       use_edge_bias=False, keep_cache=False)
    got = _run_gpu(A, h0, w, 2, use_bias=False)["hT"]
    assert np.abs(got - ref).max() <= FWD_TOL


@pytest.mark.parametrize("b,v,h,C,T", [
    (3, 20, 128, 4, 2),
    (8, 64, 128, 4, 3),
    (2, 128, 256, 8, 2),
    (4, 100, 256, 4, 3),
])
def test_backward_matches_oracle(b, v, h, C, T):
    A, h0, w = _case(b, v, h, C, T, seed=b * 13 + v)
    rng = np.random.default_rng(5)
    dhT = rng.standard_normal((b, v, h)).astype(np.float32)
    A64, w64 = A.astype(np.float64), _f64(w)
    hT, caches = O.forward(A64, h0.astype(np.float64), w64, T)
    gref = O.backward(A64, dhT.astype(np.float64), caches, w64)
    got = _run_gpu(A, h0, w, T, training=True, dhT=dhT)
    assert np.abs(got["hT"] - hT).max() <= FWD_TOL
    for k in ("h0", "edge_weights", "edge_biases", "gates_kernel", "gates_bias",
              "candidate_kernel", "candidate_bias"):
        ref = gref[k]
        g = got[k].reshape(ref.shape)
        rel = np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-12)
        assert rel <= GRAD_TOL, "%s: normalised max error %.3e" % (k, rel)
