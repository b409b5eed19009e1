"""The device-resident step scalars behind hipGraph capture (include/ggnn.h):
GGNN_SEED_DEVICE (dims.seed / the embed and heads seeds as the address of a
device uint64), ggnn_heads_{forward,backward}_dev (target_num in device
memory) and ggnn_adam_step_dev (the step count in device memory) must give
exactly what passing the same values by argument gives."""
import ctypes

import numpy as np
import pytest

import ggnn_oracle as O

pytestmark = pytest.mark.gpu


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _seed_tensor(torch, value):
    return torch.tensor([value], dtype=torch.int64, device="cuda")


@pytest.mark.parametrize("kind", [0, 1])
def test_dropout_masks_from_a_device_seed(kind):
    torch = _torch()
    from ggnn_amd import _lib
    lib = _lib.load()
    seed = 0x1234_5678_9ABC_DEF1 & 0x7FFF_FFFF_FFFF_FFFF
    st = _seed_tensor(torch, seed)
    b, v, h, C, T = 3, 20, 96, 6, 3
    shape = (C, h, h) if kind == 0 else (b, v, h)
    masks = []
    for dev_seed in (False, True):
        d = _lib.dims(b, v, h, C, T, True, "fp32", 0.8 if kind == 0 else 1.0, 0.8 if kind == 1 else 1.0,
                      st.data_ptr() if dev_seed else seed, seed_device=dev_seed)
        m = torch.empty(shape, dtype=torch.uint8, device="cuda")
        _lib.check(lib.ggnn_dropout_mask(ctypes.byref(d), kind, 1, ctypes.c_void_p(m.data_ptr()),
                                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "mask")
        masks.append(m.cpu().numpy())
    assert np.array_equal(masks[0], masks[1]) and 0 < masks[0].mean() < 1


def test_device_seed_needs_an_address_under_dropout():
    from ggnn_amd import _lib
    _torch()
    d = _lib.dims(2, 16, 128, 4, 3, True, "fp32", 0.9, 0.9, 0, seed_device=True)
    lib = _lib.load()
    size = ctypes.c_size_t(0)
    assert lib.ggnn_workspace_bytes(ctypes.byref(d), 1, ctypes.byref(size)) != 0
    assert b"GGNN_SEED_DEVICE" in lib.ggnn_last_error()


@pytest.mark.parametrize("hidden,force_generic", [(128, False), (96, True)])
def test_engine_step_with_a_device_seed(hidden, force_generic):
    """Pack, forward and backward under edge and state dropout: the same h_T
    and dL/dh0 bit for bit (the weight gradients to the atomics' rounding)."""
    torch = _torch()
    from ggnn_amd.engine import PropagationEngine
    rng = np.random.default_rng(5)
    b, v, C, T = 4, 24, 6, 3
    A, h0 = O.synthetic_batch(b, v, hidden, C, seed=5, density=0.1)
    w = O.synthetic_weights(hidden, C, seed=5)
    dev = torch.device("cuda")
    wts = {k: torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(dev) for k, x in w.items()}
    dhT = torch.from_numpy(rng.standard_normal((b, v, hidden)).astype(np.float32)).to(dev)
    seed = 987654321
    st = _seed_tensor(torch, seed)
    outs = []
    for dev_seed in (False, True):
        eng = PropagationEngine(hidden, C, True, device=dev, force_generic=force_generic)
        eng.set_adjacency(torch.from_numpy(A).to(dev))
        pack = eng.pack_weights(wts, T=T, edge_keep=0.85, seed=st.data_ptr() if dev_seed else seed,
                                seed_device=dev_seed)
        hT = eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=True, state_keep=0.8)
        g = eng.backward(dhT)
        torch.cuda.synchronize()
        outs.append((hT.cpu().numpy(), {k: None if x is None else x.cpu().numpy() for k, x in g.items()}))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1]["h0"], outs[1][1]["h0"])
    for k, x in outs[0][1].items():
        if x is not None:
            assert np.abs(x - outs[1][1][k]).max() <= 1e-6 * max(1.0, np.abs(x).max()), k


def test_heads_with_device_target_num_and_seed():
    torch = _torch()
    from ggnn_amd.heads import OutputHeads
    rng = np.random.default_rng(3)
    b, v, h, os_ = 3, 37, 128, (150, 46)
    dev = torch.device("cuda")
    hT = torch.from_numpy(rng.uniform(-1, 1, (b, v, h)).astype(np.float32)).to(dev)
    h0 = torch.from_numpy(rng.uniform(-0.5, 0.5, (b, v, h)).astype(np.float32)).to(dev)
    heads, labels = [], []
    for o in os_:
        W = (np.sqrt(6.0 / (2 * h + o)) * (2 * rng.random((2 * h, o)) - 1)).astype(np.float32)
        heads.append((torch.from_numpy(W).to(dev), torch.from_numpy(rng.normal(size=o).astype(np.float32)).to(dev)))
        y = np.zeros((b, v, o), np.float32)
        y[np.arange(b)[:, None], np.arange(v)[None, :], rng.integers(0, min(o, v), (b, v))] = 1
        labels.append(torch.from_numpy(y).to(dev))
    tn, seed = 37.0 + O.SMALL_NUMBER, 4242
    tn_t = torch.tensor([tn], dtype=torch.float32, device=dev)
    st = _seed_tensor(torch, seed)
    res = []
    for on_dev in (False, True):
        oh = OutputHeads(h)
        probs, loss = oh.forward(hT, h0, heads, labels, 0.85, st.data_ptr() if on_dev else seed,
                                 tn_t if on_dev else tn, seed_device=on_dev)
        dws, dbs, dhT, dh0 = oh.backward(hT, h0, heads, labels, probs, tn_t if on_dev else tn)
        torch.cuda.synchronize()
        res.append(([p.cpu().numpy() for p in probs], loss.cpu().numpy(), [x.cpu().numpy() for x in dws + dbs],
                    dhT.cpu().numpy(), dh0.cpu().numpy()))
    (p0, l0, w0, a0, c0), (p1, l1, w1, a1, c1) = res
    assert all(np.array_equal(x, y) for x, y in zip(p0, p1))
    assert np.allclose(l0, l1, rtol=1e-6, atol=0)   # (the per-head loss: 1/target_num applied in-kernel)
    assert np.array_equal(a0, a1) and np.array_equal(c0, c1)
    for x, y in zip(w0, w1):
        assert np.abs(x - y).max() <= 1e-6 * max(1.0, np.abs(x).max())


def test_adam_step_count_from_device_memory():
    torch = _torch()
    from ggnn_amd.optim import ClipAdam
    rng = np.random.default_rng(8)
    shapes = [(64, 32), (32,), (17, 5)]
    p0 = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    runs = []
    for on_dev in (False, True):
        params = [torch.from_numpy(x.copy()).cuda() for x in p0]
        opt = ClipAdam(params, learning_rate=0.01, clamp_gradient_norm=1.0)
        step = torch.zeros(1, dtype=torch.int64, device="cuda")
        g_rng = np.random.default_rng(9)
        for t in range(1, 4):
            grads = [torch.from_numpy(g_rng.standard_normal(s).astype(np.float32)).cuda() for s in shapes]
            if on_dev:
                step.fill_(t)
                opt.step(grads, step_dev=step)
            else:
                opt.step(grads)
        torch.cuda.synchronize()
        runs.append([p.cpu().numpy() for p in params])
    for x, y in zip(*runs):
        # the bias-corrected step size in double on the device vs the host: equal
        # to float32 rounding
        assert np.abs(x - y).max() <= 1e-7 * max(1.0, np.abs(x).max())
