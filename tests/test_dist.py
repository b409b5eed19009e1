"""Data-parallel path on CPU: world_size-2 gloo.  Each rank runs its own shard
of the batch (the oracle stands in for the engine on CPU), writes the weight
gradients into the FlatGradients views the engine writes on GPU, and ONE
all-reduce sums them; the sum must equal the full-batch gradient (graphs are
independent: chem_tensorflow_dense.py:414-428)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import ggnn_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from ggnn_amd.dist import FlatGradients, init_from_env
    import torch.distributed as tdist
    r, w, _ = init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    h, C, T = 8, 4, 2
    A, h0 = O.synthetic_batch(6, 10, h, C, seed=4, density=0.3, dtype=np.float64)
    wts = {k: v.astype(np.float64) for k, v in O.synthetic_weights(h, C, seed=4).items()}
    dhT = np.random.default_rng(1).standard_normal(h0.shape)
    sl = slice(rank * 3, rank * 3 + 3)                   # weak-scaling shard: 3 graphs per rank
    _, caches = O.forward(A[sl], h0[sl], wts, T)
    g = O.backward(A[sl], dhT[sl], caches, wts)
    fg = FlatGradients(h, C, True)
    for k, view in fg.views.items():
        view.copy_(torch.from_numpy(g[k].reshape(view.shape)))
    fg.all_reduce()
    if rank == 0:
        _, call = O.forward(A, h0, wts, T)
        gfull = O.backward(A, dhT, call, wts)
        err = max(float(np.abs(fg.views[k].numpy() - gfull[k].reshape(fg.views[k].shape)).max()) for k in fg.views)
        q.put(err)
    tdist.barrier()
    tdist.destroy_process_group()


def test_two_rank_gradient_allreduce_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    err = q.get(timeout=5)
    assert err < 1e-5, err


def test_flat_gradient_layout():
    from ggnn_amd.dist import FlatGradients, grad_shapes
    fg = FlatGradients(16, 6, True)
    assert fg.nbytes == 4 * sum(int(np.prod(s)) for s in grad_shapes(16, 6).values())
    fg.views["gates_bias"].fill_(3.0)
    assert float(fg.flat.sum()) == 3.0 * 32
    fg2 = FlatGradients(16, 6, False)
    assert "edge_biases" not in fg2.views
