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


# ---------------------------------------------------------------------------
# The data-parallel btb training loop (run_epoch / train_step with
# world_size > 1): rank-sharded bucketed batches and the union-batch loss.

def _golden_model(batch_size=6, hidden=48):
    import json
    from ggnn_amd.model import DenseGGNNChemModel
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)
    m = DenseGGNNChemModel(params={"hidden_size": hidden, "num_timesteps": 2, "batch_size": batch_size},
                           num_edge_types=int(g["num_edge_types"]), output_size_edges=int(g["output_size_edges"]),
                           pos_size=int(g["pos_size"]), bucket_max_nodes=int(g["bucket_max_nodes"]), device="cpu",
                           vocab_size=vocab, embedding_sizes=dict(loc=8, pos=4, word=8, edge=4))
    return m, data


@pytest.mark.parametrize("world", [2, 3, 5])
@pytest.mark.parametrize("training", [True, False])
def test_rank_sharded_iterator_partitions_the_schedule(world, training):
    """Every rank runs the same seeded schedule and takes batch k*N + r of
    global step k: together the ranks see exactly the single-process batches
    (chem_tensorflow_dense.py:792-875), each global step's feeds carry its
    total target count, and ranks past the last batch get empty feeds."""
    m, data = _golden_model()

    def feeds(rank, w):
        np.random.seed(0)       # chem_tensorflow.py:175
        return list(m.make_minibatch_iterator(m.process_raw_graphs(data, training), training, rank=rank,
                                              world_size=w))

    single = feeds(0, 1)
    per_rank = [feeds(r, world) for r in range(world)]
    steps = -(-len(single) // world)
    assert all(len(f) == steps for f in per_rank)
    for k in range(steps):
        group = single[k * world:(k + 1) * world]
        count = sum(float(np.asarray(f["target_mask"])[0].sum()) for f in group)
        for r in range(world):
            f = per_rank[r][k]
            assert f["global_target_count"] == count and f["global_num_graphs"] == sum(x["num_graphs"] for x in group)
            if r < len(group):
                ref = group[r]
                assert list(f["sentences_id"]) == list(ref["sentences_id"])
                assert f["num_vertices"] == ref["num_vertices"]
                np.testing.assert_array_equal(f["word_inputs"], ref["word_inputs"])
                np.testing.assert_array_equal(f["adjacency_matrix"], ref["adjacency_matrix"])
            else:
                assert f["num_graphs"] == 0


def _btb_weights(m, seed):
    rng = np.random.default_rng(seed)
    h, C = m.params["hidden_size"], m.num_channels
    o, oe = m.params["output_size"], m.output_size_edges
    u = lambda *s: rng.uniform(-0.3, 0.3, s)
    return {"loc_embeddings": u(m.max_nodes, 8), "pos_embeddings": u(m.pos_size, 4),
            "word_embeddings": u(m.vocab_size, 8), "edge_weights": u(C, h, h) * 0.5, "edge_biases": u(C, 1, h) * 0.1,
            "gates_kernel": u(2 * h, 2 * h), "gates_bias": 1.0 + u(2 * h) * 0.1, "candidate_kernel": u(2 * h, h),
            "candidate_bias": u(h) * 0.1, "head_W": u(2 * h, o), "head_b": u(o) * 0.1, "edge_W": u(2 * h, oe),
            "edge_b": u(oe) * 0.1}


_BTB_ORDER = ("edge_weights", "edge_biases", "gates_kernel", "gates_bias", "candidate_kernel", "candidate_bias",
              "loc_embeddings", "pos_embeddings", "word_embeddings", "head_W", "head_b", "edge_W", "edge_b")


def _union_feeds(m, data):
    """Two batches of one bucket (A, B) and their concatenation A+B."""
    proc = m.process_raw_graphs(data, False)
    bucketed, sizes, _ = proc
    bidx = max(bucketed, key=lambda k: len(bucketed[k]))
    els = bucketed[bidx]
    n = len(els) // 2
    v = int(sizes[bidx])
    return m._make_feed(els[:n], v, False), m._make_feed(els[n:2 * n], v, False), m._make_feed(els[:2 * n], v, False)


def _union_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from ggnn_amd.dist import init_from_env
    import torch.distributed as tdist
    init_from_env(backend="gloo")
    m, data = _golden_model(hidden=32)
    fa, fb, fab = _union_feeds(m, data)
    P = _btb_weights(m, 3)
    h, T, o, oe = m.params["hidden_size"], 2, m.params["output_size"], m.output_size_edges
    # every rank normalises by the GLOBAL target count (train_step's rule)
    count = float(np.asarray(fa["target_mask"])[0].sum() + np.asarray(fb["target_mask"])[0].sum())
    mine = (fa, fb)[rank]
    loss, g, sq = O.btb_loss_and_grads(P, mine, h, T, o, oe, count + O.SMALL_NUMBER)
    flat = torch.from_numpy(np.concatenate([g[k].ravel() for k in _BTB_ORDER] +
                                           [np.array([sq["loc_embeddings"], sq["pos_embeddings"],
                                                      sq["word_embeddings"], loss])]))
    tdist.all_reduce(flat)
    if rank == 0:
        l_u, g_u, sq_u = O.btb_loss_and_grads(P, fab, h, T, o, oe, count + O.SMALL_NUMBER)
        ref = np.concatenate([g_u[k].ravel() for k in _BTB_ORDER] +
                             [np.array([sq_u["loc_embeddings"], sq_u["pos_embeddings"], sq_u["word_embeddings"],
                                        l_u])])
        q.put(float(np.abs(flat.numpy() - ref).max() / np.abs(ref).max()))
    tdist.barrier()
    tdist.destroy_process_group()


def test_two_rank_btb_step_equals_union_batch():
    """The DP rule of train_step on the float64 oracle, two gloo ranks: each
    rank's btb loss over its own batch, normalised by the global target count
    (chem_tensorflow.py:358-360,399-403), then ONE sum of [every variable's
    gradient | the tables' IndexedSlices squared norms | the loss] equals the
    reference's step over the concatenated batch -- gradients, the clip norms
    tf.clip_by_norm sees (chem_tensorflow.py:498-500) and the loss."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_union_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    err = q.get(timeout=5)
    assert err < 1e-12, err


def test_flat_train_buffer_layout():
    from ggnn_amd.dist import FlatTrainBuffer
    ps = [torch.zeros(3, 5), torch.zeros(7), torch.zeros(2, 2, 2)]
    fb = FlatTrainBuffer(ps, n_sq=4, n_loss=2)
    assert [tuple(g.shape) for g in fb.grads] == [(3, 5), (7,), (2, 2, 2)]
    assert all(g.data_ptr() % 256 == fb.flat.data_ptr() % 256 for g in fb.grads)
    fb.grads[1].fill_(1.0)
    fb.sq.fill_(2.0)
    fb.loss.fill_(3.0)
    assert float(fb.flat.sum()) == 7.0 + 8.0 + 6.0
    fb.zero_()
    assert float(fb.flat.abs().sum()) == 0.0


def _world_one_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch.distributed as tdist
    from ggnn_amd.dist import FlatGradients, FlatTrainBuffer, all_reduce_sum, collectives_at_world_one, init_from_env
    r, w, _ = init_from_env(backend="gloo")      # explicit backend at WORLD_SIZE 1: a one-rank group
    ok = [tdist.is_initialized(), tdist.get_world_size() == 1, collectives_at_world_one()]
    fg = FlatGradients(8, 4, True)
    fg.flat.copy_(torch.arange(fg.flat.numel(), dtype=torch.float32) * 0.5)
    ref = fg.flat.clone()
    fg.all_reduce()
    fb = FlatTrainBuffer([torch.zeros(3, 5), torch.zeros(7)], n_sq=4, n_loss=2)
    fb.flat.normal_()
    ref2 = fb.flat.clone()
    ar = all_reduce_sum()
    ok += [ar is not None, torch.equal(fg.flat, ref)]
    ar(fb.flat)
    ok.append(torch.equal(fb.flat, ref2))
    tdist.barrier()
    tdist.destroy_process_group()
    q.put(ok)


def test_explicit_backend_at_world_one_runs_the_collectives():
    """init_from_env with an explicit backend at WORLD_SIZE 1 (bench.py
    --dist-backend nccl under a one-rank torchrun) creates the one-rank group
    and FlatGradients.all_reduce / all_reduce_sum issue their collective; the
    sum over one rank leaves every value unchanged (the GPU test runs the same
    calls over RCCL)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world_one_worker, args=(_free_port(), q))
    p.start()
    p.join(timeout=120)
    assert p.exitcode == 0
    assert q.get(timeout=5) == [True] * 6


def _schedule_worker(rank, world, port, diverge, q, drop_ids=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as tdist
    from ggnn_amd.dist import init_from_env
    init_from_env(backend="gloo")
    m, data = _golden_model()
    if drop_ids:           # a dataset without sentence ids: the digest keys on each element's content
        data = [{k: x for k, x in d.items() if k != "id"} for d in data]
    m.rank, m.world_size = rank, world
    if diverge and rank == 1:
        np.random.seed(123)
    sched = m.minibatch_schedule(m.process_raw_graphs(data, True), True)
    try:
        m._check_schedule_agrees(sched)
        q.put((rank, "ok"))
    except RuntimeError as e:
        q.put((rank, "raised" if "different minibatch schedules" in str(e) else repr(e)))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("drop_ids", [False, True])
@pytest.mark.parametrize("diverge", [False, True])
def test_ranks_check_that_their_schedules_agree(diverge, drop_ids):
    """The model seeds the global RNGs as the reference does
    (chem_tensorflow.py:174-175), so ranks draw the same schedule; run_epoch
    compares a digest of it across the ranks once per epoch and raises when a
    rank's shuffles differ (one collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_schedule_worker, args=(r, 2, port, diverge, q, drop_ids)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=5) for _ in range(2))
    assert got == {0: "raised", 1: "raised"} if diverge else got == {0: "ok", 1: "ok"}, got


def test_model_seeds_the_global_rngs_like_the_reference():
    import random
    np.random.seed(99)
    random.seed(99)
    _golden_model()                   # params random_seed = 0 (chem_tensorflow.py:174-175)
    a, b = np.random.rand(), random.random()
    np.random.seed(0)
    random.seed(0)
    assert (a, b) == (np.random.rand(), random.random())


# ---------------------------------------------------------------------------
# bench.py's own N-rank launch: `python bench.py --gpus N`
# without torch.distributed.run starts the N ranks itself
# ---------------------------------------------------------------------------
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=_ROOT, capture_output=True, text=True,
                          timeout=timeout, env=env)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_starts_its_own_ranks_without_torchrun(n):
    import json
    r = _bench(["--gpus", str(n), "--dist-backend", "gloo", "--launch-only"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["config"]["global_batch"] == 256 * n, res
    assert res["all_reduce"]["backend"] == "gloo" and res["launcher"] == "bench.py"
    # the strong-scaling split and the all-reduce's cost keys
    assert res["strong_scaling"]["per_rank_batch"] == 256 // n and res["strong_scaling"]["global_batch"] == 256, res
    ar = res["all_reduce"]
    assert ar["bytes"] == 3681280 and ar["isolated_ms_per_call"] > 0 and ar["bus_bandwidth_gbs"] > 0, ar
    assert ar["isolated_ms_per_call_min_rank"] <= ar["isolated_ms_per_call"], ar


def test_bench_refuses_a_world_size_that_disagrees_with_gpus():
    r = _bench(["--gpus", "2", "--launch-only"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode == 2 and "must agree" in r.stderr, (r.returncode, r.stderr[-2000:])


def test_bench_launcher_fails_when_a_rank_fails():
    """Ranks that cannot join (RCCL on a machine without a GPU) fail the whole
    job with a non-zero exit; no JSON line is relayed."""
    r = _bench(["--gpus", "2", "--dist-backend", "nccl", "--launch-only"], timeout=120)
    assert r.returncode != 0 and "exited with" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as tdist
    from ggnn_amd.dist import FlatTrainBuffer, all_reduce_sum, init_from_env
    init_from_env(backend="gloo")
    g = torch.Generator().manual_seed(100 + rank)
    params = [torch.zeros(s) for s in ((5, 7), (3,), (40, 6), (9, 2), (2,))]
    fb = FlatTrainBuffer(params, n_sq=3, n_loss=2, first=(3, 4), sparse=(2,))
    ff = FlatTrainBuffer(params, n_sq=3, n_loss=2)                        # the round-4 flat layout
    for a, b in zip(fb.grads + [fb.sq, fb.loss], ff.grads + [ff.sq, ff.loss]):
        x = torch.randn(a.shape, generator=g)
        a.copy_(x)
        b.copy_(x)
    r = all_reduce_sum()
    sparse_before = fb.grads[2].clone()
    h = r.start(fb.buckets[0])       # the heads bucket in flight while "the backward runs"
    r(fb.buckets[1])
    r.wait(h)
    r(ff.flat)
    dense_equal = all(torch.equal(a, b) for i, (a, b) in enumerate(zip(fb.grads, ff.grads)) if i != 2)
    ok = [dense_equal, torch.equal(fb.sq, ff.sq), torch.equal(fb.loss, ff.loss),
          torch.equal(fb.grads[2], sparse_before)]          # the sparse part is not all-reduced
    gathered = r.gather(torch.full((4,), float(rank)))
    ok.append(gathered.tolist() == [[0.0] * 4, [1.0] * 4])
    tdist.barrier()
    tdist.destroy_process_group()
    q.put((rank, ok))


def test_bucketed_reduction_equals_the_flat_one():
    """The data-parallel step's reduction as two buckets (heads + losses
    started asynchronously, then the rest of the dense part) sums exactly what
    one all-reduce of the round-4 flat buffer sums: bit for bit, two gloo
    ranks; the sparse region (the word table, reduced as IndexedSlices by the
    model) is left out of it; gather stacks the ranks in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get(timeout=5) for _ in range(2))
    assert got == {0: [True] * 5, 1: [True] * 5}, got
