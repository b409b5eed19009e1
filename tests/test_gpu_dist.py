"""The data-parallel path of the HIP engine itself, on the one GPU
of the test box: two ranks (child processes, gloo -- the driver's 8-GPU run
uses RCCL, one GPU per rank) each run libggnn.so's fwd + bwd on half of the
batch, all-reduce the flat gradient buffer once and apply ClipAdam with
grad_scale = 1/2.  The result must equal one process stepping the full batch.

Also rehearses bench.py's N > 1 path (torch.distributed.run, 2 ranks, gloo on
the one GPU): barrier, max-over-ranks timing, one JSON line from rank 0.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _adam_agreement(dp_params, full_params, dp_grads, full_grads, what):
    """Data parallel vs one process on the union batch, Adam at the
    reference's epsilon 1e-8 (chem_tensorflow.py:494).  The two are not bit
    for bit: the split-K chunking follows each rank's rows and each rank picks
    its backward's gradient scale from its own max |dL/dh_T|, so the gradients
    differ at the rounding level (<= 1e-4 of their max, asserted by the
    callers); Adam's g / (sqrt(v) + 1e-8) moves every weight by ~lr whatever
    its gradient's size, so an element whose gradient is itself at that
    rounding level can move differently by up to ~2 lr per step.  What must
    agree: every element whose gradient the two runs resolve to 1e-3 relative
    in every step (the weight gradients' single f16 operands round at ~5e-4)
    -- there the weights agree to lr x 1e-3 -- most elements are such; the
    others move by at most 2 lr per step apart (two steps, lr = 3e-3), and only
    a rare few by more than 1e-4 (measured: none before round 6; one element at
    2.1e-4 at config-3 shape after round 6 restored k_prop_bwd's W_c^T lo limb)."""
    lr, steps = 3e-3, 2
    dg = np.max(np.stack([np.abs(a - b) / np.maximum(np.abs(b), 1e-30) for a, b in zip(dp_grads, full_grads)]), 0)
    resolved = dg <= 1e-3
    diff = np.abs(dp_params - full_params)
    print("%s (Adam epsilon 1e-8): max param diff %.3g overall, %.3g where the gradient is resolved to 1e-3 "
          "(%d of %d elements), %d elements off by > 1e-4" % (what, diff.max(), diff[resolved].max(),
                                                               int(resolved.sum()), resolved.size,
                                                               int((diff > 1e-4).sum())))
    # resolved share: 0.95-0.99 before round 6's fp8 limb corrections in the
    # backward, 0.89 with them at config-3 shape (their rounding is relative to a
    # block's magnitude: small gradient elements carry more of it, and step 1
    # starts from weights one Adam step already moved apart)
    assert resolved.mean() >= 0.85, resolved.mean()
    assert diff[resolved].max() <= 3e-6, diff[resolved].max()
    assert diff.max() <= 2 * lr * steps, diff.max()
    assert (diff > 1e-4).mean() <= 1e-4, int((diff > 1e-4).sum())


@pytest.mark.parametrize("shape", ["8,64,128,4,3", "4,128,256,8,5"])
def test_two_rank_engine_step_equals_full_batch(tmp_path, shape):
    out = str(tmp_path / "dp.npz")
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_engine_worker.py"), out,
                                       shape], env=env, cwd=ROOT))
    codes = [p.wait(timeout=240) for p in procs]
    assert codes == [0, 0], codes
    d = np.load(out)
    # the all-reduced gradients equal the full batch's up to rounding: the
    # summation order differs, and each rank picks its backward's power-of-two
    # gradient scale from its own max |dL/dh_T| (ggnn_common.h gscale), so the
    # roundings at the bottom of the f16 / e5m2 ranges differ (the mode's own
    # error vs float64 is <= 1e-3).  Step 0 (same weights) is the equivalence
    # itself: measured 1.5-1.7e-7.  Step 1 starts from weights that one Adam
    # step already moved apart (elements whose gradient is at rounding level
    # move by ~lr either way, _adam_agreement): measured 4.7-6.7e-5 before
    # round 6's fp8 limb corrections in the backward, 0.7-1.6e-4 with them
    # (their rounding is relative to a block's magnitude, so small gradient
    # elements carry more of it).
    for s, bar in ((0, 1e-5), (1, 3e-4)):
        ref = d["full_grads"][s]
        err = np.abs(d["dp_grads"][s] - ref).max() / np.abs(ref).max()
        print("step %d: dp vs full gradients, max |diff| / max |full| = %.3g" % (s, err))
        assert err <= bar, (s, err)
    # and so do the weights after two clip + Adam steps at the reference's
    # epsilon 1e-8 (chem_tensorflow.py:494)
    step_dp = d["dp_params"] - d["init"]
    step_full = d["full_params"] - d["init"]
    assert np.abs(step_full).max() > 1e-4   # the weights did move
    _adam_agreement(d["dp_params"], d["full_params"], d["dp_grads"], d["full_grads"], "engine dp vs full")


def _spawn(script, args, tmp_path):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", script)] + args, env=env,
                                      cwd=ROOT))
    codes = [p.wait(timeout=300) for p in procs]
    assert codes == [0, 0], codes


@pytest.mark.parametrize("hidden", [128, 400])
def test_two_rank_btb_train_step_equals_union_batch(tmp_path, hidden):
    """The data-parallel training step of the WHOLE btb model (front-end,
    propagation, heads, clip + Adam; hidden 128 = specialised kernels, 400 =
    the general path): two ranks, each on one of two real dev batches of one
    bucket, one all-reduce of the flat buffer per step, equal one process
    stepping the concatenated batch -- the reference's loss over the union
    (chem_tensorflow.py:358-360,399-403) -- after two train_steps."""
    out = str(tmp_path / "dp_train.npz")
    _spawn("dist_train_worker.py", [out, str(hidden)], tmp_path)
    d = np.load(out)
    for s in range(2):
        ref = d["full_flat"][s]
        err = np.abs(d["dp_flat"][s] - ref).max() / np.abs(ref).max()
        assert err <= 1e-4, (s, err)                      # gradients, lookup norms, losses
    np.testing.assert_allclose(d["dp_loss"], d["full_loss"], rtol=1e-5)
    step_full = d["full_params"] - d["init"]
    assert np.abs(step_full).max() > 1e-4
    n = d["dp_params"].size
    _adam_agreement(d["dp_params"], d["full_params"], [f[:n] for f in d["dp_flat"]], [f[:n] for f in d["full_flat"]],
                    "btb dp vs union")
    # run_epoch with world_size 2: every batch of the single-process schedule
    # ran once (steps summed over the ranks), finite loss, LAS/UAS fractions
    tr_loss, tr_ips, tr_steps, tr_las, tr_uas, va_loss, va_ips, va_steps, va_las, va_uas, n_tr, n_va = d["epoch"]
    assert tr_steps == n_tr and va_steps == n_va
    assert np.isfinite(tr_loss) and np.isfinite(va_loss) and tr_ips > 0 and va_ips > 0
    assert 0 <= tr_las <= tr_uas <= 1 and 0 <= va_las <= va_uas <= 1


def test_bench_two_ranks_run_epoch_rehearsal():
    """bench.py's N-rank run_epoch line (the reference's own metric on its
    sentences, data parallel over every rank) under torch.distributed.run,
    2 ranks, gloo on the one GPU: what the driver's 8-GPU run executes."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--e2e-only", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    e2e = json.loads(lines[0])["end_to_end_run_epoch"]
    assert e2e["n_ranks"] == 2
    ep = e2e["epochs"][-1]
    assert ep["train_instances_per_sec"] > 0 and ep["valid_instances_per_sec"] > 0
    assert 0 < ep["valid_las"] <= ep["valid_uas"] <= 1 and ep["train_steps"] > 0


def test_bench_two_ranks_rehearsal():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--no-side", "--dist-backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "weak" and res["config"]["global_batch"] == 512
    assert res["value"] > 0 and "cpu_baseline" not in res


def test_bench_self_started_two_ranks():
    """`python bench.py --gpus 2` WITHOUT torch.distributed.run (how the driver
    starts the N = 1 line): bench.py starts both ranks itself (fresh child
    processes, before any GPU call in the parent), here as two gloo ranks on
    the one GPU, and relays rank 0's one JSON line with n_gpus = 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-side",
           "--dist-backend", "gloo", "--spawn-timeout", "240"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 512 and res["config"]["parallelism"] == "dp2"
    assert res["all_reduce"]["backend"] == "gloo" and res["value"] > 0
    # the strong leg (256 graphs split 128 per rank), the
    # all-reduce's event time and bus bandwidth, the min / max rank step
    st = res["strong_scaling"]
    assert st["per_rank_batch"] == 128 and st["global_batch"] == 256 and st["value"] > 0, st
    assert st["ms_per_step_min_rank"] <= st["ms_per_step"], st
    ar = res["all_reduce"]
    assert ar["in_step_ms"] > 0 and ar["isolated_ms_per_call"] > 0 and ar["bus_bandwidth_gbs"] > 0, ar
    assert ar["in_step_ms_min_rank"] <= ar["in_step_ms"], ar
    rs = res["rank_step_ms"]
    assert 0 < rs["min"] <= rs["max"] and abs(rs["max"] - res["ms_per_step"]) < 1e-9, rs


def test_two_rank_captured_step_returns_the_union_loss(tmp_path):
    """Edge-list feeds with hipGraph-captured steps at world size 2: the
    captured step's loss is summed inside the graph BEFORE the all-reduce,
    so the returned loss must be re-summed after it (the union-batch loss,
    chem_tensorflow.py:358-360,399-403), exactly as the eager path returns
    it; weights equal after three steps (the first batch of the shape runs
    its body eagerly, the second is captured, the third replays)."""
    out = str(tmp_path / "graph_loss.npz")
    _spawn("dist_graph_loss_worker.py", [out], tmp_path)
    d = np.load(out)
    assert int(d["uncaptured"]) == 1 and int(d["replayed"]) == 2 and int(d["eager_steps"]) == 3
    # the same launches in the same order, every reduction order-fixed: the
    # same bits (Adam at the reference's epsilon 1e-8)
    assert np.array_equal(d["graph_loss"], d["eager_loss"]), (d["graph_loss"], d["eager_loss"])
    assert float(d["param_diff"]) == 0.0


def test_sparse_word_reduction_matches_the_flat_one(tmp_path):
    """the data-parallel step's reduction as buckets (the
    heads' gradients and the losses started asynchronously before the
    propagation backward) plus the word table as IndexedSlices (the ranks'
    lookup rows all-gathered and summed in 64-bit fixed point) against the
    round-4 single all-reduce of the flat buffer, two gloo ranks on the GPU:
    every dense gradient, the losses and every non-word variable after Adam
    equal bit for bit; the word gradient and its lookup norm within fp32
    rounding (the flat path adds each rank's fp32 table, the sparse one
    converts the exact integer sum once); the sparse result identical on both
    ranks and equal to the fixed-point sum of the union's lookups."""
    out = str(tmp_path / "sparse.json")
    _spawn("dist_sparse_worker.py", [out], tmp_path)
    with open(out) as f:
        r = json.load(f)
    print("sparse word reduction:", r)
    assert r["sparse_layout"] and r["dense_grads_equal"] and r["loss_equal"] and r["params_equal_but_word"], r
    assert r["word_grad_rel"] <= 1e-6 and r["word_sq_rel"] <= 1e-5, r
    assert r["ranks_agree"] and r["union_recomputed_equal"] and r["lookups"] > 0, r
    # no reducer -> the word gradient is written densely (not stale);
    # a plain callable reducer sums the whole buffer like the dense layout
    assert r["local_step_word_grad_equal"] and r["local_step_params_equal"], r
    assert r["plain_callable_equals_dense"], r


def test_rccl_one_rank_group_runs_the_training_collectives(tmp_path):
    """The RCCL path an N-GPU run takes, executed on the test box's one GPU: a
    one-rank "nccl" group made exactly as dist.init_from_env makes it
    (device_id=), the per-step all-reduce of FlatGradients (bench.py's step)
    and of FlatTrainBuffer (train_step, eager and hipGraph-captured) issued
    through the same calls, values unchanged by the one-rank sum, then
    barrier and destroy."""
    out = str(tmp_path / "rccl.json")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_rccl_worker.py"), out], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    with open(out) as f:
        res = json.load(f)
    print("rccl one-rank:", res)
    assert res["backend"] == "nccl" and res["world"] == 1 and res["always"]
    assert res["flat_gradients_unchanged"] and res["all_reduce_sum_callable"]
    for tag in ("eager", "captured"):
        assert res[tag + "_train_buffer_unchanged"], tag
        la, l1 = res[tag + "_losses"]
        # a one-rank sum changes nothing and every reduction is order-fixed:
        # the two models stay bit-identical through Adam at epsilon 1e-8
        assert la == l1, (tag, la, l1)
        assert res[tag + "_param_max_diff"] == 0.0, (tag, res)
    assert res["captured_graph_stats"]["replayed"] == 2
    assert res["destroyed"]


def test_bench_one_rank_rccl_rehearsal():
    """bench.py under a one-rank torchrun with --dist-backend nccl: the
    one-rank RCCL group is created, the per-step all-reduce runs inside the
    timed loop, and the JSON line names the backend."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "1", "--steps", "3",
           "--warmup", "1", "--no-side", "--no-cpu-baseline", "--dist-backend", "nccl"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["value"] > 0
    assert res["all_reduce"]["backend"] == "nccl" and res["all_reduce"]["bytes_per_step"] > 0
    # the one-rank group still runs (and times) the collective; strong = weak at N = 1
    assert res["all_reduce"]["in_step_ms"] > 0 and res["all_reduce"]["isolated_ms_per_call"] > 0
    assert res["strong_scaling"]["per_rank_batch"] == 256 and res["strong_scaling"]["ms_per_step"] == res["ms_per_step"]
