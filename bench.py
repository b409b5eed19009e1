#!/usr/bin/env python3
"""Benchmark: GGNN propagation fwd+bwd, instances/sec (graphs/s).

Metric and config from BASELINE.json: hidden=256, v=128, e=4 edge types
(C = 2e = 8 adjacency channels), T=5, batch 256 graphs per GPU (configs[2]).
One "step" = one training step of the hot path over one batch already
resident in HBM: pack weights (fp32 -> MFMA fragment limbs) + stage adjacency
([b,C,v,v] fp32 -> 16-bit + transpose) + T-step forward + full backward (dL/dh0
and all six weight gradients) [+ one RCCL all-reduce of the flat gradient
buffer when N > 1] + the reference's optimizer update of the six variables
(per-tensor clip_by_norm + TF1 Adam, chem_tensorflow.py:494-503).
Weak scaling: every rank owns its own 256-graph batch; value = N*256 / t_step
with t_step the max over ranks.  Beside it (strong_scaling): one global batch
of 256 graphs split 256/N per rank, timed the same way; the per-step
all-reduce's time and bus bandwidth and the min / max rank step time.

Run:  python bench.py [--gpus N] [--steps K] [--warmup W]
      N > 1: one rank per GPU.  Under torch.distributed.run (WORLD_SIZE set)
      the ranks are torchrun's and WORLD_SIZE must equal N; started plainly,
      bench.py starts the N ranks itself (spawn_ranks: N fresh child
      processes, before this process imports torch or touches a GPU) and
      relays rank 0's JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CFG = dict(b=256, v=128, h=256, e=4, T=5)
BF16_DENSE_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16 / f16
HBM_PEAK_GBS = 8000.0


def flops_per_graph(v, h, C, T):
    """Algorithmic FLOPs per graph."""
    mt = 2 * v * h * h * C
    agg = 2 * v * v * C * h
    gru = 12 * v * h * h
    return dict(mt=mt, agg=agg, gru=gru, fwd=T * (mt + agg + gru), total=T * (2 * agg + 3 * mt + 3 * gru))


def kernel_algo_flops(kind, b, v, h, C, T):
    """Algorithmic FLOPs of ONE launch of a kernel kind at this config."""
    f = flops_per_graph(v, h, C, T)
    if kind in ("prop_fwd", "prop_bwd"):
        return b * (f["mt"] + f["agg"])
    if kind in ("gru_fwd", "gru_bwd"):
        return b * f["gru"]
    if kind == "fwd_fused":  # the whole T-step forward (messages + GRU) in one launch
        return b * f["fwd"]
    if kind == "wgrad":   # dW (MT-sized) + dWg, dWc (GRU-sized) over all T steps
        return T * b * (f["mt"] + f["gru"])
    return 0


def kernel_issued_flops(kind, b, v, h, C, T, precision):
    """MFMA FLOPs ONE launch actually issues.  fp32-parity splits every
    non-exact operand into f16 hi/lo limbs: 3 MFMA products per product, 2
    where the adjacency (exact 0/1) is one side (AGG), 1 for the weight
    gradients (single-limb operands); prop_bwd adds its dbeta product
    (dX^T . deg: one 32-column MFMA tile per channel over K = v, 2 limbs).
    Round 6: the backward's limb corrections run on the block-scaled fp8 MFMA,
    counted here in f16-equivalent cycles (one v_mfma_scale_f32_32x32x64 fp8 =
    two 32x32x16 f16): prop_bwd's dM W_c^T = hi x hi + both corrections = 2
    products, gru_bwd's dz W^T = hi x hi + e5m2 dz x e4m3 W_lo = 1.5 products.
    16-bit modes issue the algorithmic count."""
    f = flops_per_graph(v, h, C, T)
    if precision != "fp32":
        return kernel_algo_flops(kind, b, v, h, C, T)
    dbeta = 2 * 2 * v * 32 * h * C  # one 32-column MFMA tile per channel, K = v, 2 limbs
    if kind == "fwd_fused":
        return b * T * (3 * f["mt"] + 2 * f["agg"] + 3 * f["gru"])
    if kind == "prop_fwd":
        return b * (3 * f["mt"] + 2 * f["agg"])
    if kind == "prop_bwd":
        return b * (2 * f["mt"] + 2 * f["agg"] + dbeta)
    if kind == "gru_fwd":
        return 3 * b * f["gru"]
    if kind == "gru_bwd":   # f16 dz x f16 W + e5m2 dz x e4m3 W_lo (round 6): 1.5 products
        return 3 * b * f["gru"] // 2
    return kernel_algo_flops(kind, b, v, h, C, T)


def cpu_baseline(reps=5):
    """The oracle (numpy fp32 + OpenBLAS restatement of the reference math) on
    the host, SURVEY.md §8d: config 3 (fwd+bwd, the bench's workload) and
    config 2 (fwd only, its parity config), each the median of `reps` timed
    repetitions after one warm-up, on every core this process may use and on
    one core.  The thread count is the process's CPU affinity set, capped at
    OMP_NUM_THREADS (the box's CPU share for one GPU; the box's `nproc` counts
    the whole host, which other jobs share)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ggnn_oracle as O
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        affinity = nproc
    omp = os.environ.get("OMP_NUM_THREADS")
    cores = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity

    def run(threads, cfg, gb, backward):
        b_, v, h, C, T = gb, cfg["v"], cfg["h"], 2 * cfg["e"], cfg["T"]
        A, h0 = O.synthetic_batch(b_, v, h, C, seed=1)
        w = O.synthetic_weights(h, C, seed=1, parity_bias=False)
        dhT = np.ones_like(h0)
        ctx = threadpool_limits(limits=threads) if threadpool_limits else None
        try:
            times = []
            for i in range(reps + 1):  # one warm-up, then `reps` timed
                t0 = time.perf_counter()
                hT, caches = O.forward(A, h0, w, T)
                if backward:
                    O.backward(A, dhT, caches, w)
                if i:
                    times.append(time.perf_counter() - t0)
        finally:
            if ctx is not None and hasattr(ctx, "restore_original_limits"):
                ctx.restore_original_limits()
        med = float(np.median(times))
        return dict(value=gb / med, unit="graphs/s", cores=threads,
                    sample="oracle fp32 numpy %s, %d-graph batch (v=%d h=%d C=%d T=%d), median of %d after 1 warm-up "
                           "(%.3f s per batch)" % ("fwd+bwd" if backward else "fwd", gb, v, h, C, T, reps, med))

    c3 = dict(CFG)
    c2 = dict(b=32, v=64, h=128, e=2, T=3)
    main_leg = run(cores, c3, 64, True)
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    # BASELINE.md §2 asks for all cores: every CPU of the affinity set too
    # (on the shared GPU box that is the whole host, which other jobs use)
    all_leg = run(affinity, c3, 64, True) if affinity > cores else None
    return dict(main_leg, kind="port", cpu_model=model, nproc=nproc, affinity_cpus=affinity,
                omp_num_threads=omp, all_affinity_cpus=all_leg,
                single_core=run(1, c3, 4, True),
                config2_fwd=run(cores, c2, c2["b"], False),
                config2_fwd_single_core=run(1, c2, c2["b"], False))


def adjacency_feed_costs(eng, b, v, E, dev, reps=5):
    """Side measurement (SURVEY §8f compact adjacency producer): staging one
    batch of dependency-tree-shaped graphs (v-1 labelled edges each) from the
    reference's dense [b, 2E, v, v] feed (host copy + ggnn_set_adjacency) vs
    from edge lists (ggnn_set_adjacency_edges)."""
    import torch
    import ggnn_oracle as O
    rng = np.random.default_rng(5)
    graphs = []
    for _ in range(b):
        dst = np.arange(1, v)
        src = np.array([rng.integers(0, i) for i in dst])       # a random tree: head before dependent
        lab = rng.integers(1, E + 1, v - 1)
        graphs.append(np.stack([src, lab, dst], 1).tolist())
    A = np.stack([O.graph_to_adj_mat_bd(g, v, E) for g in graphs]).astype(np.float32)
    A_host = torch.from_numpy(A)
    A_dev = A_host.to(dev)
    e_np = np.concatenate([np.asarray(g, np.int32) for g in graphs])
    offs = np.arange(0, b * (v - 1) + 1, v - 1, dtype=np.int32)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    ms_dense_dev = timed(lambda: eng.set_adjacency(A_dev))
    ms_dense_h2d = timed(lambda: eng.set_adjacency(A_host.to(dev)))
    ms_edges_h2d = timed(lambda: eng.set_adjacency_edges(
        (torch.from_numpy(e_np).to(dev), torch.from_numpy(offs).to(dev)), v, E))
    return {"graphs": "random dependency trees, v-1 edges each", "dense_bytes": int(A.nbytes),
            "edge_bytes": int(e_np.nbytes + offs.nbytes),
            "dense_in_hbm_ms": ms_dense_dev, "dense_from_host_ms": ms_dense_h2d, "edges_from_host_ms": ms_edges_h2d}


def _timed_events(fn, reps):
    """Mean ms of fn() over reps runs on the current stream (HIP events)."""
    import torch
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def callers_side(dev, b, v, h, reps=10):
    """Side measurement: the btb front-end (embedding
    lookups + dropout, fwd+bwd) and both output heads (logits GEMM, softmax,
    cross-entropy, dW/db/dX) at the bench's b, v, h.  The reference's
    80+50+100+80 = 310-wide concat does not fit hidden 256, so the
    tables are 64/32/96/64 wide here; heads o = 150 (output_size) and 46
    (output_size_edges of the WSJ std->nivre lists)."""
    import torch
    from ggnn_amd.heads import EmbeddingFrontEnd, OutputHeads
    rng = np.random.default_rng(11)
    mk = lambda *s: torch.from_numpy(rng.uniform(-0.1, 0.1, s).astype(np.float32)).to(dev)
    loc, pos, word = mk(150, 64), mk(46, 32), mk(40000, 96)
    segs = [(loc, 0), (pos, 1), (word, 2), (loc, 3)]
    wi = torch.from_numpy(np.stack([rng.integers(0, 150, (b, v)), rng.integers(0, 46, (b, v)),
                                    rng.integers(0, 40000, (b, v)), rng.integers(0, 150, (b, v))],
                                   2).astype(np.int32)).to(dev)
    fe, oh = EmbeddingFrontEnd(h), OutputHeads(h)
    heads = [(mk(2 * h, 150), mk(150)), (mk(2 * h, 46), mk(46))]
    labels = []
    for o in (150, 46):
        y = np.zeros((b, v, o), np.float32)
        y[np.arange(b)[:, None], np.arange(v)[None, :], rng.integers(0, o, (b, v))] = 1
        labels.append(torch.from_numpy(y).to(dev))
    hT, h0 = mk(b, v, h), mk(b, v, h)
    dh0 = mk(b, v, h)
    shared = torch.empty_like(loc)
    dt = [shared, torch.empty_like(pos), torch.empty_like(word), shared]
    state = {}

    def heads_fb():
        probs, _ = oh.forward(hT, h0, heads, labels, 0.85, 3, float(b))
        oh.backward(hT, h0, heads, labels, probs, float(b))

    ms_embed = _timed_events(lambda: (fe.forward(segs, wi, 0.55, 5), fe.backward(segs, wi, dh0, 0.55, 5, dtables=dt)),
                             reps)
    ms_heads = _timed_events(heads_fb, reps)
    flops = 3 * 2 * b * v * 2 * h * (150 + 46)      # logits, dX, dW GEMMs
    return {"embed_fwd_bwd_ms": ms_embed, "heads_fwd_bwd_ms": ms_heads,
            "heads_gemm_tflops_algorithmic": flops / (ms_heads * 1e-3) / 1e12,
            "note": "heads: both heads' logits, d[hT|h0] and dW as one MFMA product each (k_gemm_ring, split f16 "
                    "limbs = fp32 parity) + softmax / dZ kernels; fwd+bwd incl. weight dropout; tables 64/32/96/64 "
                    "wide, heads o=150 and 46"}


def precision_error(dev, precision, host, T):
    """The mode's measured error against the float64 reference on a slice of
    the bench's own batch (configs[2] data, T = 5): forward h_T and every
    gradient, normalised RMS and max |err| (north_star: 1e-2 for 16-bit;
    tests/test_precision_policies.py shows why bf16 cannot meet it on this
    data and test_gpu_parity.py::test_fp16_within_1e_2_rms_on_config3_t5 pins
    the f16 mode)."""
    import torch
    import ggnn_oracle as O
    from ggnn_amd.engine import PropagationEngine
    A, h0, w = host
    b, C, v, _ = A.shape
    h = h0.shape[-1]
    dhT = np.random.default_rng(3).standard_normal(h0.shape).astype(np.float32)
    A64, w64 = A.astype(np.float64), {k: x.astype(np.float64) for k, x in w.items()}
    ref, caches = O.forward(A64, h0.astype(np.float64), w64, T)
    gref = O.backward(A64, dhT.astype(np.float64), caches, w64)
    eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=precision)
    pack = eng.pack_weights({k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}, T=T)
    eng.set_adjacency(torch.from_numpy(np.ascontiguousarray(A)).to(dev))
    got = eng.forward(torch.from_numpy(np.ascontiguousarray(h0)).to(dev), pack, T, training=True).cpu().numpy()
    g = eng.backward(torch.from_numpy(dhT).to(dev))
    nr = lambda x, r: float(np.sqrt(np.mean((x - r) ** 2)) / np.sqrt(np.mean(r ** 2)))
    out = {"slice": "%d graphs of the bench batch, T=%d" % (b, T), "hT_nrms": nr(got, ref),
           "hT_max_abs": float(np.abs(got - ref).max())}
    out["grads_nrms"] = {k: nr(g[k].cpu().numpy().reshape(gref[k].shape), gref[k]) for k in gref}
    return out


def strong_split_side(dev, A, h0, dhT, w_d, v, h, C, T, precision, steps=20):
    """Side measurement (rank 0 at N = 1): the step on 256/N graphs -- the
    per-rank work of the strong-scaling leg at N = 2, 4, 8 -- on this one GPU,
    without the all-reduce: the strong-scaling curve's compute part.  One
    workgroup per graph in the fused forward and k_prop_bwd means a batch
    below 256 graphs leaves CUs idle, so this is where strong scaling stops."""
    import torch
    from ggnn_amd.dist import FlatGradients
    from ggnn_amd.engine import PropagationEngine
    res = {}
    for n in (2, 4, 8):
        bs = A.shape[0] // n
        eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=precision)
        grads = FlatGradients(h, C, True, device=dev)
        gv = dict(grads.views)
        gv["h0"] = torch.empty((bs, v, h), dtype=torch.float32, device=dev)
        out = torch.empty((bs, v, h), dtype=torch.float32, device=dev)
        A_s, h0_s, d_s = (torch.from_numpy(np.ascontiguousarray(x[:bs])).to(dev) for x in (A, h0, dhT))

        def step():
            pack = eng.pack_weights(w_d, T=T)
            eng.set_adjacency(A_s)
            eng.forward(h0_s, pack, T, training=True, out=out)
            eng.backward(d_s, gv)

        ms = _timed_events(step, steps)
        res["n%d" % n] = {"per_rank_batch": bs, "ms_per_step": ms, "graphs_per_s_per_gpu": bs / (ms * 1e-3)}
        del eng, grads, gv, out, A_s, h0_s, d_s
        torch.cuda.empty_cache()
    res["note"] = ("fwd+bwd of 256/N graphs on one GPU (no optimizer, no all-reduce): the per-rank compute of the "
                   "strong-scaling leg; strong-scaling speedup <= 256-graph step / this step")
    return res


def gru_inference_leg(eng, h0_d, w_d, A_d, b, v, h, C, T, precision, steps=10):
    """The unfused forward in inference mode (training=False: no saves for the
    backward), k_gru_fwd timed per launch with HIP events.  SURVEY §8(d)'s GRU
    bytes -- X, h in + h' out, fp32: 12 v h per graph-step -- are the contract
    north_star's ">= 50 % of HBM peak on the fused GRU" is quoted on (25.2 us
    per timestep at config 3); traffic: PMC bytes per launch of the same
    inference-only launches (tools/gru_infer_probe.py under rocprofv3 --pmc,
    profiles/pmc_traffic_<precision>_infer.json)."""
    import torch
    from ggnn_amd import _lib
    out = torch.empty((b, v, h), dtype=torch.float32, device=h0_d.device)
    pack = eng.pack_weights(w_d, T=T)
    eng.set_adjacency(A_d)

    def fwd():
        eng.forward(h0_d, pack, T, training=False, out=out)

    ms = _timed_events(fwd, steps)
    timer = _lib.KernelTimer(max_launches=50 * steps)
    with timer:
        for _ in range(steps):
            fwd()
        torch.cuda.synchronize()
    res = {"ms_per_forward": ms, "graphs_per_s": b / (ms * 1e-3), "kernels": {}}
    tr = load_traffic(precision + "_infer") or {}
    for k in ("prop_fwd", "gru_fwd"):
        if not timer.launches.get(k):
            continue
        avg = timer.total_ms[k] / timer.launches[k]
        fl = kernel_algo_flops(k, b, v, h, C, T)
        d = {"avg_launch_ms": avg, "launches_per_forward": timer.launches[k] / steps,
             "frac_of_bf16_peak": fl / (avg * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS}
        if k == "gru_fwd":
            ab = 12 * v * h * b
            d.update(algorithmic_bytes_per_launch=ab,
                     frac_of_hbm_peak_algorithmic=ab / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     north_star_us_per_timestep_at_half_peak=ab / (0.5 * HBM_PEAK_GBS * 1e9) * 1e6)
        kt = tr.get("kernels", {}).get(k)
        if kt:
            gbs = kt["hbm_bytes_per_launch"] / (avg * 1e-3) / 1e9
            d.update(traffic=kt["hbm_bytes_per_launch"], hbm_read_bytes=kt["hbm_read_bytes"],
                     hbm_write_bytes=kt["hbm_write_bytes"], hbm_gbs=gbs, frac_of_hbm_peak=gbs / HBM_PEAK_GBS,
                     frac_roofline=max(d["frac_of_bf16_peak"], gbs / HBM_PEAK_GBS),
                     traffic_source="profiles/pmc_traffic_%s_infer.json" % precision)
        res["kernels"][k] = d
    return res


def precision_side(dev, precision, A_d, h0_d, w_d, dhT, b, v, h, C, T, steps=10, unfused=False, host=None):
    """The same fwd+bwd step in a reduced-precision mode (single 16-bit MFMA
    operands): graphs/s and the prop kernels' fraction of the dense bf16 MFMA
    peak (north_star's >= 30 % target is quoted on bf16 tiles).  unfused: the
    forward as separate k_prop_fwd + k_gru_fwd launches (GGNN_UNFUSED_FWD), the
    kernels north_star's adj x h and fused-GRU targets name."""
    import torch
    from ggnn_amd import _lib
    from ggnn_amd.dist import FlatGradients
    from ggnn_amd.engine import PropagationEngine
    eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=precision, unfused_forward=unfused)
    grads = FlatGradients(h, C, True, device=dev)
    gv = dict(grads.views)
    gv["h0"] = torch.empty((b, v, h), dtype=torch.float32, device=dev)
    out = torch.empty((b, v, h), dtype=torch.float32, device=dev)

    def step():
        pack = eng.pack_weights(w_d, T=T)
        eng.set_adjacency(A_d)
        eng.forward(h0_d, pack, T, training=True, out=out)
        eng.backward(dhT, gv)

    ms = _timed_events(step, steps)
    timer = _lib.KernelTimer(max_launches=200 * steps)
    with timer:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    fr = {}
    tr = load_traffic(precision) or {}
    for k in ("fwd_fused", "prop_fwd", "prop_bwd", "gru_fwd", "gru_bwd", "wgrad"):
        if timer.launches.get(k):
            avg = timer.total_ms[k] / timer.launches[k]
            fl = kernel_algo_flops(k, b, v, h, C, T)
            d = {"avg_launch_ms": avg, "tflops": fl / (avg * 1e-3) / 1e12,
                 "frac_of_bf16_peak": fl / (avg * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS}
            if k == "gru_fwd":
                # SURVEY §8(d)'s algorithmic GRU bytes: X, h in + h' out as fp32
                # (12 v h b) plus the saved r, u, c (12 v h b) -- the contract's
                # bytes, not the kernel's own traffic
                ab = 24 * v * h * b
                d.update(algorithmic_bytes_per_launch=ab,
                         frac_of_hbm_peak_algorithmic=ab / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS)
            kt = tr.get("kernels", {}).get(k)
            if kt:
                # PMC HBM bytes per launch (profiles/pmc_traffic_<precision>.json);
                # a kernel's roofline fraction is max(F/P_mfma, B/P_hbm)
                gbs = kt["hbm_bytes_per_launch"] / (avg * 1e-3) / 1e9
                d.update(traffic=kt["hbm_bytes_per_launch"], hbm_gbs=gbs, frac_of_hbm_peak=gbs / HBM_PEAK_GBS,
                         frac_roofline=max(d["frac_of_bf16_peak"], gbs / HBM_PEAK_GBS),
                         traffic_source="profiles/pmc_traffic_%s.json" % precision)
            fr[k] = d
    out = {"precision": precision, "value": b / (ms * 1e-3), "unit": "graphs/s", "ms_per_step": ms,
           "step": "pack + adjacency + fwd + bwd (no optimizer)", "kernels": fr}
    if unfused:
        out["inference"] = gru_inference_leg(eng, h0_d, w_d, A_d, b, v, h, C, T, precision, steps)
    if host is not None:
        out["error_vs_float64"] = precision_error(dev, precision, host, T)
    if not unfused:
        u = precision_side(dev, precision, A_d, h0_d, w_d, dhT, b, v, h, C, T, steps, unfused=True)
        out["unfused_forward"] = {"value": u["value"], "ms_per_step": u["ms_per_step"],
                                  "kernels": {k: u["kernels"][k] for k in ("prop_fwd", "gru_fwd") if k in u["kernels"]},
                                  "inference": u["inference"],
                                  "note": "the forward as per-timestep k_prop_fwd + k_gru_fwd launches "
                                          "(GGNN_UNFUSED_FWD): north_star's adj x h (>= 30 % of bf16 MFMA peak) "
                                          "and fused-GRU (>= 50 % of HBM peak) targets are quoted on these kernels"}
    return out


def tree_pair_count(graphs, v, E):
    """(node, channel) pairs with an incoming edge (graph_to_adj_mat_bd's four
    entries per edge, distinct per receiving row and channel): the rows pair
    mode (GGNN_SPARSE_PAIRS) runs the message transform over."""
    pairs = 0
    for g in graphs:
        s = set()
        for src, lab, dst in g:
            prv = dst - 1 if dst >= 1 else v - 1
            s.update(((dst, lab - 1), (src, lab - 1 + E), (dst, E - 1), (prv, 2 * E - 1)))
        pairs += len(s)
    return pairs


def real_density_side(dev, b=256, v=30, h=256, E=46, T=5, steps=5, both=True):
    """Side measurement (SURVEY §8f rank 3 / configs[4] shapes): the fwd+bwd
    step on dependency-tree graphs with the real btb label set (std->nivre,
    E = 46 -> C = 92 channels, most of them empty per graph), with empty-channel
    skipping on (the default) and off (GGNN_DENSE_CHANNELS).  Sentence-sized
    graphs (the real dev set: mean 24.6 nodes; bucket v <= 32),
    n ~ U{v/2..v} nodes, random heads before dependents, Zipf-like labels
    (P(label k) ~ 1/k: a few labels such as punct/nsubj/det dominate a treebank).
    both: also the reference's own model (hidden 400, T = 4) on the general
    path, in pair mode (GGNN_SPARSE_PAIRS, the default for edge-list batches)
    and with the dense (graph, channel) tiles, each with its algorithmic rate."""
    import torch
    from ggnn_amd.dist import FlatGradients
    from ggnn_amd.engine import PropagationEngine
    import ggnn_oracle as O
    rng = np.random.default_rng(13)
    C = 2 * E
    pz = 1.0 / np.arange(1, E + 1)
    pz /= pz.sum()
    graphs = []
    for _ in range(b):
        n = int(rng.integers(v // 2, v + 1))
        graphs.append([(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)])
    occ = [int((O.graph_to_adj_mat_bd(g_, v, E, dtype=np.float32).reshape(C, -1).max(1) > 0).sum()) for g_ in graphs]
    pairs = tree_pair_count(graphs, v, E)
    w = O.synthetic_weights(h, C, seed=3)
    w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    h0 = torch.from_numpy(rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)).to(dev)
    dhT = torch.from_numpy(rng.standard_normal((b, v, h)).astype(np.float32)).to(dev)
    res = {"workload": "b=%d dependency trees, v=%d, hidden=%d, E=%d (C=%d), T=%d, fwd+bwd" % (
        b, v, h, E, C, T), "nonempty_channels_per_graph_mean": float(np.mean(occ)),
        "pairs_per_node": pairs / float(b * v)}
    # algorithmic work of the re-associated contraction (per step, fwd + bwd):
    # MT over the pair rows 2 P h^2 (x3: fwd, dY, dW), GRU 12 N h^2 (x3), the
    # adjacency sums (gather / scatter of rows) are not MFMA work
    N = b * v
    algo = T * (3 * 2 * pairs * h * h + 3 * 12 * N * h * h)
    # SURVEY §8(d)'s per-graph formula over each graph's non-empty channels
    # (the count the round-2 verdict quoted): T (2 AGG + 3 MT + 3 GRU)
    survey = sum(T * (2 * 2 * v * v * ch * h + 3 * 2 * v * h * h * ch + 3 * 12 * v * h * h) for ch in occ)
    variants = (("skip", dict()), ("dense", dict(skip_empty_channels=False))) if both else ()
    if h not in (128, 256):
        variants = ()
    variants += tuple(((("pairs", dict(sparse_pairs=True)), ("tiles", dict(sparse_pairs=False, force_generic=True)))
                       if h % 4 == 0 and not both else ()))
    for name, kw in variants:
        eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision="fp32", **kw)
        eng.set_adjacency_edges(graphs, v, E)
        grads = FlatGradients(h, C, True, device=dev)
        gv = dict(grads.views)
        gv["h0"] = torch.empty((b, v, h), dtype=torch.float32, device=dev)
        out = torch.empty((b, v, h), dtype=torch.float32, device=dev)

        def step():
            pack = eng.pack_weights(w_d, T=T)
            eng.forward(h0, pack, T, training=True, out=out)
            eng.backward(dhT, gv)

        ms = _timed_events(step, steps)
        r = {"ms_per_step": ms, "graphs_per_s": b / (ms * 1e-3)}
        if name == "pairs":
            # the training feed the reference uses: keep 0.9 for both the edge-weight
            # and the state dropout (chem_tensorflow_dense.py:155-159, 860-861)
            nd = [0]

            def step_drop(keep=0.9):
                nd[0] += 1
                pack = eng.pack_weights(w_d, T=T, edge_keep=keep, seed=nd[0])
                eng.forward(h0, pack, T, training=True, out=out, state_keep=keep)
                eng.backward(dhT, gv)

            msd = _timed_events(step_drop, steps)
            r["training_dropout"] = {"edge_keep": 0.9, "state_keep": 0.9, "ms_per_step": msd,
                                     "graphs_per_s": b / (msd * 1e-3)}
        if name in ("pairs", "tiles"):
            tf = algo / (ms * 1e-3) / 1e12
            ts = survey / (ms * 1e-3) / 1e12
            r.update(algorithmic_tflops=tf, frac_of_bf16_peak=tf / BF16_DENSE_PEAK_TFLOPS,
                     survey_formula_tflops=ts, survey_formula_frac_of_bf16_peak=ts / BF16_DENSE_PEAK_TFLOPS)
        res[name] = r
        del eng, grads, gv, out
        torch.cuda.empty_cache()
    if both:
        res["speedup"] = res["dense"]["ms_per_step"] / res["skip"]["ms_per_step"]
        # the reference's own model on these graphs: hidden_size 400, num_timesteps 4
        # (chem_tensorflow.py:95-96, configs[0] / configs[4]), general path
        r4 = real_density_side(dev, b, v, 400, E, 4, steps, both=False)
        res["reference_defaults_h400_T4"] = {
            "workload": r4["workload"], **r4["pairs"], "pair_mode": "GGNN_SPARSE_PAIRS",
            "dense_tiles": r4["tiles"], "pairs_per_node": r4["pairs_per_node"],
            "algorithmic_work": "T*(3*2*P*h^2 + 3*12*N*h^2), P = (node, channel) pairs with an incoming edge, "
                                "N = b*v rows (the re-associated contraction); survey_formula_*: SURVEY §8d's "
                                "T*(2 AGG + 3 MT + 3 GRU) per graph over its non-empty channels (every row of "
                                "every non-empty tile, the work the dense-tile loop does)"}
    return res


def end_to_end_side(dev, rank=0, world=1, epochs=1, restrict=True):
    """Side measurement (SURVEY §8f rank 4 / configs[0] / configs[4]): the
    reference's own metric, instance_per_sec of run_epoch
    (chem_tensorflow.py:528-667, :660) -- host batching in a background thread,
    train step (front-end, propagation, heads, clip + Adam) or eval forward,
    host LAS/UAS per batch -- with the reference's default params
    (hidden_size 400, num_timesteps 4, batch_size 20, embeddings 80/50/100/80,
    std -> nivre: C = 92 channels, 12 output labels) on the reference's OWN
    sentences in its --train_with_dev mode (chem_tensorflow.py:36-45): train on
    the 1700 std dev sentences, validate on the 2416 std test sentences
    (data/, written from the reference's JSON; the train split is absent).
    One warm-up epoch, then `epochs` timed train + valid epochs.  With
    world > 1 every rank runs it: data-parallel run_epoch (rank-sharded
    bucketed batches, one RCCL all-reduce of the whole model's flat gradient
    buffer per global step), so the value is the N-rank job's instances/sec.
    restrict: also the README's sample run (--restrict_data 100, epoch 1 of a
    fresh model, train + valid; README.md:25-43)."""
    from ggnn_amd import _lib
    from ggnn_amd.batching import TRAIN_WITH_DEV, wsj_model_sizes
    from ggnn_amd.model import DenseGGNNChemModel

    def fresh(graphs=True):
        np.random.seed(0)                      # chem_tensorflow.py:175
        return DenseGGNNChemModel(params={"compact_adjacency": True, "hip_graphs": graphs}, seed=0, device=dev,
                                  rank=rank, world_size=world, **wsj_model_sizes())

    m = fresh()
    t0 = time.perf_counter()
    train = m.load_data(TRAIN_WITH_DEV["train_file"], True)
    valid = m.load_data(TRAIN_WITH_DEV["valid_file"], False)
    load_s = time.perf_counter() - t0
    # warm-up: every shape's first batch runs eagerly, its second is captured
    # (ggnn_amd/graphs.py); a training run of the reference's 200 epochs is
    # in this steady state from epoch 2 on
    for _ in range(2):
        m.run_epoch("warm-up", train, True)
        m.run_epoch("warm-up", valid, False)
    res = {"params": {k: m.params[k] for k in ("hidden_size", "num_timesteps", "batch_size")},
           "data": "WSJ std->nivre btb, --train_with_dev: train = std dev (1700 sentences), valid = std test (2416)",
           "n_ranks": world, "load_and_process_s": load_s, "epochs": [],
           "step": "hipGraph-captured per batch shape (one H2D copy + one graph launch per batch; "
                   "all-reduce and Adam eager when n_ranks > 1)"}
    for e in range(epochs):
        s0 = dict(m.graph_stats)
        tr = m.run_epoch("train", train, True)
        s1 = dict(m.graph_stats)
        va = m.run_epoch("valid", valid, False)
        s2 = dict(m.graph_stats)
        res["epochs"].append({"train_instances_per_sec": tr[3], "train_steps": tr[4], "train_loss": tr[0],
                              "train_las": tr[5], "train_uas": tr[6], "train_uas_e": tr[16],
                              "valid_instances_per_sec": va[3], "valid_loss": va[0], "valid_las": va[5],
                              "valid_uas": va[6], "valid_uas_e": va[16],
                              "train_batches_by_path": {k: s1[k] - s0[k] for k in s0},
                              "valid_batches_by_path": {k: s2[k] - s1[k] for k in s1}})
    res.update({k: res["epochs"][-1][k] for k in ("train_instances_per_sec", "valid_instances_per_sec",
                                                   "valid_las", "valid_uas")})
    import torch
    res["device_memory"] = {"peak_reserved_gb": torch.cuda.max_memory_reserved(dev) / 2 ** 30,
                            "peak_allocated_gb": torch.cuda.max_memory_allocated(dev) / 2 ** 30,
                            "captured_steps": len(m._graphs), "captured_steps_gb": m.graph_stats["cache_bytes"] / 2 ** 30,
                            "cache_budget_gb": m.params["hip_graph_cache_mb"] / 1024,
                            "note": "peak over the warm-up and timed epochs of the captured-step model (process "
                                    "totals: the bench's earlier lines included)"}
    # the same epochs on the eager path (every library call launched from the
    # host): the graphs' gain, and the launches per batch they replace
    me = fresh(graphs=False)
    np.random.seed(1)
    train_e = me.load_data(TRAIN_WITH_DEV["train_file"], True)
    valid_e = me.load_data(TRAIN_WITH_DEV["valid_file"], False)
    timer = _lib.KernelTimer(max_launches=400000)
    with timer:
        wt = me.run_epoch("warm-up", train_e, True)
        wv = me.run_epoch("warm-up", valid_e, False)
    tr_e = me.run_epoch("train", train_e, True)
    va_e = me.run_epoch("valid", valid_e, False)
    res["eager_step"] = {"train_instances_per_sec": tr_e[3], "valid_instances_per_sec": va_e[3],
                         "library_launches_per_batch": sum(timer.launches.values()) / max(wt[4] + wv[4], 1),
                         "note": "params['hip_graphs'] = False; launches counted over one train + one valid "
                                 "epoch (kernels, fills and copies of libggnn; plus the host-side uploads)"}
    if restrict:
        # README.md:25-43's sample run: --restrict_data 100 (100 sentences per
        # split: small bucketed batches), epoch 1 of a fresh model (cold: the
        # first batch of every bucket shape allocates its workspace)
        m2 = fresh()
        small = m2.load_data(TRAIN_WITH_DEV["train_file"], True, restrict=100)
        small_v = m2.load_data(TRAIN_WITH_DEV["valid_file"], False, restrict=100)
        tr100 = m2.run_epoch("train r100", small, True)
        va100 = m2.run_epoch("valid r100", small_v, False)
        res["restrict_data_100_epoch1"] = {
            "train_instances_per_sec": tr100[3], "train_steps": tr100[4], "avg_train_batch": 100 / max(tr100[4], 1),
            "train_las_uas_uas_e": [tr100[5], tr100[6], tr100[16]],
            "valid_instances_per_sec": va100[3], "valid_las_uas_uas_e": [va100[5], va100[6], va100[16]],
            "reference_readme": {"train_instances_per_sec": 13.91, "valid_instances_per_sec": 31.51,
                                 "train_las_uas_uas_e": [0.106, 0.147, 0.576],
                                 "valid_las_uas_uas_e": [0.191, 0.232, 0.750],
                                 "hardware": "unstated (BASELINE.md §1)"}}
    res["note"] = ("the reference's run_epoch metric (host batching + LAS/UAS included), not the hot-path value; "
                   "dropout as the reference feeds it in training (0.9 / 0.55 / 0.85), none in validation")
    return res


def load_ceilings():
    """Library MFMA / copy ceilings measured on the box (tools/ceilings.py)."""
    p = os.path.join(ROOT, "profiles", "ceilings.json")
    try:
        with open(p) as f:
            return json.load(f)
    except Exception:
        return None


def load_traffic(precision="fp32"):
    """Per-launch HBM bytes per kernel kind from the committed PMC summary of
    this precision mode (tools/pmc_profile.sh)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json" if precision == "fp32" else
                     "pmc_traffic_%s.json" % precision)
    if os.path.exists(p):
        try:
            with open(p) as f:
                return json.load(f)
        except Exception:
            return None
    return None


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int, argv, timeout_s: float | None = None) -> int:
    """Start an n-rank job of this script: n child processes with RANK /
    LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set
    as torch.distributed.run sets them (one node, rendezvous on 127.0.0.1), one
    rank per GPU.  The parent never imports torch and never touches a GPU (the
    children are fresh processes, not forks or execs of an initialised one).
    Rank 0's stdout (the JSON line) is relayed to stdout; the other ranks'
    stdout goes to stderr; stderr is inherited.  If a rank fails, the others
    are terminated and the exit code is the first failure's (else 0).
    Replaces the reference's unused tf.distribute.MirroredStrategy
    (chem_tensorflow_dense.py:1327-1328) with N processes over RCCL."""
    import subprocess
    import threading
    port = _free_port()
    procs, pumps = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                             stdout=subprocess.PIPE, text=True, bufsize=1)
        sink = sys.stdout if r == 0 else sys.stderr

        def pump(pp=p, out=sink):
            for line in pp.stdout:
                out.write(line)
                out.flush()
        th = threading.Thread(target=pump, daemon=True)
        th.start()
        procs.append(p)
        pumps.append(th)
    t_end = None if timeout_s is None else time.monotonic() + timeout_s
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print("bench.py: rank %d exited with %d; stopping the other ranks" % (r, c), file=sys.stderr)
                for q in live:
                    procs[q].terminate()
        if t_end is not None and time.monotonic() > t_end and live:
            print("bench.py: ranks %s still running after %.0f s; stopping them" % (sorted(live), timeout_s),
                  file=sys.stderr)
            for q in live:
                procs[q].terminate()
            rc = rc or 124
            t_end = None
        time.sleep(0.05)
    for th in pumps:
        th.join(timeout=5)
    return rc


def strong_batch(world: int) -> int:
    """Per-rank batch of the strong-scaling leg: the
    global batch of configs[2] (256 graphs) split evenly over the ranks."""
    if CFG["b"] % world:
        raise SystemExit("bench.py: the strong-scaling leg splits b=%d over %d ranks evenly" % (CFG["b"], world))
    return CFG["b"] // world


def rank_spread(vals, dev=None):
    """(max, min) over the ranks of each value in `vals` (one MAX all-reduce
    of [x, -x]); the values themselves outside a process group."""
    import torch
    import torch.distributed as tdist
    if not tdist.is_initialized():
        return list(vals), list(vals)
    t = torch.tensor(list(vals) + [-x for x in vals], dtype=torch.float64, device=dev)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    n = len(vals)
    t = t.cpu().tolist()
    return t[:n], [-x for x in t[n:]]


def all_reduce_costs(flat, reps, on_gpu=True):
    """The gradient all-reduce alone: `reps` back-to-back all-reduces of the
    flat gradient buffer after a barrier, timed with a HIP event pair on the
    stream torch.distributed makes wait for the collective (RCCL runs it on
    its own stream; the current stream's events bracket its completion), or
    with the host clock for gloo on CPU tensors.  Bus bandwidth as RCCL's
    tests define it for a ring all-reduce: 2 (N-1)/N S / t.  Max over ranks."""
    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import _reducing
    if not _reducing(None):
        return None
    world = tdist.get_world_size()
    tdist.all_reduce(flat)                        # warm-up (communicator setup)
    tdist.barrier()
    if on_gpu:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            tdist.all_reduce(flat)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
    else:
        t0 = time.perf_counter()
        for _ in range(reps):
            tdist.all_reduce(flat)
        ms = (time.perf_counter() - t0) / reps * 1e3
    (ms_max,), (ms_min,) = rank_spread([ms], flat.device if on_gpu else None)
    S = flat.numel() * flat.element_size()
    return {"isolated_ms_per_call": ms_max, "isolated_ms_per_call_min_rank": ms_min, "reps": reps,
            "bytes": S, "bus_bandwidth_gbs": 2.0 * (world - 1) / world * S / (ms_max * 1e-3) / 1e9 if world > 1
            else None, "algo_bandwidth_gbs": S / (ms_max * 1e-3) / 1e9}


def launch_rehearsal(args):
    """--launch-only: the N-rank launch and its process group without the
    propagation step (no GPU work, runs on CPU with --dist-backend gloo): every
    rank joins the group and all-reduces its rank's batch of the weak leg and
    of the strong leg, then times the all-reduce of a CPU buffer the size of
    the flat gradient buffer (all_reduce_costs, host clock); rank 0 prints one
    JSON line with the world size, the global batches and the keys the bench
    line carries.  It is not a measurement of the path (no metric, no value)."""
    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import grad_shapes, init_from_env
    rank, world, _ = init_from_env(args.dist_backend)
    bs = strong_batch(world)
    b = torch.tensor([float(CFG["b"]), float(bs)])
    if tdist.is_initialized():
        tdist.all_reduce(b)
    n = sum(int(np.prod(s)) for s in grad_shapes(CFG["h"], 2 * CFG["e"]).values())
    ar = all_reduce_costs(torch.zeros(n), reps=5, on_gpu=False) if tdist.is_initialized() else None
    if rank == 0:
        print(json.dumps({"launch_rehearsal": True, "n_gpus": world, "world_size": world,
                          "config": {"global_batch": int(b[0].item()), "parallelism": "dp%d" % world},
                          "strong_scaling": {"per_rank_batch": bs, "global_batch": int(b[1].item())},
                          "all_reduce": dict(ar or {}, backend=tdist.get_backend() if tdist.is_initialized()
                                             else None),
                          "pid": os.getpid(), "launcher": os.environ.get("GGNN_BENCH_LAUNCHER", "external")}),
              flush=True)
    if tdist.is_initialized():
        tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dropout-keep", type=float, default=0.9,
                    help="keep probability of the dropout-on line (graph_state_dropout_keep_prob)")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side measurements (front-end/heads, bf16 mode)")
    ap.add_argument("--e2e-only", action="store_true",
                    help="of the side measurements, only the reference's run_epoch line (every rank; rehearsal)")
    ap.add_argument("--dist-backend", default=None, choices=(None, "nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (default nccl = RCCL; gloo only to rehearse "
                         "several ranks on one GPU).  Given explicitly at N = 1 (a one-rank torchrun), the "
                         "one-rank group is created and the per-step all-reduce runs anyway: the RCCL path "
                         "of an N-GPU run, executed on one GPU")
    ap.add_argument("--pmc-unfused-leg", action="store_true",
                    help="after the timed work, two steps with the unfused forward (k_prop_fwd + k_gru_fwd), so a "
                         "PMC pass over this command covers those kernels too (tools/profile_round.sh)")
    ap.add_argument("--precision", default="fp32", choices=("fp32", "fp16", "bf16"),
                    help="fp32: GGNN_FP32_PARITY (matches the reference fp32 math to <= 1e-3, the "
                         "parity mode); fp16 / bf16: single 16-bit MFMA operands (reduced precision)")
    ap.add_argument("--no-dropout-leg", action="store_true",
                    help="skip the dropout-on leg (a rocprofv3 run then sees only the dropout-off steps the "
                         "roofline is computed from)")
    ap.add_argument("--launch-only", action="store_true",
                    help="only start the N ranks, make the process group and all-reduce once (no GPU work; "
                         "the launcher's CPU test)")
    ap.add_argument("--spawn-timeout", type=float, default=None,
                    help="seconds after which the self-started ranks are stopped (N > 1 without torchrun)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # plain `python bench.py --gpus N`: start the N ranks here, before any
        # torch import or GPU call in this process
        os.environ["GGNN_BENCH_LAUNCHER"] = "bench.py"
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], args.spawn_timeout))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE %s: one rank per GPU, the two must agree" % (args.gpus, env_world),
              file=sys.stderr)
        sys.exit(2)
    if args.launch_only:
        return launch_rehearsal(args)

    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import FlatGradients, init_from_env
    from ggnn_amd.engine import PropagationEngine
    from ggnn_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ggnn_oracle as O  # synthetic input generator; not timed

    rank, world, local = init_from_env(args.dist_backend)
    local = local % max(torch.cuda.device_count(), 1)  # (ranks sharing a GPU: the gloo rehearsal only)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    b, v, h, T = CFG["b"], CFG["v"], CFG["h"], CFG["T"]
    C = 2 * CFG["e"]
    A, h0 = O.synthetic_batch(b, v, h, C, seed=1 + 1000 * rank)
    w = O.synthetic_weights(h, C, seed=1)
    A_d = torch.from_numpy(A).to(dev)
    h0_d = torch.from_numpy(h0).to(dev)
    w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    dhT = torch.from_numpy(np.random.default_rng(7 + rank).standard_normal((b, v, h)).astype(np.float32)).to(dev)
    eng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=args.precision)
    grads = FlatGradients(h, C, True, device=dev)
    from ggnn_amd.dist import GRAD_ORDER
    from ggnn_amd.optim import ClipAdam
    opt = ClipAdam([w_d[k] for k in GRAD_ORDER], learning_rate=0.003, clamp_gradient_norm=1.0)
    gviews = dict(grads.views)
    gviews["h0"] = torch.empty((b, v, h), dtype=torch.float32, device=dev)
    out = torch.empty((b, v, h), dtype=torch.float32, device=dev)

    nstep = [0]
    ar_events = []          # (start, end) event pairs around the in-step all-reduce (instrumented pass)

    def make_step(eng_, A_, h0_, dhT_, gviews_, grads_, out_):
        def step(keep=1.0, ev=None):
            # keep < 1: the reference's training feed (edge-weight + state dropout,
            # chem_tensorflow_dense.py:860-861), a fresh Philox seed every step
            nstep[0] += 1
            pack = eng_.pack_weights(w_d, T=T, edge_keep=keep, seed=nstep[0])
            eng_.set_adjacency(A_)
            eng_.forward(h0_, pack, T, training=True, out=out_, state_keep=keep)
            eng_.backward(dhT_, gviews_)
            if ev is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                grads_.all_reduce()
                e1.record()
                ev.append((e0, e1))
            else:
                grads_.all_reduce()
            opt.step([grads_.views[k] for k in GRAD_ORDER], grad_scale=1.0 / world)
        return step

    step = make_step(eng, A_d, h0_d, dhT, gviews, grads, out)

    def barrier():
        if tdist.is_initialized():
            tdist.barrier()
        torch.cuda.synchronize()

    def timed(fn, n, *a):
        barrier()
        t_ = time.perf_counter()
        for _ in range(n):
            fn(*a)
        barrier()
        return (time.perf_counter() - t_) / n

    for _ in range(args.warmup):
        step()
    barrier()
    # timed region: exactly K steps, nothing else on the stream
    dt = timed(step, args.steps)
    # the same K steps again with a HIP event pair around every library launch
    # (kernel durations for the roofline; the events add gaps between launches,
    # so this pass is not the headline time) and around the all-reduce
    timer = _lib.KernelTimer(max_launches=200 * max(args.steps, 1))
    with timer:
        dt_instr = timed(step, args.steps, 1.0, ar_events)
    # the same step with the training-feed dropout (keep 0.9 for both), reported beside
    # Timed in alternating blocks of K/2 steps (off, on, off, on) so that the
    # two are compared on the same clock state: a leg timed minutes after the
    # headline region sees another DVFS state of the chip
    dt_drop = dt_drop_off = float("nan")
    if not args.no_dropout_leg:
        for _ in range(args.warmup):
            step(args.dropout_keep)
        half = max(args.steps // 2, 1)
        on, off = [], []
        for _ in range(2):
            off.append(timed(step, half))
            on.append(timed(step, half, args.dropout_keep))
        dt_drop, dt_drop_off = float(np.mean(on)), float(np.mean(off))
    # strong scaling: the global batch of 256 graphs split
    # 256/N per rank, timed exactly like the weak leg.  At N = 1 it IS the weak leg.
    bs = strong_batch(world)
    dt_strong = dt
    if world > 1:
        # rank r takes graphs [r*bs, (r+1)*bs) of ONE global batch (rank 0's seed)
        As, h0s = (A, h0) if rank == 0 else O.synthetic_batch(b, v, h, C, seed=1)
        sl = slice(rank * bs, (rank + 1) * bs)
        As_d = torch.from_numpy(np.ascontiguousarray(As[sl])).to(dev)
        h0s_d = torch.from_numpy(np.ascontiguousarray(h0s[sl])).to(dev)
        eng_s = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=args.precision)
        grads_s = FlatGradients(h, C, True, device=dev)
        gv_s = dict(grads_s.views)
        gv_s["h0"] = torch.empty((bs, v, h), dtype=torch.float32, device=dev)
        out_s = torch.empty((bs, v, h), dtype=torch.float32, device=dev)
        step_s = make_step(eng_s, As_d, h0s_d, dhT[sl].contiguous(), gv_s, grads_s, out_s)
        for _ in range(args.warmup):
            step_s()
        dt_strong = timed(step_s, args.steps)
        del eng_s, grads_s, gv_s, out_s, As_d, h0s_d
        torch.cuda.empty_cache()
    ar_in_step = None
    from ggnn_amd.dist import _reducing
    if ar_events and _reducing(None):
        torch.cuda.synchronize()
        ar_in_step = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ar_events]))
    ar_iso = all_reduce_costs(grads.flat, reps=max(args.steps, 10))
    (dt, dt_drop, dt_strong, dt_instr, ar_max, dt_drop_off), (dt_min, dt_drop_min, dt_strong_min, _, ar_min, _) = \
        rank_spread([dt, dt_drop, dt_strong, dt_instr, ar_in_step if ar_in_step is not None else float("nan"),
                     dt_drop_off], dev)

    if args.pmc_unfused_leg:
        ueng = PropagationEngine(h, C, use_edge_bias=True, device=dev, precision=args.precision,
                                 unfused_forward=True)
        for _ in range(2):
            pack = ueng.pack_weights(w_d, T=T)
            ueng.set_adjacency(A_d)
            ueng.forward(h0_d, pack, T, training=True, out=out)
            ueng.backward(dhT, gviews)
        barrier()

    # roofline of the dominant kernel (largest total time in the timed region)
    kinds = {k: ms for k, ms in timer.total_ms.items() if timer.launches.get(k)}
    dom = max(kinds, key=kinds.get)
    n_l = timer.launches[dom]
    avg_ms = timer.total_ms[dom] / n_l
    fl = kernel_algo_flops(dom, b, v, h, C, T)
    achieved = fl / (avg_ms * 1e-3) / 1e12 if fl else None
    traffic = None
    tr = load_traffic(args.precision)
    traffic_src = None
    if tr and tr.get("precision", "fp32") == args.precision and dom in tr.get("kernels", {}):
        traffic = tr["kernels"][dom]["hbm_bytes_per_launch"]
        traffic_src = ("profiles/pmc_traffic.json (%s): rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE per launch, "
                       "collected in separate passes of this bench's command (PMC passes cannot run inside "
                       "the timed process)" % tr.get("run", "?"))
    roof = {"bound": "mfma", "kernel": dom, "achieved": achieved, "peak": BF16_DENSE_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": (achieved / BF16_DENSE_PEAK_TFLOPS) if achieved else None,
            "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": avg_ms,
            "algo_flops_per_launch": fl}
    ceil = load_ceilings()
    if ceil:
        # library ceilings measured on an MI355X box (tools/ceilings.py): the
        # f16 GEMM for the f16 / fp32-parity limbs, the bf16 GEMM for bf16
        key = "gemm_bf16_tflops" if args.precision == "bf16" else "gemm_f16_tflops"
        roof["measured_peak"] = ceil[key]
        roof["measured_peak_source"] = "profiles/ceilings.json (%s, hipBLASLt 8192^3)" % key
        if achieved:
            roof["frac_of_measured"] = achieved / ceil[key]
    ifl = kernel_issued_flops(dom, b, v, h, C, T, args.precision)
    if ifl and avg_ms:
        # the MFMA pipes' real load: issued products (limb split included) / peak
        roof["issued_flops_per_launch"] = ifl
        roof["frac_issued"] = ifl / (avg_ms * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS
        if ceil:
            roof["frac_issued_of_measured"] = ifl / (avg_ms * 1e-3) / 1e12 / roof["measured_peak"]
    # the same figures for every MFMA kernel of the step (k_gru_bwd beside the dominant one)
    roof["kernels"] = {}
    for k in ("fwd_fused", "gru_bwd", "prop_bwd", "wgrad"):
        if not timer.launches.get(k):
            continue
        am = timer.total_ms[k] / timer.launches[k]
        afl, ifl_k = kernel_algo_flops(k, b, v, h, C, T), kernel_issued_flops(k, b, v, h, C, T, args.precision)
        kd = {"avg_launch_ms": am, "launches_per_step": timer.launches[k] / args.steps,
              "algo_flops_per_launch": afl, "frac": afl / (am * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS,
              "issued_flops_per_launch": ifl_k, "frac_issued": ifl_k / (am * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS}
        if ceil:
            kd["frac_issued_of_measured"] = ifl_k / (am * 1e-3) / 1e12 / ceil["gemm_bf16_tflops" if
                                                                             args.precision == "bf16" else
                                                                             "gemm_f16_tflops"]
        if tr and k in tr.get("kernels", {}):
            kd["traffic"] = tr["kernels"][k]["hbm_bytes_per_launch"]
            kd["hbm_frac"] = kd["traffic"] / (am * 1e-3) / 1e9 / HBM_PEAK_GBS
        roof["kernels"][k] = kd
    breakdown = {k: {"ms_per_step": timer.total_ms[k] / args.steps, "launches_per_step": timer.launches[k] / args.steps}
                 for k in kinds}

    # the reference's own end-to-end run_epoch on its sentences: every rank
    # (data-parallel when world > 1), before the rank-0-only side lines
    e2e = end_to_end_side(dev, rank, world, restrict=(world == 1)) if not args.no_side else None
    if args.e2e_only:
        args.no_side = True
    feed_cmp = adjacency_feed_costs(eng, b, v, CFG["e"], dev) if rank == 0 else None
    callers = callers_side(dev, b, v, h) if rank == 0 and not args.no_side else None
    host_slice = (A[:2], h0[:2], w)
    bf16 = (precision_side(dev, "bf16", A_d, h0_d, w_d, dhT, b, v, h, C, T, host=host_slice)
            if rank == 0 and not args.no_side and args.precision != "bf16" else None)
    fp16 = (precision_side(dev, "fp16", A_d, h0_d, w_d, dhT, b, v, h, C, T, host=host_slice)
            if rank == 0 and not args.no_side and args.precision != "fp16" else None)
    real = real_density_side(dev) if rank == 0 and not args.no_side else None
    strong1 = (strong_split_side(dev, A, h0, dhT.cpu().numpy(), w_d, v, h, C, T, args.precision)
               if rank == 0 and world == 1 and not args.no_side else None)

    if rank == 0:
        fpg = flops_per_graph(v, h, C, T)["total"]
        value = world * b / dt
        res = {
            "metric": "instances/sec (graphs/s) GGNN fwd+bwd, hidden=256 v=128 e=4 T=5",
            "value": value,
            "unit": "graphs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"fp32": "fp32", "fp16": "fp16", "bf16": "bf16"}[args.precision],
            "precision_note": {"fp32": "fp32-class: every non-exact MFMA operand of the forward and of the "
                                       "dh/dX chain as an f16 hi/lo limb pair (3 products), fp32 accumulation, "
                                       "except k_gru_bwd's Wc^T / Wg^T (the hi limb only: dz hi/lo x W hi, 2 "
                                       "products) and k_prop_bwd's dM W_c^T (hi x hi on f16 MFMAs, both limb "
                                       "corrections on the block-scaled fp8 MFMA: e5m2 dM, e4m3 W_c^T); the "
                                       "weight-gradient GEMMs (k_wgrad256) take SINGLE f16 "
                                       "operands, on a power-of-two-scaled gradient; parity <= 1e-3 vs the fp32 "
                                       "reference (tests/test_gpu_parity.py, incl. loss-scale gradients; the "
                                       "backward's limb policy: tests/test_precision_policies.py)",
                               "fp16": "f16 MFMA operands, fp32 accumulation (reduced precision)",
                               "bf16": "bf16 MFMA operands, fp32 accumulation (reduced precision)"}[args.precision],
            "data": "synthetic (SURVEY §8d generator: Bernoulli(0.1) adjacency on n~U{v/2..v} active nodes, glorot weights)",
            "config": {"workload": "configs[2]: b=256 graphs/GPU, v=128, hidden=256, e=4 (C=8), T=5, fwd+bwd",
                       "global_batch": world * b, "parallelism": "dp%d" % world},
            "roofline": roof,
            "achieved_step_tflops": world * b * fpg / dt / 1e12,
            "kernel_breakdown": breakdown,
            "rank_step_ms": {"max": dt * 1e3, "min": dt_min * 1e3,
                             "note": "each rank's K-step average; value uses the max (the slowest rank)"},
            "strong_scaling": {"value": b / dt_strong, "unit": "graphs/s", "ms_per_step": dt_strong * 1e3,
                               "ms_per_step_min_rank": dt_strong_min * 1e3, "per_rank_batch": bs,
                               "global_batch": b, "scaling": "strong",
                               "note": "global batch of 256 graphs split 256/N per rank (SURVEY §8d, config 4), "
                                       "same step and timing as the weak value; at N = 1 the weak leg itself"},
            "all_reduce": dict(ar_iso or {}, **{
                           "backend": tdist.get_backend() if tdist.is_initialized() else None,
                           "bytes_per_step": grads.nbytes,
                           "in_step_ms": None if np.isnan(ar_max) else ar_max,
                           "in_step_ms_min_rank": None if np.isnan(ar_min) else ar_min,
                           "in_step_bus_bandwidth_gbs": (2.0 * (world - 1) / world * grads.nbytes / (ar_max * 1e-3)
                                                         / 1e9) if world > 1 and not np.isnan(ar_max) else None,
                           "note": "one all-reduce of the flat fp32 gradient buffer per step (RCCL = backend "
                                   "nccl); none without a process group.  in_step_ms: HIP events on the step's "
                                   "stream around the collective in the instrumented pass (includes waiting for "
                                   "the slowest rank); isolated_ms_per_call: back-to-back all-reduces after a "
                                   "barrier; bus bandwidth 2(N-1)/N S / t"}),
            "launcher": os.environ.get("GGNN_BENCH_LAUNCHER", "external (torch.distributed.run)"
                                       if "WORLD_SIZE" in os.environ else "single process"),
            "ms_per_step_event_instrumented": dt_instr * 1e3,
            "adjacency_feed": feed_cmp,
            "dropout_on": None if args.no_dropout_leg else {
                           "edge_keep": args.dropout_keep, "state_keep": args.dropout_keep,
                           "value": world * b / dt_drop, "ms_per_step": dt_drop * 1e3,
                           "dropout_off_adjacent_ms_per_step": dt_drop_off * 1e3,
                           "ratio_to_adjacent_off": dt_drop / dt_drop_off,
                           "note": "same step with the reference's training-feed dropout (:860-861), timed in "
                                   "alternating K/2-step blocks with the dropout-off step (off, on, off, on): "
                                   "ms_per_step = the on blocks, dropout_off_adjacent_ms_per_step = the off "
                                   "blocks; value above is dropout off (keep 1, the parity setting)"},
            "callers": callers,
            "bf16_mode": bf16,
            "fp16_mode": fp16,
            "real_density_c92": real,
            "strong_split_one_gpu": strong1,
            "end_to_end_run_epoch": e2e,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_reps)
        print(json.dumps(res), flush=True)
    if tdist.is_initialized():
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
