"""A/B timing of the config-3 training step (bench.py's step without the side
lines): engine variants alternate in one process, so box-to-box clock
differences cancel.  Prints one JSON line per variant and round with the clean
step time and the HIP-event kernel breakdown.

    python tools/ab_step.py --variants skip,dense --rounds 3
    GGNN_LIB=other.so python tools/ab_step.py ...   (a library build A/B: two runs)

Variants: skip (channel skipping, the default engine), dense
(skip_empty_channels=False), keepXX (training dropout at keep 0.XX), ekXX /
stXX (edge-weight / state dropout alone at keep 0.XX).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="skip,dense")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--trees", action="store_true", help="b=256 dependency trees, v=30, C=92 (real density)")
    ap.add_argument("--reference", action="store_true",
                    help="with --trees: the reference's model (hidden 400, T = 4), edge lists staged once, pair mode")
    ap.add_argument("--batch", type=int, default=256, help="graphs per batch (20: run_epoch's batch_size)")
    args = ap.parse_args()
    import torch
    from ggnn_amd import _lib
    from ggnn_amd.dist import GRAD_ORDER, FlatGradients
    from ggnn_amd.engine import PropagationEngine
    from ggnn_amd.optim import ClipAdam
    import ggnn_oracle as O

    dev = torch.device("cuda", 0)
    b, v, h, C, T = args.batch, 128, 256, 8, 5
    if args.reference:
        args.trees, h, T = True, 400, 4
    graphs = None
    if args.trees:
        v, C = 30, 92
        rng = np.random.default_rng(13)
        E = C // 2
        pz = 1.0 / np.arange(1, E + 1)
        pz /= pz.sum()
        A = np.zeros((b, C, v, v), np.float32)
        graphs = []
        for g in range(b):
            n = int(rng.integers(v // 2, v + 1))
            ed = [(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)]
            graphs.append(ed)
            A[g] = O.graph_to_adj_mat_bd(ed, v, E, dtype=np.float32)
        h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    else:
        A, h0 = O.synthetic_batch(b, v, h, C, seed=1)
    w = O.synthetic_weights(h, C, seed=1)
    A_d, h0_d = torch.from_numpy(A).to(dev), torch.from_numpy(h0).to(dev)
    w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    dhT = torch.from_numpy(np.random.default_rng(7).standard_normal((b, v, h)).astype(np.float32)).to(dev)
    opt = ClipAdam([w_d[k] for k in GRAD_ORDER], learning_rate=0.003)

    def make(variant):
        keep = 1.0
        ekeep = skeep = None     # edge / state keep when they differ (variants ekXX, stXX)
        kw = {}
        if variant == "dense":
            kw["skip_empty_channels"] = False
        elif variant.startswith("keep"):
            keep = float("0." + variant[4:])
        elif variant.startswith("ek"):
            ekeep, skeep = float("0." + variant[2:]), 1.0
        elif variant.startswith("st"):
            ekeep, skeep = 1.0, float("0." + variant[2:])
        eng = PropagationEngine(h, C, device=dev, **kw)
        if args.reference:
            eng.set_adjacency_edges(graphs, v, C // 2)      # once, as bench.py's real-density lines
        grads = FlatGradients(h, C, True, device=dev)
        gv = dict(grads.views)
        gv["h0"] = torch.empty((b, v, h), device=dev)
        out = torch.empty((b, v, h), device=dev)
        n = [0]

        def step():
            n[0] += 1
            ek = keep if ekeep is None else ekeep
            sk = keep if skeep is None else skeep
            pack = eng.pack_weights(w_d, T=T, edge_keep=ek, seed=n[0])
            if not args.reference:
                eng.set_adjacency(A_d)
            eng.forward(h0_d, pack, T, training=True, out=out, state_keep=sk)
            eng.backward(dhT, gv)
            opt.step([grads.views[k] for k in GRAD_ORDER])
        return step

    steps = {vn: make(vn) for vn in args.variants.split(",")}
    for r in range(args.rounds):
        for vn, step in steps.items():
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            timer = _lib.KernelTimer(max_launches=200 * args.steps)
            with timer:
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
            br = {k: round(timer.total_ms[k] / args.steps, 4) for k in timer.total_ms if timer.launches.get(k)}
            print(json.dumps({"variant": vn, "round": r, "ms_per_step": round(dt * 1e3, 4), "kernels": br,
                              "lib": os.environ.get("GGNN_LIB", "ggnn_amd/libggnn.so"), "trees": args.trees}),
                  flush=True)


if __name__ == "__main__":
    main()
