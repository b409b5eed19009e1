"""Pair mode vs the dense-tile general path vs the fast path on the
reference's configuration (dependency trees, E = 46 -> C = 92, v = 30,
hidden 400 / 256, T = 4): fwd+bwd ms per b = 256 step, kernel-kind breakdown.

    python tools/pairs_probe.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import ggnn_oracle as O
    from ggnn_amd import _lib
    from ggnn_amd.dist import FlatGradients
    from ggnn_amd.engine import PropagationEngine
    dev = torch.device("cuda", 0)
    b, v, E = 256, 30, 46
    C = 2 * E
    rng = np.random.default_rng(13)
    pz = 1.0 / np.arange(1, E + 1)
    pz /= pz.sum()
    graphs = []
    for _ in range(b):
        n = int(rng.integers(v // 2, v + 1))
        graphs.append([(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)])
    out = {}
    for h, T in ((400, 4), (256, 5)):
        w = O.synthetic_weights(h, C, seed=3)
        w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
        h0 = torch.from_numpy(rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)).to(dev)
        dhT = torch.from_numpy(rng.standard_normal((b, v, h)).astype(np.float32)).to(dev)
        for name, kw in (("pairs", dict(sparse_pairs=True)), ("dense_tiles", dict(sparse_pairs=False, force_generic=True)),
                         ("fast", dict(sparse_pairs=False))):
            if name == "fast" and h not in (128, 256):
                continue
            for keep in (1.0, 0.9):
                eng = PropagationEngine(h, C, device=dev, precision="fp32", **kw)
                grads = FlatGradients(h, C, True, device=dev)
                gv = dict(grads.views)
                gv["h0"] = torch.empty((b, v, h), dtype=torch.float32, device=dev)
                o = torch.empty((b, v, h), dtype=torch.float32, device=dev)
                eng.set_adjacency_edges(graphs, v, E)
                step = [0]

                def run():
                    step[0] += 1
                    pack = eng.pack_weights(w_d, T=T, edge_keep=keep, seed=step[0])
                    eng.forward(h0, pack, T, training=True, out=o, state_keep=keep)
                    eng.backward(dhT, gv)
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 5
                timer = _lib.KernelTimer(max_launches=5000)
                with timer:
                    run()
                    torch.cuda.synchronize()
                key = "h%d_T%d_%s_keep%g" % (h, T, name, keep)
                out[key] = {"ms_per_step": ms, "sparse": eng.sparse,
                            "kernels_ms": {k: round(x, 4) for k, x in timer.total_ms.items() if x}}
                print(key, json.dumps(out[key]), flush=True)
                del eng, grads, gv, o
                torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pairs_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
