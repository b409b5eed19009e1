"""Time the general path (k_gemm + k_generic.h) on a few shapes: config 3 forced
through it, hidden 400 (the reference default) dense and on C = 92 dependency trees.
Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggnn_oracle as O  # noqa: E402
from bench import _timed_events, flops_per_graph  # noqa: E402
from ggnn_amd.dist import FlatGradients  # noqa: E402
from ggnn_amd.engine import PropagationEngine  # noqa: E402


def run(b, v, h, C, T, generic, trees=False, steps=5):
    dev = torch.device("cuda", 0)
    if trees:
        rng = np.random.default_rng(1)
        E = C // 2
        pz = 1.0 / np.arange(1, E + 1)
        pz /= pz.sum()
        graphs = [[(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, int(rng.integers(v // 2, v + 1)))]
                  for _ in range(b)]
        h0 = rng.uniform(-0.2, 0.2, (b, v, h)).astype(np.float32)
    else:
        A, h0 = O.synthetic_batch(b, v, h, C, seed=1)
    w = O.synthetic_weights(h, C, seed=1)
    eng = PropagationEngine(h, C, device=dev, precision="fp32", force_generic=generic)
    if trees:
        eng.set_adjacency_edges(graphs, v, C // 2)
    else:
        eng.set_adjacency(torch.from_numpy(A).to(dev))
    w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    h0_d = torch.from_numpy(h0).to(dev)
    dhT = torch.from_numpy(np.random.default_rng(2).standard_normal((b, v, h)).astype(np.float32)).to(dev)
    grads = FlatGradients(h, C, True, device=dev)
    gv = dict(grads.views)
    gv["h0"] = torch.empty((b, v, h), dtype=torch.float32, device=dev)

    def step():
        pack = eng.pack_weights(w_d, T=T)
        eng.forward(h0_d, pack, T, training=True)
        eng.backward(dhT, gv)

    ms = _timed_events(step, steps)
    f = flops_per_graph(v, h, C, T)["total"] * b
    return {"shape": [b, v, h, C, T], "generic": generic, "trees": trees, "ms": ms, "graphs_per_s": b / ms * 1e3,
            "algo_tflops": f / ms / 1e9}


if __name__ == "__main__":
    out = [run(256, 128, 256, 8, 5, False), run(256, 128, 256, 8, 5, True), run(256, 128, 400, 8, 5, False),
           run(256, 30, 400, 92, 4, False, trees=True), run(64, 198, 400, 92, 4, False, trees=True)]
    for r in out:
        print(json.dumps(r))
