"""Per-kernel time of the config-3 step with and without the training feed's
dropout (edge-weight + state keep 0.9, chem_tensorflow_dense.py:860-861)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ggnn_oracle as O  # noqa: E402
from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.dist import FlatGradients  # noqa: E402
from ggnn_amd.engine import PropagationEngine  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    b, v, h, C, T = 256, 128, 256, 8, 5
    A, h0 = O.synthetic_batch(b, v, h, C, seed=1)
    w = O.synthetic_weights(h, C, seed=1)
    A_d, h0_d = torch.from_numpy(A).to(dev), torch.from_numpy(h0).to(dev)
    w_d = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    dhT = torch.randn(b, v, h, device=dev)
    eng = PropagationEngine(h, C, device=dev)
    g = FlatGradients(h, C, True, device=dev)
    gv = dict(g.views)
    gv["h0"] = torch.empty((b, v, h), device=dev)
    out = torch.empty((b, v, h), device=dev)
    res = {}
    for keep in (1.0, 0.9):
        def step(i):
            pack = eng.pack_weights(w_d, T=T, edge_keep=keep, seed=i + 1)
            eng.set_adjacency(A_d)
            eng.forward(h0_d, pack, T, training=True, out=out, state_keep=keep)
            eng.backward(dhT, gv)
        for i in range(3):
            step(i)
        torch.cuda.synchronize()
        tm = _lib.KernelTimer()
        with tm:
            for i in range(20):
                step(i)
            torch.cuda.synchronize()
        res[keep] = {k: round(tm.total_ms[k] / 20, 4) for k in tm.total_ms if tm.launches.get(k)}
    print(json.dumps(res))
