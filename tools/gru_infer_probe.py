"""The unfused forward in inference mode only (training=False: k_prop_fwd +
k_gru_fwd per timestep, no saves), configs[2] shape, so that a rocprofv3
--pmc pass over this script sees inference launches of k_gru_fwd and nothing
else of that name (bench.py's gru_inference_leg reads the bytes per launch
from profiles/pmc_traffic_<precision>_infer.json).

    python tools/gru_infer_probe.py [precision] [forwards]
    bash tools/pmc_profile_infer.sh OUTDIR [precision]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.engine import PropagationEngine  # noqa: E402
import ggnn_oracle as O  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
b, v, h, C, T = 256, 128, 256, 8, 5
A, h0 = O.synthetic_batch(b, v, h, C, seed=1)
w = O.synthetic_weights(h, C, seed=1)
eng = PropagationEngine(h, C, device=dev, precision=prec, unfused_forward=True)
pack = eng.pack_weights({k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}, T=T)
eng.set_adjacency(torch.from_numpy(A).to(dev))
h0_d = torch.from_numpy(h0).to(dev)
out = torch.empty((b, v, h), device=dev)
timer = _lib.KernelTimer()
with timer:
    for _ in range(n):
        eng.forward(h0_d, pack, T, training=False, out=out)
    torch.cuda.synchronize()
print(json.dumps({k: {"launches": timer.launches[k], "avg_ms": timer.total_ms[k] / timer.launches[k]}
                  for k in timer.launches if timer.launches[k]}))
