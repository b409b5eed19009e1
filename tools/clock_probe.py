"""In-kernel clock of the config-3 step's MFMA kernels (MI355X_MICROARCH.md
"DVFS give-back" item 6): a diagnostic build (-DGGNN_TS) stamps s_memtime and
s_memrealtime at every workgroup's start and end (TSCLK, ggnn_common.h); after
>= 2 s of back-to-back steps on random data the clock of each workgroup is
d(memtime) / d(memrealtime) x 100 MHz, reported as the median over workgroups.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -DGGNN_TS \\
        -o tools/lib_ts.so ggnn_amd/csrc/ggnn_api.hip
    GGNN_LIB=tools/lib_ts.so python tools/clock_probe.py [seconds]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.dist import FlatGradients  # noqa: E402
from ggnn_amd.engine import PropagationEngine  # noqa: E402
import ggnn_oracle as O  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
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


def step():
    pack = eng.pack_weights(w_d, T=T)
    eng.set_adjacency(A_d)
    eng.forward(h0_d, pack, T, training=True, out=out)
    eng.backward(dhT, gv)


t0 = time.time()
n = 0
while time.time() - t0 < secs:
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    n += 20
lib = _lib.load()
lib.ggnn_dbg_clk.argtypes = [ctypes.c_void_p]
buf = np.zeros((4, 2048, 4), np.uint64)
assert lib.ggnn_dbg_clk(buf.ctypes.data_as(ctypes.c_void_p)) == 0
res = {"steps": n, "seconds": secs}
for k, nm in ((0, "k_wgrad256"), (1, "k_gru_bwd"), (2, "k_fwd_fused"), (3, "k_prop_bwd")):
    x = buf[k].astype(np.int64)
    ok = (x[:, 0] != 0) & (x[:, 2] > x[:, 0])
    if not ok.any():
        continue
    drt = (x[ok, 2] - x[ok, 0]).astype(np.float64)
    dmt = (x[ok, 3] - x[ok, 1]).astype(np.float64)
    ghz = dmt / drt * 0.1
    res[nm] = {"workgroups": int(ok.sum()), "clock_ghz_median": float(np.median(ghz)),
               "clock_ghz_p10": float(np.percentile(ghz, 10)), "clock_ghz_p90": float(np.percentile(ghz, 90)),
               "wg_us_median": float(np.median(drt) * 0.01)}
print(json.dumps(res))
