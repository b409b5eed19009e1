"""Phase timeline of the hot kernels (experiment build with -DGGNN_TS).

GGNN_LIB=ggnn_amd/exp/lib_ts.so python tools/ts_probe.py
Prints, per kernel, the median per-workgroup duration of every phase and the
spread of workgroup start/end times (s_memrealtime, 100 MHz).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.engine import PropagationEngine  # noqa: E402
import ggnn_oracle as O  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
b, v, h, C, T = 256, 128, 256, 8, 5
A, h0 = O.synthetic_batch(b, v, h, C, seed=1, density=0.1)
w = O.synthetic_weights(h, C, seed=1)
eng = PropagationEngine(h, C, precision=prec)
dev = eng.device
pack = eng.pack_weights({k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()})
eng.set_adjacency(torch.from_numpy(A).to(dev))
h0d = torch.from_numpy(h0).to(dev)
dhT = torch.randn(b, v, h, device=dev)
for _ in range(3):
    eng.forward(h0d, pack, T, training=True)
    eng.backward(dhT)
torch.cuda.synchronize()
lib = _lib.load()
buf = np.zeros((4, 2048, 8), np.uint64)
assert lib.ggnn_dbg_ts(buf.ctypes.data_as(ctypes.c_void_p)) == 0
names = {0: ("gru_fwd", 512, ["stage", "passA", "rh", "passB", "blend+st"]),
         1: ("gru_bwd", 512, ["ph1", "prod1", "ph2", "prod2+st"]),
         2: ("fwd_fused (last t)", 256, ["msg", "X out", "passA", "rh", "passB", "blend"]),
         3: ("prop_bwd", 256, ["stage", "chan loop", "dh out"])}
for k, (nm, nwg, phases) in names.items():
    nwg = int((buf[k, :, 0] != 0).sum())
    if nwg == 0:
        continue
    t = buf[k, :nwg, :len(phases) + 1].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) * 0.01  # us
    d = np.diff(t, axis=1)
    print("%-8s kernel span %.1f us | WG dur median %.1f us | start: min %.1f med %.1f max %.1f | end: min %.1f max %.1f"
          % (nm, t[:, -1].max(), np.median(t[:, -1] - t[:, 0]), t[:, 0].min(), np.median(t[:, 0]), t[:, 0].max(),
             t[:, -1].min(), t[:, -1].max()))
    print("          phases (median / p90 us): " + "  ".join(
        "%s %.1f/%.1f" % (p, np.median(d[:, i]), np.percentile(d[:, i], 90)) for i, p in enumerate(phases)))
    if k < 2:
        st = np.sort(t[:, 0])
        print("          start-time quartiles: %s" % np.round(np.percentile(st, [10, 25, 50, 75, 90]), 1))

