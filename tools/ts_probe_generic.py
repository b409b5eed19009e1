"""Per-workgroup phase stamps of the general path's products at the reference's
batch (experiment build with -DGGNN_TS; GemmArgs::tsprobe picks the launches).

    hipcc ... -DGGNN_TS -o tools/lib_ts.so ggnn_amd/csrc/ggnn_api.hip
    GGNN_LIB=tools/lib_ts.so python tools/ts_probe_generic.py

Slots: 0 = the pair dW over all timesteps (term groups), 1 = the GRU weight
gradient dWc[:H] (the first of the four), 2 = the pair message product Y W_c
(last forward timestep), 3 = its backward dXg W_c^T (timestep 0).  Marks per
workgroup: 0 start, 1 after the prologue, 2 after the K loop, 3 after the
epilogue; 5 = its slice count, 6 = its z.  s_memrealtime runs at 100 MHz.
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.batching import TRAIN_WITH_DEV, wsj_model_sizes  # noqa: E402
from ggnn_amd.model import DenseGGNNChemModel  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    m = DenseGGNNChemModel(params={"compact_adjacency": True, "hip_graphs": False}, seed=0, device=dev,
                           **wsj_model_sizes())
    train = m.load_data(TRAIN_WITH_DEV["train_file"], True)
    it = m.make_minibatch_iterator(train, True)
    feeds = []
    for f in it:
        if int(f["num_graphs"]) == m.params["batch_size"]:
            feeds.append(f)
        if len(feeds) == 8:
            break
    lib = _lib.load()
    for f in feeds[:7]:
        f["out_layer_dropout_keep_prob"] = m.params["out_layer_dropout_keep_prob"]
        m.train_step(f)
    torch.cuda.synchronize()
    assert lib.ggnn_dbg_ts_clear() == 0
    f = feeds[7]
    f["out_layer_dropout_keep_prob"] = m.params["out_layer_dropout_keep_prob"]
    m.train_step(f)
    torch.cuda.synchronize()
    buf = np.zeros((4, 2048, 8), np.uint64)
    assert lib.ggnn_dbg_ts(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    print("batch: %d graphs, v = %d" % (int(f["num_graphs"]), int(f["num_vertices"])))
    names = ["pair dW (term groups)", "GRU dWc[:H]", "pair fwd Y W_c (t = T-1)", "pair bwd dXg W_c^T (t = 0)"]
    for k, nm in enumerate(names):
        st = buf[k, :, 0].astype(np.int64)
        wg = np.nonzero(st)[0]
        if wg.size == 0:
            print("%s: no stamps" % nm)
            continue
        t = buf[k, wg, :4].astype(np.int64)
        t0 = st[wg].min()
        live = t[:, 1] != 0
        rel = np.where(t > 0, (t - t0) * 0.01, np.nan)  # us
        span = np.nanmax(rel)
        print("%s: %d workgroups stamped, %d live (past the z / zmask checks), kernel span %.1f us"
              % (nm, wg.size, int(live.sum()), span))
        if not live.any():
            continue
        r = rel[live]
        nit = buf[k, wg[live], 5].astype(np.int64)
        pro, loop = r[:, 1] - r[:, 0], r[:, 2] - r[:, 1]
        epi = r[:, 3] - r[:, 2]
        print("   start: min %.1f med %.1f max %.1f us | live end (mark 3): med %.1f max %.1f"
              % (np.nanmin(r[:, 0]), np.nanmedian(r[:, 0]), np.nanmax(r[:, 0]), np.nanmedian(r[:, 3]),
                 np.nanmax(r[:, 3])))
        print("   prologue med %.2f us | K loop med %.2f max %.2f us | epilogue med %.2f max %.2f us"
              % (np.nanmedian(pro), np.nanmedian(loop), np.nanmax(loop), np.nanmedian(epi), np.nanmax(epi)))
        for n in sorted(set(nit.tolist()))[:12]:
            sel = nit == n
            print("     slices %3d: %4d WGs, loop med %.2f us (%.3f us/slice), epilogue med %.2f us"
                  % (n, int(sel.sum()), np.nanmedian(loop[sel]), np.nanmedian(loop[sel]) / max(n, 1),
                     np.nanmedian(epi[sel])))
        dead = ~live
        if dead.any():
            print("   idle workgroups: start med %.1f max %.1f us" % (np.nanmedian(rel[dead, 0]), np.nanmax(rel[dead, 0])))


if __name__ == "__main__":
    main()
