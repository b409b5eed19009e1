"""Where run_epoch's time goes at the reference's default params on its own
sentences (--train_with_dev): wall time per batch vs the library's kernel
time per batch (HIP events around every launch), and a cProfile of the host.

    python tools/e2e_profile.py [--no-cprofile]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ggnn_amd import _lib  # noqa: E402
from ggnn_amd.batching import TRAIN_WITH_DEV, wsj_model_sizes  # noqa: E402
from ggnn_amd.model import DenseGGNNChemModel  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    # the kernel timer sees eager launches only (no records inside a hipGraph
    # capture, none around a replay): time the kernels on the eager path and
    # the wall clock on the captured one
    m = DenseGGNNChemModel(params={"compact_adjacency": True, "hip_graphs": False}, seed=0, device=dev,
                           **wsj_model_sizes())
    train = m.load_data(TRAIN_WITH_DEV["train_file"], True)
    valid = m.load_data(TRAIN_WITH_DEV["valid_file"], False)
    m.run_epoch("warm-up", train, True)
    for name, data, tr in (("train", train, True), ("valid", valid, False)):
        timer = _lib.KernelTimer(max_launches=400000)
        t0 = time.perf_counter()
        with timer:
            r = m.run_epoch(name, data, tr)
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ks = {k: v for k, v in timer.total_ms.items() if v}
        print("%s: %d batches, %.1f inst/s (timed run: wall %.1f ms/batch, kernels %.2f ms/batch, launches %.0f/batch)"
              % (name, r[4], r[3], wall * 1e3 / r[4], sum(ks.values()) / r[4],
                 sum(timer.launches.values()) / r[4]))
        print("   per kind ms/batch:", {k: round(v / r[4], 3) for k, v in ks.items()})
    np.random.seed(0)
    m = DenseGGNNChemModel(params={"compact_adjacency": True}, seed=0, device=dev, **wsj_model_sizes())
    train = m.load_data(TRAIN_WITH_DEV["train_file"], True)
    valid = m.load_data(TRAIN_WITH_DEV["valid_file"], False)
    for _ in range(2):
        m.run_epoch("warm-up", train, True)
        m.run_epoch("warm-up", valid, False)
    for name, data, tr in (("train", train, True), ("valid", valid, False)):
        t0 = time.perf_counter()
        r = m.run_epoch(name, data, tr)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print("%s (hipGraph steps): %.1f inst/s, wall %.2f ms/batch, %s" % (name, r[3], wall * 1e3 / r[4],
                                                                          m.graph_stats))
    if "--no-cprofile" not in sys.argv:
        for name, data, tr_ in (("train", train, True), ("valid", valid, False)):
            pr = cProfile.Profile()
            pr.enable()
            r = m.run_epoch(name, data, tr_)
            pr.disable()
            print("%s inst/s (cProfile on) %.1f" % (name, r[3]))
            st = pstats.Stats(pr)
            st.sort_stats("tottime").print_stats(30)
