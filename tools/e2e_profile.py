"""cProfile of one run_epoch at the reference's default params (the
end_to_end_run_epoch side line of bench.py): where the host time goes."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402

from ggnn_amd.batching import synthetic_treebank  # noqa: E402
from ggnn_amd.model import DenseGGNNChemModel  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    raw = synthetic_treebank(1200, seed=2)
    m = DenseGGNNChemModel(num_edge_types=46, output_size_edges=12, pos_size=46, vocab_size=39549,
                           params={"compact_adjacency": True}, seed=0, device=dev)
    train = m.process_raw_graphs(raw[:1000], True)
    valid = m.process_raw_graphs(raw[1000:], False)
    m.run_epoch("warm-up", train, True)
    pr = cProfile.Profile()
    pr.enable()
    tr = m.run_epoch("train", train, True)
    va = m.run_epoch("valid", valid, False)
    pr.disable()
    print("train inst/s %.1f  valid inst/s %.1f" % (tr[3], va[3]))
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)
