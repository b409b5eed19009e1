"""One rank of the two-rank captured-step test (tests/test_gpu_dist.py):
edge-list feeds (params compact_adjacency) with hipGraph-captured steps on
and off.  Each rank trains its batch of a pair of real dev batches for three
steps with one all-reduce per step; the captured path (first batch eager on
the step's inputs, then capture and replays) must return the same union-batch
loss and leave the same weights as the eager path.  gloo over the one GPU of
the test box.  Rank 0 writes both loss lists and the weight difference to
argv[1] (.npz)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import all_reduce_sum, init_from_env
    from ggnn_amd.model import DenseGGNNChemModel

    rank, world, _ = init_from_env("gloo")
    torch.cuda.set_device(0)
    g = np.load(os.path.join(ROOT, "tests", "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)

    def model(graphs):
        params = {"hidden_size": 128, "num_timesteps": 2, "batch_size": 8, "graph_state_dropout_keep_prob": 1.0,
                  "emb_dropout_keep_prob": 1.0, "out_layer_dropout_keep_prob": 1.0, "compact_adjacency": True,
                  "hip_graphs": graphs}
        m = DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                               output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                               bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                               embedding_sizes=dict(loc=16, pos=8, word=16, edge=8), seed=5, rank=rank,
                               world_size=world)
        # (Adam as the reference configures it: epsilon 1e-8, chem_tensorflow.py:494)
        return m

    mg, me = model(True), model(False)
    bucketed, sizes, _ = mg.process_raw_graphs(data, False)
    bidx = max(bucketed, key=lambda k: len(bucketed[k]))
    els = bucketed[bidx]
    n = len(els) // 2
    v = int(sizes[bidx])
    fa, fb = mg._make_feed(els[:n], v, False), mg._make_feed(els[n:2 * n], v, False)
    assert fa["adjacency_matrix"] is None
    count = float(np.asarray(fa["target_mask"])[0].sum() + np.asarray(fb["target_mask"])[0].sum())
    mine = (fa, fb)[rank]
    ar = all_reduce_sum()
    lg, le = [], []
    for _ in range(3):
        lg.append(float(mg.train_step(dict(mine), all_reduce=ar, target_count=count)))
        le.append(float(me.train_step(dict(mine), all_reduce=ar, target_count=count)))
    torch.cuda.synchronize()
    pg = np.concatenate([p.detach().cpu().numpy().ravel() for p in mg.trainable_variables()])
    pe = np.concatenate([p.detach().cpu().numpy().ravel() for p in me.trainable_variables()])
    st = mg.graph_stats
    if rank == 0:
        np.savez(out, graph_loss=np.array(lg), eager_loss=np.array(le), param_diff=np.abs(pg - pe).max(),
                 param_scale=np.abs(pe).max(), replayed=st["replayed"], uncaptured=st["uncaptured"],
                 eager_steps=me.graph_stats["eager"])
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
