"""One rank of the data-parallel btb TRAINING STEP of the whole drop-in model
(front-end + propagation + heads + clip/Adam), for tests/test_gpu_dist.py.
Started as a child process per rank before any GPU call (gloo over the one GPU
of the test box; the 8-GPU driver run uses RCCL, one GPU per rank).

Rank r trains on batch r of a pair (A, B) of real WSJ dev batches of one bucket,
normalised by the pair's global target count, with ONE all-reduce of the flat
buffer per step (DenseGGNNChemModel.train_step).  Rank 0 then trains a fresh
model with the same initial weights on the concatenated batch A+B in one
process and writes both results to argv[1] (.npz).  Then every rank runs one
data-parallel training epoch and one evaluation epoch of run_epoch over the
golden sentences (rank 0 saves the returned counters)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, hidden = sys.argv[1], int(sys.argv[2])
    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import all_reduce_sum, init_from_env
    from ggnn_amd.model import DenseGGNNChemModel

    rank, world, _ = init_from_env("gloo")
    torch.cuda.set_device(0)
    g = np.load(os.path.join(ROOT, "tests", "golden", "batching_golden.npz"))
    data = json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)

    def model(r=0, w=1):
        params = {"hidden_size": hidden, "num_timesteps": 3, "batch_size": 8, "graph_state_dropout_keep_prob": 1.0,
                  "emb_dropout_keep_prob": 1.0, "out_layer_dropout_keep_prob": 1.0}
        m = DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                               output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                               bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                               embedding_sizes=dict(loc=16, pos=8, word=16, edge=8), seed=5, rank=r, world_size=w)
        # (Adam as the reference configures it: epsilon 1e-8, chem_tensorflow.py:494)
        return m

    m = model(rank, world)
    bucketed, sizes, _ = m.process_raw_graphs(data, False)
    bidx = max(bucketed, key=lambda k: len(bucketed[k]))
    els = bucketed[bidx]
    n = len(els) // 2
    v = int(sizes[bidx])
    fa, fb, fab = m._make_feed(els[:n], v, False), m._make_feed(els[n:2 * n], v, False), \
        m._make_feed(els[:2 * n], v, False)
    count = float(np.asarray(fab["target_mask"])[0].sum())
    init = np.concatenate([p.detach().cpu().numpy().ravel() for p in m.trainable_variables()])
    ar = all_reduce_sum()

    def run(mm, feed, reduce, tc):
        flats, losses = [], []
        for _ in range(2):
            loss = mm.train_step(dict(feed), all_reduce=reduce, target_count=tc)
            fl = mm.train_buffer()     # (variables in trainable order: the layouts differ with world size)
            flats.append(torch.cat([g.reshape(-1) for g in fl.grads] + [fl.sq, fl.loss]).cpu().numpy().copy())
            losses.append(float(loss))
        torch.cuda.synchronize()
        return np.concatenate([p.detach().cpu().numpy().ravel() for p in mm.trainable_variables()]), \
            np.stack(flats), np.array(losses)

    dp_params, dp_flat, dp_loss = run(m, (fa, fb)[rank], ar, count)
    res = {}
    if rank == 0:
        m1 = model()
        full_params, full_flat, full_loss = run(m1, fab, None, None)
        res.update(dp_params=dp_params, full_params=full_params, dp_flat=dp_flat, full_flat=full_flat, init=init,
                   dp_loss=dp_loss, full_loss=full_loss)
    # one data-parallel epoch of run_epoch (training, then evaluation)
    np.random.seed(0)
    m2 = model(rank, world)
    tr = m2.run_epoch("dp train", m2.process_raw_graphs(data, True), True)
    va = m2.run_epoch("dp valid", m2.process_raw_graphs(data, False), False)
    if rank == 0:
        np.random.seed(0)
        single = model()
        n_train = len(list(single.make_minibatch_iterator(single.process_raw_graphs(data, True), True)))
        n_valid = len(list(single.make_minibatch_iterator(single.process_raw_graphs(data, False), False)))
        res.update(epoch=np.array([tr[0], tr[3], tr[4], tr[5], tr[6], va[0], va[3], va[4], va[5], va[6],
                                   n_train, n_valid]))
        np.savez(out, **res)
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
