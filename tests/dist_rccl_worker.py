"""One-rank RCCL rehearsal for tests/test_gpu_dist.py: started with
WORLD_SIZE=1 and an explicit backend "nccl", so dist.init_from_env creates a
one-rank RCCL group exactly as an N-GPU run does (device_id=) and turns the
collectives on at world size 1.  Through the calls bench.py and train_step
use, it all-reduces a FlatGradients buffer written by the engine's backward
and a FlatTrainBuffer written by a whole btb training step (eager and
hipGraph-captured), checks that the one-rank sum changed nothing, then
barriers and destroys the group.  Writes a JSON verdict to argv[1]."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    out = sys.argv[1]
    import torch
    import torch.distributed as tdist
    from ggnn_amd.dist import (GRAD_ORDER, FlatGradients, all_reduce_sum, collectives_at_world_one,
                               init_from_env)
    from ggnn_amd.engine import PropagationEngine
    from ggnn_amd.model import DenseGGNNChemModel
    import ggnn_oracle as O

    rank, world, local = init_from_env("nccl")
    res = {"backend": tdist.get_backend(), "world": tdist.get_world_size(), "always": collectives_at_world_one()}
    dev = torch.device("cuda", local)

    # the propagation step's buffer (bench.py's step): engine backward -> FlatGradients
    b, v, h, C, T = 4, 128, 256, 8, 3
    A, h0 = O.synthetic_batch(b, v, h, C, seed=3)
    w = O.synthetic_weights(h, C, seed=3)
    eng = PropagationEngine(h, C, device=dev)
    wd = {k: torch.from_numpy(np.ascontiguousarray(x)).to(dev) for k, x in w.items()}
    pack = eng.pack_weights(wd, T=T)
    eng.set_adjacency(torch.from_numpy(A).to(dev))
    eng.forward(torch.from_numpy(h0).to(dev), pack, T, training=True)
    grads = FlatGradients(h, C, True, device=dev)
    gv = dict(grads.views)
    gv["h0"] = torch.empty((b, v, h), device=dev)
    eng.backward(torch.from_numpy(np.random.default_rng(1).standard_normal((b, v, h)).astype(np.float32)).to(dev), gv)
    before = grads.flat.clone()
    grads.all_reduce()
    torch.cuda.synchronize()
    res["flat_gradients_unchanged"] = bool(torch.equal(before, grads.flat))
    res["flat_gradients_bytes"] = grads.nbytes

    # the whole btb training step: FlatTrainBuffer through train_step's all_reduce
    import json as _json
    g = np.load(os.path.join(ROOT, "tests", "golden", "batching_golden.npz"))
    data = _json.loads(str(g["raw_json"]))
    vocab = 1 + max(max(d["words_index"]) for d in data)

    def model(compact):
        params = {"hidden_size": 128, "num_timesteps": 2, "batch_size": 8, "graph_state_dropout_keep_prob": 1.0,
                  "emb_dropout_keep_prob": 1.0, "out_layer_dropout_keep_prob": 1.0, "compact_adjacency": compact}
        m = DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                               output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                               bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                               embedding_sizes=dict(loc=16, pos=8, word=16, edge=8), seed=5, device=dev)
        # (Adam as the reference configures it, epsilon 1e-8, chem_tensorflow.py:494:
        # the library's reductions are order-fixed, so the two models stay bit-identical)
        return m

    ar = all_reduce_sum()
    res["all_reduce_sum_callable"] = ar is not None
    for compact in (False, True):          # eager step / hipGraph-captured step (edge-list feeds)
        m_ar, m_1 = model(compact), model(compact)
        bucketed, sizes, _ = m_ar.process_raw_graphs(data, False)
        bidx = max(bucketed, key=lambda k: len(bucketed[k]))
        feed = m_ar._make_feed(bucketed[bidx][:6], int(sizes[bidx]), False)
        la, l1 = [], []
        for _ in range(3):
            la.append(float(m_ar.train_step(dict(feed), all_reduce=ar)))
            l1.append(float(m_1.train_step(dict(feed))))
        fl = m_ar.train_buffer()
        snap = fl.flat.clone()
        ar(fl.flat)
        torch.cuda.synchronize()
        tag = "captured" if compact else "eager"
        res[tag + "_train_buffer_unchanged"] = bool(torch.equal(snap, fl.flat))
        res[tag + "_losses"] = [la, l1]
        pa = torch.cat([p.detach().reshape(-1) for p in m_ar.trainable_variables()])
        p1 = torch.cat([p.detach().reshape(-1) for p in m_1.trainable_variables()])
        res[tag + "_param_max_diff"] = float((pa - p1).abs().max())
        res[tag + "_param_scale"] = float(p1.abs().max())
        res[tag + "_graph_stats"] = dict(m_ar.graph_stats)
    tdist.barrier()
    tdist.destroy_process_group()
    res["destroyed"] = not tdist.is_initialized()
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
