"""Two ranks (gloo, one GPU) of tests/test_gpu_dist.py::
test_sparse_word_reduction_matches_the_flat_one: the data-parallel btb step
with the word table reduced densely (one all-reduce of the flat buffer, the
round-4 path; params['sparse_embedding_reduce'] False) and as IndexedSlices
(the ranks' lookup rows all-gathered, accumulated in 64-bit fixed point;
the heads bucket started asynchronously).  Writes rank 0's comparison to
argv[1]."""
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

    def model(sparse):
        params = {"hidden_size": 128, "num_timesteps": 2, "batch_size": 8, "sparse_embedding_reduce": sparse,
                  "hip_graphs": False}
        return DenseGGNNChemModel(params=params, num_edge_types=int(g["num_edge_types"]),
                                  output_size_edges=int(g["output_size_edges"]), pos_size=int(g["pos_size"]),
                                  bucket_max_nodes=int(g["bucket_max_nodes"]), precision="fp32", vocab_size=vocab,
                                  embedding_sizes=dict(loc=16, pos=8, word=16, edge=8), seed=5, rank=rank,
                                  world_size=world)

    md, ms = model(False), model(True)
    bucketed, sizes, _ = md.process_raw_graphs(data, True)
    bidx = max(bucketed, key=lambda k: len(bucketed[k]))
    els = bucketed[bidx]
    n = len(els) // 2
    v = int(sizes[bidx])
    feed = md._make_feed(els[rank * n:(rank + 1) * n], v, True)
    count = float(np.asarray(md._make_feed(els[:2 * n], v, True)["target_mask"])[0].sum())
    ar = all_reduce_sum()
    md.train_step(dict(feed), all_reduce=ar, target_count=count)
    ms.train_step(dict(feed), all_reduce=ar, target_count=count)
    torch.cuda.synchronize()
    fd, fs = md.train_buffer(), ms.train_buffer()
    params = md.trainable_variables()
    wi = next(i for i, p in enumerate(params) if p is md.weights["word_embeddings"])
    res = {"sparse_layout": list(fs.sparse) == [wi] and not fd.sparse,
           "dense_grads_equal": all(torch.equal(a, b) for i, (a, b) in enumerate(zip(fd.grads, fs.grads)) if i != wi),
           "loss_equal": bool(torch.equal(fd.loss, fs.loss)),
           "word_grad_rel": float((fd.grads[wi] - fs.grads[wi]).abs().max() / fd.grads[wi].abs().max()),
           "word_sq_rel": float(((fd.sq - fs.sq).abs() / fd.sq.abs().clamp_min(1e-30)).max()),
           "params_equal_but_word": all(torch.equal(a.detach(), b.detach()) for i, (a, b) in
                                        enumerate(zip(params, ms.trainable_variables())) if i != wi)}
    # every rank holds the same sparse result: compare rank 1's with rank 0's
    word = fs.grads[wi].clone()
    other = ar.gather(word)
    res["ranks_agree"] = bool(torch.equal(other[0], other[1]))
    # and it is the fixed-point sum of the union of the lookups, recomputed here
    rows, ids = ms._lookup_rows()
    gr, gi = ar.gather(rows), ar.gather(ids)
    from ggnn_amd.heads import EmbeddingFrontEnd
    again = torch.empty_like(word)
    sq = torch.empty(1, device=word.device)
    EmbeddingFrontEnd(128).union_backward(ms.weights["word_embeddings"], again, gr.view(-1, rows.shape[1]),
                                          gi.view(-1), sq)
    res["union_recomputed_equal"] = bool(torch.equal(again, word))
    res["lookups"] = int((gi >= 0).sum())
    # the word table's layout is decided per call.  A sparse-layout
    # model stepped WITHOUT a reducer (a local step) writes its word gradient
    # densely, exactly as a dense-layout model does; with a plain callable
    # reducer it sums the whole buffer and equals the dense-layout Reducer step
    ml_d, ml_s = model(False), model(True)
    ml_d.train_step(dict(feed), all_reduce=None, target_count=count)
    ml_s.train_step(dict(feed), all_reduce=None, target_count=count)
    torch.cuda.synchronize()
    ld, ls = ml_d.train_buffer(), ml_s.train_buffer()
    res["local_step_word_grad_equal"] = bool(torch.equal(ld.grads[wi], ls.grads[wi])) and \
        float(ls.grads[wi].abs().max()) > 0
    res["local_step_params_equal"] = all(torch.equal(a.detach(), b.detach()) for a, b in
                                         zip(ml_d.trainable_variables(), ml_s.trainable_variables()))
    mp = model(True)
    mp.train_step(dict(feed), all_reduce=lambda t: tdist.all_reduce(t), target_count=count)
    torch.cuda.synchronize()
    fp = mp.train_buffer()
    res["plain_callable_equals_dense"] = all(torch.equal(a, b) for a, b in zip(fd.grads, fp.grads)) and \
        bool(torch.equal(fd.sq, fp.sq)) and bool(torch.equal(fd.loss, fp.loss))
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)
    tdist.barrier()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
