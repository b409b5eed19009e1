"""Generate golden batching/adjacency fixtures from the REFERENCE's own numpy
helpers (run here, in the build container; /root/reference is not on the GPU
box).  TensorFlow and docopt are absent from the image, so
they are stubbed in sys.modules -- only the reference's numpy code runs:
graph_to_adj_mat_bd, process_raw_graphs and make_minibatch_iterator of
chem_tensorflow_dense.py.  Output: tests/golden/batching_golden.npz.

    python tests/golden/make_golden.py
"""
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "batching_golden.npz")


def stub_modules():
    tf = types.ModuleType("tensorflow")
    tf.compat = types.SimpleNamespace(v1=types.SimpleNamespace())
    tf.Tensor = object
    tf.float32 = "float32"
    sys.modules["tensorflow"] = tf
    dm = types.ModuleType("docopt")
    dm.docopt = lambda *a, **k: {}
    sys.modules["docopt"] = dm


def vocab_from_conll(files):
    deps, pos, max_nodes = set(), set(), 0
    for fn in files:
        last = None
        with open(os.path.join(REF, "parser", fn)) as f:
            for line in f:
                if line.strip() == "":
                    if last is not None:
                        max_nodes = max(max_nodes, int(last[0]) + 1)
                    continue
                cols = line.split("\t")
                pos.add(cols[3])
                deps.add(cols[7].strip())
                last = cols
    return sorted(deps), ["zero"] + sorted(pos), max_nodes


def main():
    stub_modules()
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "parser"))
    import chem_tensorflow_dense as ref

    dep_in, pos_list, max_nodes = vocab_from_conll(
        ["en-wsj-std-dev-stanford-3.3.0-tagged.conll", "en-wsj-std-test-stanford-3.3.0-tagged.conll"])
    dep_out, _, _ = vocab_from_conll(["en-wsj-ym-nivre-dev.conll", "en-wsj-ym-nivre-test.conll"])
    with open(os.path.join(REF, "en-wsj-std-dev-stanford-3.3.0-tagged_btb.json")) as f:
        data = json.load(f)[:48]

    m = ref.DenseGGNNChemModel({"--pr": "btb", "dummy": True})
    m.num_edge_types = len(dep_in) + 1
    m.output_size_edges = len(dep_out)
    # the train CoNLL (absent) holds tags the dev/test files lack:
    # size the POS vocabulary to cover every index present in the JSON
    m.pos_size = max(len(pos_list), 1 + max(max(d["node_features"]) for d in data))
    bs = m.get_bucket_sizes()
    m.bucket_max_nodes = int(bs[np.argmax(bs > max_nodes)])
    m.params = {"batch_size": 8, "output_size": 150, "task_ids": [0], "task_sample_ratios": {},
                "tie_fwd_bkwd": True, "hidden_size": 400, "graph_state_dropout_keep_prob": 0.9,
                "emb_dropout_keep_prob": 0.55}
    names = ["target_values_head", "target_values_edges", "target_mask", "num_graphs", "num_vertices",
             "adjacency_matrix", "node_mask", "node_mask_edges", "graph_state_keep_prob",
             "edge_weight_dropout_keep_prob", "emb_dropout_keep_prob", "sentences_id", "word_inputs",
             "target_pos", "initial_node_representation"]
    m.placeholders = {n: n for n in names}

    out = {"num_edge_types": m.num_edge_types, "output_size_edges": m.output_size_edges,
           "pos_size": m.pos_size, "bucket_max_nodes": m.bucket_max_nodes,
           "raw_json": np.array(json.dumps(data))}
    # (1) adjacency of single graphs
    for i in range(6):
        g = data[i]["graph"]
        v = int(bs[np.argmax(bs > max(max(e[0], e[2]) for e in g))])
        out["adj_%d" % i] = ref.graph_to_adj_mat_bd(g, v, m.num_edge_types).astype(np.uint8)
    # (2) evaluation-order batches
    proc = m.process_raw_graphs(data, is_training_data=False)
    feeds = list(m.make_minibatch_iterator(proc, is_training=False))
    out["n_eval_batches"] = len(feeds)
    for bi, fd in enumerate(feeds):
        out["eval%d_adjacency" % bi] = np.asarray(fd["adjacency_matrix"]).astype(np.uint8)
        out["eval%d_word_inputs" % bi] = np.asarray(fd["word_inputs"]).astype(np.int32)
        for k in ("node_mask", "node_mask_edges", "target_values_head", "target_values_edges",
                  "target_mask", "target_pos"):
            out["eval%d_%s" % (bi, k)] = np.asarray(fd[k]).astype(np.float32)
        out["eval%d_scalars" % bi] = np.array([fd["num_graphs"], fd["num_vertices"],
                                               fd["graph_state_keep_prob"], fd["emb_dropout_keep_prob"]])
        out["eval%d_ids" % bi] = np.array(fd["sentences_id"])
    # (3) training-order batches (global numpy RNG seeded as chem_tensorflow.py:175)
    np.random.seed(0)
    proc = m.process_raw_graphs(data, is_training_data=True)
    tfeeds = list(m.make_minibatch_iterator(proc, is_training=True))
    out["n_train_batches"] = len(tfeeds)
    for bi, fd in enumerate(tfeeds):
        out["train%d_ids" % bi] = np.array(fd["sentences_id"])
        out["train%d_scalars" % bi] = np.array([fd["num_graphs"], fd["num_vertices"],
                                                fd["graph_state_keep_prob"], fd["emb_dropout_keep_prob"]])
    np.savez_compressed(OUT, **out)
    print("wrote %s (%d eval batches, %d train batches)" % (OUT, len(feeds), len(tfeeds)))


if __name__ == "__main__":
    main()
