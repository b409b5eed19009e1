"""Generate golden batching/adjacency fixtures from the REFERENCE's own numpy
helpers (run here, in the build container; /root/reference is not on the GPU
box).  TensorFlow and docopt are absent from the image, so
they are stubbed in sys.modules -- only the reference's numpy code runs:
graph_to_adj_mat_bd, process_raw_graphs and make_minibatch_iterator of
chem_tensorflow_dense.py.  Outputs:

* tests/golden/batching_golden.npz -- adjacency / feed / batch-order fixtures;
* tests/golden/eval_golden.npz -- the host LAS/UAS scoring of the reference's
  own adj_mat_to_target, get_las_uas and humanize_batch_results_btb
  (chem_tensorflow_dense.py:106-131, 1160-1215, 1304-1319) on real dev batches
  with seeded random head / label probabilities (quantised to uint8 levels so
  the fixture stores them exactly);
* data/wsj_std_{dev,test}_btb.json.xz -- the reference's std dev / test btb
  treebank JSON (data, xz-compressed) and data/wsj_vocab.json -- the label /
  POS lists of get_dep_and_pos_list (parser/to_graph.py:206-255) from the
  dev + test CoNLL (the train CoNLL is absent) and the vocabulary
  size from the JSON's word indices: the inputs of the --train_with_dev run
  (chem_tensorflow.py:36-45) on the GPU box, where /root/reference is absent.

    python tests/golden/make_golden.py
"""
import json
import lzma
import os
import sys
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "batching_golden.npz")
EVAL_OUT = os.path.join(HERE, "eval_golden.npz")
DATA = os.path.join(os.path.dirname(os.path.dirname(HERE)), "data")


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
    eval_fixtures(ref, m, data, feeds)
    data_fixtures(dep_in, dep_out, pos_list, max_nodes)


def eval_fixtures(ref, m, data, feeds):
    """LAS/UAS of the reference's own scoring functions on real dev batches."""
    m.args = {"--pr": "btb"}
    o, oe = m.params["output_size"], m.output_size_edges
    rng = np.random.default_rng(2024)
    out = {"output_size": o, "output_size_edges": oe, "num_edge_types": m.num_edge_types}
    nb = 0
    for bi, fd in enumerate(feeds[:6]):
        b, v = int(fd["num_graphs"]), int(fd["num_vertices"])
        labels = np.asarray(fd["target_values_head"])
        labels_e = np.asarray(fd["target_values_edges"])
        # probabilities: uint8 levels / 255 (ties when the levels are few);
        # half of the batches get the target boosted so LAS/UAS are not ~0
        levels = 255 if bi % 2 == 0 else 7
        ph = rng.integers(0, levels + 1, labels.shape).astype(np.uint8)
        pe = rng.integers(0, levels + 1, labels_e.shape).astype(np.uint8)
        if bi % 3 != 2:
            boost = rng.random(labels.shape) < 0.6
            ph = np.where((labels > 0) & boost, np.uint8(levels), ph)
            boost_e = rng.random(labels_e.shape) < 0.6
            pe = np.where((labels_e > 0) & boost_e, np.uint8(levels), pe)
        cv = ph.astype(np.float32) / np.float32(levels)
        cv_e = pe.astype(np.float32) / np.float32(levels)
        mask, mask_e = np.asarray(fd["node_mask"]), np.asarray(fd["node_mask_edges"])
        adms = np.asarray(fd["adjacency_matrix"])
        las, uas, uas_e = m.humanize_batch_results_btb(
            labels=labels, computed_values=cv, num_vertices=v, mask=mask, ids=fd["sentences_id"], adms=adms,
            labels_e=labels_e, computed_values_e=cv_e, mask_edges=mask_e)
        # per graph: the reference's target / result graphs
        _, res, tgt = m.get_results_reshaped(targets=labels, computed_values=cv, mask=mask, num_vertices=v)
        _, res_e, tgt_e = m.get_results_reshaped(targets=labels_e, computed_values=cv_e, mask=mask_e,
                                                 num_vertices=v, is_edge=True)
        graphs = []
        for i in range(b):
            tg = m.merge_head_and_edge_graph(ref.adj_mat_to_target(tgt[i]), ref.adj_mat_to_target(tgt_e[i]))
            rg_h = ref.adj_mat_to_target(res[i], is_probability=True)
            rg_e = ref.adj_mat_to_target(res_e[i], is_probability=True)
            rg = m.merge_head_and_edge_graph(rg_h, rg_e)
            l1, u1 = m.get_las_uas(tg, rg)
            graphs.append(dict(target=tg, result=rg, result_e=rg_e, las=l1, uas=u1))
        pre = "b%d_" % bi
        out[pre + "levels"] = levels
        out[pre + "probs_head"] = ph
        out[pre + "probs_edges"] = pe
        out[pre + "batch"] = bi
        out[pre + "las_uas_uase"] = np.array([las, uas, uas_e], np.float64)
        out[pre + "graphs"] = np.array(json.dumps(graphs, default=int))
        nb += 1
    out["n_batches"] = nb
    np.savez_compressed(EVAL_OUT, **out)
    print("wrote %s (%d batches)" % (EVAL_OUT, nb))


def data_fixtures(dep_in, dep_out, pos_list, max_nodes):
    os.makedirs(DATA, exist_ok=True)
    words = 0
    for src, dst in (("en-wsj-std-dev-stanford-3.3.0-tagged_btb.json", "wsj_std_dev_btb.json.xz"),
                     ("en-wsj-std-test-stanford-3.3.0-tagged_btb.json", "wsj_std_test_btb.json.xz")):
        with open(os.path.join(REF, src), "rb") as f:
            raw = f.read()
        words = max(words, max(max(d["words_index"]) for d in json.loads(raw)))
        with lzma.open(os.path.join(DATA, dst), "wb", preset=9) as f:
            f.write(raw)
    vocab = {"source": "parser/to_graph.py:206-255 get_dep_and_pos_list over the std / nivre dev + test CoNLL "
                       "(train CoNLL absent); vocab_size = 1 + max words_index of the std dev + test JSON",
             "dep_list_std": dep_in, "dep_list_nivre": dep_out, "pos_list_std": pos_list, "max_nodes": max_nodes,
             "vocab_size": words + 1}
    with open(os.path.join(DATA, "wsj_vocab.json"), "w") as f:
        json.dump(vocab, f, indent=1)
    print("wrote %s" % DATA)


if __name__ == "__main__":
    main()
