"""Host-side batching for the bank-to-bank ("btb") task: the producer of the
propagation path's inputs.

Re-implements, with the same names, arguments and outputs, the numpy data path
of the reference's ``DenseGGNNChemModel``:

* ``graph_to_adj_mat_bd``      chem_tensorflow_dense.py:65-83
* ``target_to_adj_mat``        chem_tensorflow_dense.py:93-104
* ``process_raw_graphs``       chem_tensorflow_dense.py:519-582
* ``get_bucket_sizes``         chem_tensorflow_dense.py:584-585
* ``vectorize_node_features``  chem_tensorflow_dense.py:587-613 (btb branch)
* ``get_mask``                 chem_tensorflow_dense.py:633-660
* ``get_labels_padded``        chem_tensorflow_dense.py:675-696 (btb branch)
* ``make_batch``               chem_tensorflow_dense.py:734-773
* ``make_minibatch_iterator``  chem_tensorflow_dense.py:792-875
* ``get_word_inputs_padded``, ``get_target_values_edges_formatted``,
  ``get_target_values_formatted``  chem_tensorflow_dense.py:877-922

Feed dicts are keyed by placeholder NAME (the reference keys them by TF
placeholder objects whose names are these strings).  Pinned against the
reference's own helpers by ``tests/golden`` fixtures (tests/test_batching.py).
The random calls (``np.random.shuffle`` on the global numpy RNG) happen in the
reference's order so seeded training batches coincide.
"""
from __future__ import annotations

import json
import lzma
import os
from collections import defaultdict

import numpy as np

# the reference's WSJ btb treebank files (std dev / test JSON, xz-compressed)
# and their label / POS lists, written by tests/golden/make_golden.py
DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
# --train_with_dev (chem_tensorflow.py:36-45, std input bank): train on the std
# dev set, validate on the std test set (the train split is absent)
TRAIN_WITH_DEV = {"train_file": "wsj_std_dev_btb.json.xz", "valid_file": "wsj_std_test_btb.json.xz"}


def read_btb_json(path):
    """A btb treebank JSON (parser/to_graph.py's output), plain or .xz."""
    opener = lzma.open if path.endswith(".xz") else open
    with opener(path, "rt") as f:
        return json.load(f)


def wsj_model_sizes(data_dir=None):
    """The vocabulary-derived sizes of the reference's std -> nivre btb model
    (chem_tensorflow.py:183-199): num_edge_types = len(dep_list) + 1,
    output_size_edges = len(dep_list_out), pos_size = len(pos_list) (at least
    1 + the largest POS index of the JSON: the absent train CoNLL holds tags
    the dev / test files lack), vocab_size, max_nodes and bucket_max_nodes
    (the first bucket above max_nodes, :191-193)."""
    with open(os.path.join(data_dir or DATA_DIR, "wsj_vocab.json")) as f:
        voc = json.load(f)
    buckets = np.array(list(range(4, 200, 2)))
    return {"num_edge_types": len(voc["dep_list_std"]) + 1, "output_size_edges": len(voc["dep_list_nivre"]),
            "pos_size": max(len(voc["pos_list_std"]), 46), "vocab_size": int(voc["vocab_size"]),
            "max_nodes": int(voc["max_nodes"]),
            "bucket_max_nodes": int(buckets[np.argmax(buckets > int(voc["max_nodes"]))])}


def graph_to_adj_mat_bd(graph, max_n_vertices, num_edge_types):
    """[2E, v, v] float64 adjacency, row = receiving node (see module doc).
    Vectorised form of chem_tensorflow_dense.py:65-83."""
    E, v = int(num_edge_types), int(max_n_vertices)
    amat = np.zeros((2 * E, v, v))
    if len(graph) == 0:
        return amat
    g = np.asarray(graph, dtype=np.int64).reshape(-1, 3)
    src, lab, dst = g[:, 0], g[:, 1] - 1, g[:, 2]
    amat[lab, dst, src] = 1            # incoming edge, channel e-1
    amat[lab + E, src, dst] = 1        # outgoing edge, channel e-1+E
    amat[E - 1, dst, dst - 1] = 1      # previous-word edge
    amat[2 * E - 1, dst - 1, dst] = 1  # next-word edge
    return amat


def target_to_adj_mat(target, max_n_vertices, num_edge_types, output_size, tie_fwd_bkwd=True):
    """[e, v, o] one-hot target heads: node i+1 has head src with label e
    (chem_tensorflow_dense.py:93-104)."""
    amat = np.zeros((int(num_edge_types), int(max_n_vertices), int(output_size)))
    for i, (src, e) in enumerate(target):
        amat[e - 1, i + 1, src] = 1
    return amat


class ThreadedIterator:
    """Builds the next feed dicts in a background thread (utils.py:17-37): the
    host batching overlaps the GPU step.  Elements must not be None; an
    exception in the producer is re-raised in the consumer."""

    _END = object()

    def __init__(self, original_iterator, max_queue_size: int = 2):
        import queue
        import threading
        self._queue = queue.Queue(maxsize=max_queue_size)
        self._thread = threading.Thread(target=self._worker, args=(original_iterator,), daemon=True)
        self._thread.start()

    def _worker(self, it):
        try:
            for element in it:
                assert element is not None, "iterator elements must not be None"
                self._queue.put(element, block=True)
        except BaseException as e:  # pragma: no cover - surfaced in __iter__
            self._queue.put(e, block=True)
            return
        self._queue.put(self._END, block=True)

    def __iter__(self):
        while True:
            x = self._queue.get(block=True)
            if x is self._END:
                break
            if isinstance(x, BaseException):
                raise x
            yield x
        self._thread.join()


def synthetic_treebank(n_sentences, num_edge_types=46, output_size_edges=12, pos_size=46, vocab_size=39549,
                       max_nodes=119, seed=0):
    """Raw btb examples in the reference's JSON layout (keys as the parser
    writes them, parser/to_graph.py; read by process_raw_graphs): sentence
    lengths around the WSJ dev set's (mean ~25 nodes incl. ROOT, max 119;
    SURVEY App. B), one input edge [head, label, dependent] per word with
    Zipf-distributed labels 1..E-1, one target [head, label] per word.  For
    benchmarks and tests only: the treebank itself is not distributed."""
    rng = np.random.default_rng(seed)
    E = int(num_edge_types)
    pz = 1.0 / np.arange(1, E)
    pz /= pz.sum()
    out = []
    for s in range(int(n_sentences)):
        n = int(np.clip(round(rng.gamma(4.0, 6.0)), 3, max_nodes))
        heads = [int(rng.integers(0, n)) for _ in range(1, n)]
        heads = [h if h != i + 1 else 0 for i, h in enumerate(heads)]
        graph = [[heads[i - 1], int(rng.choice(E - 1, p=pz)) + 1, i] for i in range(1, n)]
        pos = [0] + [int(x) for x in rng.integers(1, pos_size, n - 1)]
        out.append({
            "graph": graph,
            "targets": [[int(rng.integers(0, n)), int(rng.integers(1, output_size_edges + 1))] for _ in range(1, n)],
            "node_features": pos,
            "node_features_target": pos,
            "words_index": [0] + [int(x) for x in rng.integers(1, vocab_size, n - 1)],
            "raw_sentence": "",
            "id": "%05d" % s,
        })
    return out


class BtbBatching:
    """Mixin with the reference's btb batching API.  Requires the attributes
    the reference reads from ``self``: ``params`` (batch_size, output_size,
    task_ids, task_sample_ratios, tie_fwd_bkwd, hidden_size,
    graph_state_dropout_keep_prob, emb_dropout_keep_prob), ``num_edge_types``,
    ``output_size_edges``, ``pos_size``, ``bucket_max_nodes``."""

    # ---------------------------------------------------------------- buckets
    def get_bucket_sizes(self):
        return np.array(list(range(4, 200, 2)))

    # ------------------------------------------------------------ per graph
    def get_pos_vector(self, node_feature, deactivate_pos=False):
        if deactivate_pos:
            return []
        vec = [0] * self.pos_size
        vec[node_feature] = 1
        return vec

    def get_dep_vector(self, node_edge, deactivate_pos=True):
        if deactivate_pos:
            return []
        vec = [0] * (self.num_edge_types + 1)
        vec[node_edge[1]] = 1
        return vec

    def vectorize_node_features(self, node_features, v, graph):
        """btb: [one-hot(node index) padded to bucket_max_nodes | one-hot(POS)]."""
        n = len(node_features)
        width = int(self.bucket_max_nodes) + int(self.pos_size)
        out = np.zeros((n, width), dtype=np.int64)
        out[np.arange(n), np.arange(n)] = 1
        out[np.arange(n), int(self.bucket_max_nodes) + np.asarray(node_features, dtype=np.int64)] = 1
        return [row for row in out]

    def get_mask(self, n_active_nodes, chosen_bucket_size, is_edge=False):
        """btb masks: [v*o] with 1 where (i < n and j < n); edge mask [v*e_o]
        with 1 where i < n (closed form of chem_tensorflow_dense.py:633-660)."""
        v, n = int(chosen_bucket_size), int(n_active_nodes)
        if is_edge:
            m = np.zeros((v, self.output_size_edges))
            m[:n, :] = 1.0
            return m.reshape(-1)
        o = self.params["output_size"]
        m = np.zeros((v, o))
        m[:n, :n] = 1.0
        return m.reshape(-1)

    def get_labels_padded(self, data_dict, chosen_bucket_size, n_active_nodes):
        return target_to_adj_mat(data_dict["targets"], chosen_bucket_size, self.output_size_edges,
                                 chosen_bucket_size, self.params.get("tie_fwd_bkwd", True))

    # ------------------------------------------------------------- datasets
    def load_data(self, file_name, is_training_data, data_dir=None, restrict=None, skip=None):
        """chem_tensorflow.py:241-269: read a btb JSON from data_dir (default:
        the repo's data/), drop the first ``skip`` graphs (--skip_data), keep
        the first ``restrict`` (--restrict_data), then process_raw_graphs."""
        data = read_btb_json(os.path.join(data_dir or DATA_DIR, file_name))
        if skip is not None and int(skip) > 0:
            data = data[int(skip):]
        if restrict is not None and int(restrict) > 0:
            data = data[:int(restrict)]
        return self.process_raw_graphs(data, is_training_data)

    def process_raw_graphs(self, raw_data, is_training_data, bucket_sizes=None):
        """Bucket graphs by max node id, densify adjacency per graph.
        Returns (bucketed, bucket_sizes, bucket_at_step)."""
        if bucket_sizes is None:
            bucket_sizes = self.get_bucket_sizes()
        bucketed = defaultdict(list)
        for d in raw_data:
            if len(d["graph"]) == 0:
                continue
            max_id = max(max(e[0], e[2]) for e in d["graph"])
            bidx = int(np.argmax(bucket_sizes > max_id))
            v = int(bucket_sizes[bidx])
            n = len(d["node_features"])
            feats = self.vectorize_node_features(d["node_features"], v, d["graph"])
            xdim = len(feats[0])
            heads = [0] + [e[0] for e in d["graph"]]
            # params['compact_adjacency']: keep only the edge list (the engine
            # stages it on the device, ggnn_set_adjacency_edges) instead of the
            # dense [2E, v, v] float64 matrix per graph
            compact = bool(self.params.get("compact_adjacency", False))
            bucketed[bidx].append({
                "adj_mat": None if compact else graph_to_adj_mat_bd(d["graph"], v, self.num_edge_types),
                "graph": d["graph"],
                "init": feats + [np.zeros(xdim, dtype=np.int64) for _ in range(v - n)],
                "labels": self.get_labels_padded(d, v, n),
                "mask": self.get_mask(n, v),
                "mask_edges": self.get_mask(n, v, is_edge=True),
                "raw_sentence": d.get("raw_sentence"),
                "id": d.get("id"),
                "words_pos": d["node_features"],
                "words_loc": list(range(n)),
                "words_index": d["words_index"],
                "words_head": heads,
                "words_head_pos": [d["node_features"][x] for x in heads],
                "edges_index": [0] + [e[1] for e in d["graph"]],
                "target_pos": d["node_features_target"],
            })
        if is_training_data:
            for bidx, bucket in bucketed.items():
                np.random.shuffle(bucket)
                for task_id in self.params["task_ids"]:
                    ratio = self.params.get("task_sample_ratios", {}).get(str(task_id))
                    if ratio is not None:
                        for ex in range(int(len(bucket) * ratio), len(bucket)):
                            bucket[ex]["labels"][task_id] = None
        bs = self.params["batch_size"]
        bucket_at_step = [bidx for bidx, data in bucketed.items() for _ in range(1 + (len(data) - 1) // bs)]
        return bucketed, bucket_sizes, bucket_at_step

    def make_batch(self, elements):
        keys = ("adj_mat", "graph", "init", "node_mask", "node_mask_edges", "sentences_id", "words_pos",
                "words_loc", "words_index", "words_head", "words_head_pos", "edges_index", "target_pos")
        batch = {k: [] for k in keys}
        batch["labels"], batch["task_masks"] = [], []
        src = {"node_mask": "mask", "node_mask_edges": "mask_edges", "sentences_id": "id"}
        for d in elements:
            for k in keys:
                batch[k].append(d[src.get(k, k)])
            vals, mask = [], []
            for tv in d["labels"]:
                vals.append(0.0 if tv is None else tv)
                mask.append(0.0 if tv is None else 1.0)
            batch["labels"].append(vals)
            batch["task_masks"].append(mask)
        return batch

    @staticmethod
    def get_word_inputs_padded(words_pos, b, v):
        out = np.zeros([b, v])
        for i, row in enumerate(words_pos):
            out[i, :len(row)] = row
        return out

    def get_target_values_edges_formatted(self, labels):
        lab = np.asarray(labels)                       # [b, e, v', v]
        b, e, v, _ = lab.shape
        return lab.sum(axis=3).transpose(0, 2, 1).reshape(b, v * e)

    def get_target_values_formatted(self, labels, no_labels=True):
        lab = np.asarray(labels)                       # [b, e, v', v]
        b, e, v, _ = lab.shape
        o = self.params["output_size"]
        out = np.zeros((b, v, o))
        out[:, :, :v] = lab.sum(axis=1)                # sum over e, pad v -> o
        return out.reshape(b, v * o)

    def minibatch_schedule(self, data, is_training):
        """The batches of one epoch as (bucket index, elements) in the order the
        reference yields them (chem_tensorflow_dense.py:792-875): the shuffles
        (bucket_at_step, then every bucket, on the global numpy RNG) happen
        before the first batch, as at the top of the reference's generator."""
        bucketed, bucket_sizes, bucket_at_step = data
        if is_training:
            np.random.shuffle(bucket_at_step)
            for _, bd in bucketed.items():
                np.random.shuffle(bd)
        counters = defaultdict(int)
        bs = self.params["batch_size"]
        out = []
        for bidx in bucket_at_step:
            out.append((bidx, bucketed[bidx][counters[bidx] * bs:(counters[bidx] + 1) * bs]))
            counters[bidx] += 1
        return out

    def target_count(self, elements, task_id=0):
        """sum(target_mask[task]) of a batch of these elements: make_batch's
        task mask is 0 for a label set to None by task_sample_ratios, else 1
        (chem_tensorflow_dense.py:757-767, chem_tensorflow.py:358-360)."""
        internal = self.params["task_ids"].index(task_id)
        return float(sum(0.0 if d["labels"][internal] is None else 1.0 for d in elements))

    def make_minibatch_iterator(self, data, is_training, rank=0, world_size=1, schedule=None):
        """Yields feed dicts keyed by placeholder name (chem_tensorflow_dense.py:792-875).

        Data parallel (world_size > 1): every rank computes the same schedule
        (the same seeded shuffles) and global step k takes its batches
        k*N .. k*N+N-1, batch k*N+r going to rank r, so N consecutive batches
        of the single-process order run at once.  Each feed carries
        ``global_target_count`` / ``global_num_graphs`` of its global step
        (train_step's loss normaliser; no communication needed).  A rank
        without a batch in the last global step gets a feed with
        num_graphs == 0 (it still joins the step's all-reduce).  ``schedule``:
        the epoch's minibatch_schedule, when the caller drew it already."""
        sched = self.minibatch_schedule(data, is_training) if schedule is None else schedule
        bucket_sizes = data[1]
        if world_size <= 1:
            for bidx, elements in sched:
                yield self._make_feed(elements, int(bucket_sizes[bidx]), is_training)
            return
        if not 0 <= rank < world_size:
            raise ValueError("rank %d outside world_size %d" % (rank, world_size))
        for k in range(0, len(sched), world_size):
            group = sched[k:k + world_size]
            count = sum(self.target_count(el) for _, el in group)
            graphs = sum(len(el) for _, el in group)
            if rank < len(group):
                bidx, elements = group[rank]
                feed = self._make_feed(elements, int(bucket_sizes[bidx]), is_training)
            else:
                feed = {"num_graphs": 0}
            feed["global_target_count"] = count
            feed["global_num_graphs"] = graphs
            yield feed

    def _make_feed(self, elements, v, is_training):
        keep = self.params.get("graph_state_dropout_keep_prob", 1.0) if is_training else 1.0
        emb_keep = self.params.get("emb_dropout_keep_prob", 1.0) if is_training else 1.0
        # the output-layer keep is fed 1.0 outside training (run_epoch, chem_tensorflow.py:586-592)
        out_keep = self.params.get("out_layer_dropout_keep_prob", 1.0) if is_training else 1.0
        batch = self.make_batch(elements)
        b = len(batch["init"])
        pad = lambda key: self.get_word_inputs_padded(batch[key], b, v)
        word_inputs = np.stack((pad("words_loc"), pad("words_pos"), pad("words_index"),
                                pad("words_head"), pad("words_head_pos"), pad("edges_index")), axis=2)
        return {
            "target_values_head": self.get_target_values_formatted(batch["labels"]),
            "target_values_edges": self.get_target_values_edges_formatted(batch["labels"]),
            "target_mask": np.transpose(batch["task_masks"], axes=[1, 0]),
            "num_graphs": b,
            "num_vertices": v,
            "adjacency_matrix": None if batch["adj_mat"][0] is None else batch["adj_mat"],
            "adjacency_edges": batch["graph"],
            "node_mask": np.array(batch["node_mask"]),
            "node_mask_edges": np.array(batch["node_mask_edges"]),
            "graph_state_keep_prob": keep,
            "edge_weight_dropout_keep_prob": keep,
            "emb_dropout_keep_prob": emb_keep,
            "out_layer_dropout_keep_prob": out_keep,
            "sentences_id": batch["sentences_id"],
            "word_inputs": word_inputs,
            "target_pos": pad("target_pos"),
        }
