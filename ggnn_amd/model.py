"""Drop-in ``DenseGGNNChemModel`` for the propagation hot path.

Mirrors the part of the reference class (chem_tensorflow_dense.py:147-437 and
chem_tensorflow.py:70-136) that the hot path reads, with the same names:

* ``params['hidden_size', 'num_timesteps', 'use_edge_bias', ...]``
  (``default_params``, chem_tensorflow.py:77-112, chem_tensorflow_dense.py:152-161)
* ``num_edge_types`` (C = 2 * num_edge_types adjacency channels, :192-206)
* ``weights['edge_weights', 'edge_biases', 'edge_weights_fixed',
  'edge_biases_fixed', 'node_gru']`` (``prepare_specific_graph_model``, :163-241)
* ``placeholders`` -- here a feed dict keyed by name; ``feed()`` stages a
  minibatch produced by ``make_minibatch_iterator`` (the reference's
  ``sess.run(feed_dict=...)``, chem_tensorflow.py:595)
* ``compute_final_node_representations(initial_node_representations,
  fixed_ts=None)`` -> [b, v, h] (:312-340), differentiable: its backward is the
  engine's HIP backward (the reference's TF autodiff, chem_tensorflow.py:496)
* ``process_raw_graphs`` / ``make_minibatch_iterator`` (``BtbBatching``)
* ``save_progress`` / ``restore_progress`` in the reference's pickle format
  (chem_tensorflow.py:796-855; ``checkpoint.py``) and the host LAS/UAS scoring
  ``get_las_uas`` / ``evaluate_batch`` (chem_tensorflow_dense.py:1160-1215,
  1304-1319; ``evaluation.py``)
* the callers either side of the path:
  ``get_initial_node_representation`` (embedding front-end, :264-306),
  ``gated_regression`` + the btb loss (:439-516, chem_tensorflow.py:326-421)
  via ``build_loss()``, and ``train_step()`` (loss -> backward -> clip + Adam,
  chem_tensorflow.py:483-506) -- all on the HIP library (``heads.py``).

The arithmetic runs in libggnn.so; torch tensors only hold device memory and
carry the autograd graph around the call.
"""
from __future__ import annotations

import random
import time
from collections import OrderedDict

import numpy as np
import torch

from . import checkpoint as _ckpt
from . import dist as _dist
from . import evaluation as _eval
from .batching import BtbBatching, ThreadedIterator
from .dist import FlatTrainBuffer
from .engine import PropagationEngine
from .graphs import CapturedStep, PinnedRing, StepLayout, edge_arrays
from .heads import SMALL_NUMBER, EmbedFunction, EmbeddingFrontEnd, HeadsFunction, OutputHeads, word_inputs_tensor
from .optim import ClipAdam
from .upload import Uploader

GRU_KEYS = ("gates_kernel", "gates_bias", "candidate_kernel", "candidate_bias")


def mlp_init(shape, rng):
    """utils.py MLP.init_weights: sqrt(6/(in+out)) * (2*rand - 1)."""
    return (np.sqrt(6.0 / (shape[-2] + shape[-1])) * (2 * rng.rand(*shape).astype(np.float32) - 1)).astype(np.float32)


def glorot_init(shape, rng=None):
    """U(+-sqrt(6/(fan_in+fan_out))) on the last two dims (utils.py:11-14)."""
    rng = np.random if rng is None else rng
    lim = np.sqrt(6.0 / (shape[-2] + shape[-1]))
    return rng.uniform(low=-lim, high=lim, size=shape).astype(np.float32)


class _StepFeed:
    """One step's inputs as the library calls take them: device tensors
    (word_inputs, labels), the seeds as values or as device addresses
    (seed_device, GGNN_SEED_DEVICE), target_num as a number or a device
    scalar, the engine and heads that run the step and how the engine stages
    the batch's adjacency."""

    def __init__(self, wi, seeds, seed_values, seed_device, labels, target_num, engine, heads, stage, b, v,
                 target_num_value=None):
        self.wi, self.seeds, self.seed_values, self.seed_device = wi, seeds, seed_values, seed_device
        self.labels, self.target_num, self.engine, self.heads, self.stage = labels, target_num, engine, heads, stage
        self.b, self.v = b, v
        self.target_num_value = target_num if target_num_value is None else target_num_value


class _Propagate(torch.autograd.Function):
    """h_T = GGNN_T(h0; W, beta, GRU) through the HIP engine."""

    @staticmethod
    def forward(ctx, h0, W, beta, Wg, bg, Wc, bc, engine, T, edge_keep=1.0, state_keep=1.0, seed=0):
        weights = {"edge_weights": W.contiguous(), "edge_biases": beta.contiguous() if beta is not None else None,
                   "gates_kernel": Wg.contiguous(), "gates_bias": bg.contiguous(),
                   "candidate_kernel": Wc.contiguous(), "candidate_bias": bc.contiguous()}
        pack = engine.pack_weights(weights, T=T, edge_keep=edge_keep, seed=seed, batch=True)
        # (autograd runs Function.forward with grad mode off: ask the ctx)
        training = any(ctx.needs_input_grad[:7])
        out = engine.forward(h0.contiguous(), pack, T, training=training, state_keep=state_keep)
        ctx.engine = engine
        ctx.generation = engine.generation
        ctx.has_beta = beta is not None
        ctx.beta_shape = None if beta is None else tuple(beta.shape)
        ctx.pack = pack
        return out

    @staticmethod
    def backward(ctx, g_out):
        eng = ctx.engine
        if eng.generation != ctx.generation:
            raise RuntimeError("the engine ran another forward since this output was produced; "
                               "call backward before re-using the same call site")
        g = eng.backward(g_out.contiguous())
        db = g["edge_biases"]
        if ctx.has_beta and db is not None:
            db = db.view(ctx.beta_shape)
        return (g["h0"], g["edge_weights"], db if ctx.has_beta else None, g["gates_kernel"], g["gates_bias"],
                g["candidate_kernel"], g["candidate_bias"], None, None, None, None, None)


class DenseGGNNChemModel(BtbBatching):
    """Hot-path subset of the reference's DenseGGNNChemModel (btb task)."""

    def __init__(self, args=None, params=None, num_edge_types=None, output_size_edges=12, pos_size=46,
                 bucket_max_nodes=120, device=None, seed=None, precision="fp32", vocab_size=1000, max_nodes=None,
                 embedding_sizes=None, rank=0, world_size=1, group=None):
        """rank, world_size, group: data-parallel training (one process per GPU,
        ``torch.distributed`` initialised by the caller, e.g. dist.init_from_env):
        run_epoch then draws this rank's share of every global step's batches
        and train_step sums the flat gradient buffer over the group (RCCL)."""
        self.args = dict(args or {"--pr": "btb"})
        self.rank, self.world_size, self.group = int(rank), int(world_size), group
        if not 0 <= self.rank < self.world_size:
            raise ValueError("rank %d outside world_size %d" % (self.rank, self.world_size))
        self.params = self.default_params()
        if params:
            self.params.update(params)
        if num_edge_types is None:
            raise ValueError("num_edge_types is required (len(dep_list)+1 in the reference, "
                             "chem_tensorflow.py:198)")
        self.num_edge_types = int(num_edge_types)
        self.output_size_edges = int(output_size_edges)
        self.pos_size = int(pos_size)
        self.bucket_max_nodes = int(bucket_max_nodes)
        # front-end sizes (chem_tensorflow.py:184-189; vocab/max_nodes come from
        # the treebank lists there).  The reference's concat is 80+50+100+80 =
        # 310 wide, so hidden_size < 310 needs smaller embeddings:
        # embedding_sizes = dict(loc=, pos=, word=, edge=)
        es = dict(loc=80, pos=50, word=100, edge=50)
        es.update(embedding_sizes or {})
        self.loc_embedding_size, self.pos_embedding_size = int(es["loc"]), int(es["pos"])
        self.word_embedding_size, self.edge_embedding_size = int(es["word"]), int(es["edge"])
        self.vocab_size = int(vocab_size)
        self.max_nodes = int(max_nodes if max_nodes is not None else self.bucket_max_nodes)
        self.precision = precision
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.placeholders = {}
        self.weights = {}
        self.ops = {}
        self._engines = {}
        self._up_labels, self._up_labels_e = Uploader(), Uploader()
        # the reference seeds Python's and numpy's global RNGs here
        # (chem_tensorflow.py:174-175): minibatch_schedule shuffles with the
        # global numpy RNG, so ranks of a data-parallel job that construct their
        # models alike run the same schedule (run_epoch checks that they do)
        random.seed(self.params["random_seed"])
        np.random.seed(self.params["random_seed"])
        rs = self.params["random_seed"] if seed is None else seed
        self._rng = np.random.RandomState(rs)
        self.prepare_specific_graph_model()

    # ------------------------------------------------------------- params
    def default_params(self):
        """chem_tensorflow.py:77-112 (btb) + chem_tensorflow_dense.py:152-161."""
        return {
            "batch_size": 20, "num_epochs": 200, "patience": 15, "learning_rate": 0.003,
            "clamp_gradient_norm": 1.0, "out_layer_dropout_keep_prob": 0.85, "emb_dropout_keep_prob": 0.55,
            "hidden_size": 400, "num_timesteps": 4, "use_graph": True, "tie_fwd_bkwd": True,
            "task_ids": [0], "random_seed": 0, "output_size": 150,
            "graph_state_dropout_keep_prob": 0.9, "task_sample_ratios": {}, "use_edge_bias": True,
            "edge_weight_dropout_keep_prob": 1,
            "compact_adjacency": False,   # not in the reference: edge-list feed (ggnn_set_adjacency_edges)
            "hip_graphs": True,           # not in the reference: captured steps for edge-list feeds (graphs.py)
            "hip_graph_cache_mb": 16384,  # not in the reference: device memory the captured steps may hold
        }

    @property
    def num_channels(self) -> int:
        return 2 * self.num_edge_types

    # ------------------------------------------------------------ weights
    def prepare_specific_graph_model(self) -> None:
        """Create the path's variables with the reference's initialisers
        (chem_tensorflow_dense.py:202-212, GRUCell defaults :238)."""
        h, C = self.params["hidden_size"], self.num_channels
        dev = self.device
        t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev, requires_grad=True)
        self.weights["edge_weights"] = t(glorot_init([C, h, h], self._rng))
        self.weights["edge_weights_fixed"] = t(glorot_init([C, h, h], self._rng))
        if self.params["use_edge_bias"]:
            self.weights["edge_biases"] = t(np.zeros([C, 1, h], np.float32))
            self.weights["edge_biases_fixed"] = t(np.zeros([C, 1, h], np.float32))
        self.weights["node_gru"] = {
            "gates_kernel": t(glorot_init([2 * h, 2 * h], self._rng)),
            "gates_bias": t(np.ones([2 * h], np.float32)),
            "candidate_kernel": t(glorot_init([2 * h, h], self._rng)),
            "candidate_bias": t(np.zeros([h], np.float32)),
        }
        # front-end tables (chem_tensorflow_dense.py:214-235; tf.get_variable's
        # default initializer is glorot-uniform)
        self.weights["loc_embeddings"] = t(glorot_init([self.max_nodes, self.loc_embedding_size], self._rng))
        self.weights["head_loc_embeddings"] = t(glorot_init([self.max_nodes, self.loc_embedding_size], self._rng))
        self.weights["pos_embeddings"] = t(glorot_init([self.pos_size, self.pos_embedding_size], self._rng))
        self.weights["word_embeddings"] = t(glorot_init([self.vocab_size, self.word_embedding_size], self._rng))
        self.weights["edge_embeddings"] = t(glorot_init([self.num_edge_types + 1, self.edge_embedding_size],
                                                        self._rng))
        # out layers (chem_tensorflow.py:332-341): MLP(in, out, []) = one W, b;
        # the regression_transform MLPs are built but unused by btb (:466)
        o, oe = self.params["output_size"], self.output_size_edges
        for task_id in self.params["task_ids"]:
            for name, shape in (("regression_gate_task%i", [2 * h, o]), ("regression_gate_task_edges%i", [2 * h, oe]),
                                ("regression_transform_task%i", [h, o]),
                                ("regression_transform_task_edges%i", [h, oe])):
                self.weights[name % task_id] = {"weights": [t(mlp_init(shape, self._rng))],
                                                "biases": [t(np.zeros([shape[1]], np.float32))]}
        self._front_end = None
        self._heads = None
        self._flat = None
        self._rows = None          # the word segment's lookup rows / ids (sparse data-parallel reduction)
        # hipGraph-captured steps by batch shape (graphs.py), least recently
        # used first; bounded by params['hip_graph_cache_mb'] (_evict_graphs)
        self._graphs = OrderedDict()
        self._ring = None
        # batches by path: captured-step replays, first batches of a shape
        # (eager, on the step's device inputs), the plain eager path
        self.graph_stats = {"captured": 0, "replayed": 0, "uncaptured": 0, "eager": 0, "evicted": 0, "cache_bytes": 0}
        self.lookup_sqnorm = {}
        self.optimizer = None

    def _seed(self) -> int:
        """A fresh 64-bit Philox seed from the model's RandomState (a new mask
        per step, like TF's stateful RNG).  Rank r of a data-parallel job XORs
        a rank constant in, so the ranks' masks are independent (rank 0, and a
        single process, keep the plain draw)."""
        s = int(self._rng.randint(0, 2 ** 31 - 1)) << 32 | int(self._rng.randint(0, 2 ** 31 - 1))
        return s ^ ((self.rank * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)

    def parameters(self):
        ps = [self.weights["edge_weights"], self.weights["edge_weights_fixed"]]
        if self.params["use_edge_bias"]:
            ps += [self.weights["edge_biases"], self.weights["edge_biases_fixed"]]
        ps += [self.weights["node_gru"][k] for k in GRU_KEYS]
        return ps

    def trainable_variables(self):
        """The variables the btb loss reaches (TF passes None gradients for the
        rest: the *_fixed twins, head_loc/edge embeddings, regression_transform)."""
        ps = [self.weights["edge_weights"]]
        if self.params["use_edge_bias"]:
            ps.append(self.weights["edge_biases"])
        ps += [self.weights["node_gru"][k] for k in GRU_KEYS]
        ps += [self.weights[k] for k in ("loc_embeddings", "pos_embeddings", "word_embeddings")]
        for task_id in self.params["task_ids"]:
            for name in ("regression_gate_task%i", "regression_gate_task_edges%i"):
                mlp = self.weights[name % task_id]
                ps += [mlp["weights"][0], mlp["biases"][0]]
        return ps

    # -------------------------------------------------------------- feeds
    def feed(self, feed_dict: dict) -> None:
        """Stage one minibatch (a dict from ``make_minibatch_iterator`` or any
        dict with ``adjacency_matrix``, ``num_vertices``, ``num_graphs``)."""
        adj = feed_dict.get("adjacency_matrix")
        self.placeholders = dict(feed_dict)
        if adj is None:
            # compact feed: edge lists only (params['compact_adjacency'])
            if feed_dict.get("adjacency_edges") is None:
                raise ValueError("feed needs adjacency_matrix or adjacency_edges")
            self.placeholders["adjacency_matrix"] = None
            self._fed = False
            return
        if not isinstance(adj, torch.Tensor):
            adj = torch.from_numpy(np.ascontiguousarray(np.asarray(adj, dtype=np.float32)))
        adj = adj.to(device=self.device, dtype=torch.float32).contiguous()
        self.placeholders["adjacency_matrix"] = adj
        b, C, v, _ = adj.shape
        if C != self.num_channels:
            raise ValueError("adjacency has %d channels, model expects 2*num_edge_types = %d" % (C, self.num_channels))
        if int(feed_dict.get("num_vertices", v)) != v or int(feed_dict.get("num_graphs", b)) != b:
            raise ValueError("num_vertices/num_graphs disagree with adjacency shape %s" % (tuple(adj.shape),))
        self._fed = False

    def _engine(self, site):
        key = (self.params["hidden_size"], self.num_channels, bool(self.params["use_edge_bias"]), site)
        eng = self._engines.get(key)
        if eng is None:
            eng = PropagationEngine(key[0], key[1], key[2], device=self.device,
                                    precision=self.precision)  # one per call site
            self._engines[key] = eng
        return eng

    # ------------------------------------------------------------ hot path
    def compute_final_node_representations(self, initial_node_representations, fixed_ts=None):
        """[b, v, h] -> [b, v, h] after T = num_timesteps (or fixed_ts) GGNN
        steps (chem_tensorflow_dense.py:312-340).  ``fixed_ts`` selects the
        ``*_fixed`` edge weights/biases, as compute_timestep_fast does (:396-412)."""
        if "adjacency_matrix" not in self.placeholders and "adjacency_edges" not in self.placeholders:
            raise RuntimeError("feed() a minibatch before compute_final_node_representations()")
        # --old (compute_timestep_normal, :350-389) is the same contraction in
        # another summation order with element-wise independent edge-weight
        # dropout, so the engine serves it too (tests: oracle ordering="old");
        # the identity task is out of scope
        if self.args.get("--pr", "btb") != "btb":
            raise NotImplementedError("only --pr btb is supported by the engine")
        T = self.params["num_timesteps"] if fixed_ts is None else int(fixed_ts)
        # compute_timestep_fast picks the *_fixed twins when fixed_ts is given
        # (:396-412); compute_timestep_normal (--old, :350-389) always uses the
        # main edge_weights / edge_biases
        fixed = fixed_ts is not None and not self.args.get("--old")
        W = self.weights["edge_weights_fixed"] if fixed else self.weights["edge_weights"]
        beta = None
        if self.params["use_edge_bias"]:
            beta = self.weights["edge_biases_fixed"] if fixed else self.weights["edge_biases"]
        h0 = initial_node_representations
        if not isinstance(h0, torch.Tensor):
            h0 = torch.from_numpy(np.ascontiguousarray(np.asarray(h0, dtype=np.float32)))
        h0 = h0.to(device=self.device, dtype=torch.float32)
        eng = self._engine("main" if fixed_ts is None else "fixed")
        self._stage_adjacency(eng)
        gru = self.weights["node_gru"]
        # dropout as fed (chem_tensorflow_dense.py:860-861 training, :938-940 eval);
        # a fresh Philox seed per call = fresh masks per step, like TF's stateful RNG
        edge_keep, state_keep = self._path_keeps()
        seed = self._seed()
        out = _Propagate.apply(h0, W, beta, gru["gates_kernel"], gru["gates_bias"],
                               gru["candidate_kernel"], gru["candidate_bias"], eng, T, edge_keep, state_keep, seed)
        self.last_dropout = dict(edge_keep=edge_keep, state_keep=state_keep, seed=seed)
        self.ops["final_node_representations" if fixed_ts is None else "second_node_representations"] = out
        return out

    def _stage_adjacency(self, eng) -> None:
        if self.placeholders["adjacency_matrix"] is not None:
            eng.set_adjacency(self.placeholders["adjacency_matrix"])
        else:
            eng.set_adjacency_edges(self.placeholders["adjacency_edges"], int(self.placeholders["num_vertices"]),
                                    self.num_edge_types)

    def _path_keeps(self):
        """(edge_weight_dropout_keep_prob, graph_state_keep_prob) as fed."""
        return (float(self.placeholders.get("edge_weight_dropout_keep_prob", 1.0)),
                float(self.placeholders.get("graph_state_keep_prob", 1.0)))

    # ------------------------------------------------- §8f rank 1: callers
    def _front_end_segments(self):
        """(tables, word_inputs columns) of the btb front-end in concat order."""
        W = self.weights
        return (W["loc_embeddings"], W["pos_embeddings"], W["word_embeddings"], W["loc_embeddings"]), (0, 1, 2, 3)

    def get_initial_node_representation(self):
        """btb front-end (chem_tensorflow_dense.py:264-306): lookups of
        word_inputs columns 0 (loc), 1 (pos), 2 (word), 3 (head loc, the loc
        table again), each dropped out with emb_dropout_keep_prob, concatenated
        and zero-padded to hidden_size.  Columns 4, 5 (head POS, edge) are
        looked up by the reference but unused; they are not gathered here."""
        if "word_inputs" not in self.placeholders:
            raise RuntimeError("feed() a minibatch with word_inputs first")
        h = self.params["hidden_size"]
        width = self.loc_embedding_size * 2 + self.pos_embedding_size + self.word_embedding_size
        if width > h:
            raise ValueError("embedding concat width %d > hidden_size %d: the reference's tf.pad fails here "
                             "(SURVEY F7); pass smaller embedding_sizes" % (width, h))
        tables, cols = self._front_end_segments()
        wi = word_inputs_tensor(self.placeholders["word_inputs"], self.device,
                                {c: tb.shape[0] for tb, c in zip(tables, cols)})
        keep = float(self.placeholders.get("emb_dropout_keep_prob", 1.0))
        seed = self._seed()
        if self._front_end is None:
            self._front_end = EmbeddingFrontEnd(h)
        h0 = EmbedFunction.apply(self._front_end, self, wi, keep, seed, cols, *tables)
        self.last_embed = dict(keep=keep, seed=seed)
        self.ops["initial_node_representations"] = h0
        return h0

    def build_loss(self, task_id=0):
        """make_model for btb (chem_tensorflow.py:326-421): h0 -> h_T -> both
        gated_regression heads on [h_T, h0] -> loss = heads CE + edges CE, each
        over task_target_num = sum(target_mask[task]) + SMALL_NUMBER."""
        h0 = self.get_initial_node_representation()
        hT = self.compute_final_node_representations(h0)
        b, v, h = hT.shape
        o, oe = self.params["output_size"], self.output_size_edges
        labels = self._head_labels(b, v)
        target_num = float(self._target_count(task_id) + SMALL_NUMBER)
        keep = self._out_keep()
        seed = self._seed()
        if self._heads is None:
            self._heads = OutputHeads(h)
        g = self.weights["regression_gate_task%i" % task_id]
        ge = self.weights["regression_gate_task_edges%i" % task_id]
        loss, probs, probs_e = HeadsFunction.apply(self._heads, labels, keep, seed, target_num, hT, h0,
                                                   g["weights"][0], g["biases"][0], ge["weights"][0], ge["biases"][0])
        self.ops["loss"] = loss
        self.ops["computed_values"] = probs.reshape(b, v * o)
        self.ops["computed_values_edges"] = probs_e.reshape(b, v * oe)
        self.last_heads = dict(keep=keep, seed=seed, target_num=target_num)
        return loss

    def _head_labels(self, b, v):
        """The two heads' targets [b, v, o] / [b, v, e_o] on the device
        (placeholders target_values_head / _edges, chem_tensorflow.py:372-376)."""
        o, oe = self.params["output_size"], self.output_size_edges
        if v > o:
            raise ValueError("num_vertices %d > output_size %d" % (v, o))
        y_h = self._up_labels(np.asarray(self.placeholders["target_values_head"], np.float32).reshape(b, v, o),
                              self.device)
        y_e = self._up_labels_e(np.asarray(self.placeholders["target_values_edges"], np.float32).reshape(b, v, oe),
                                self.device)
        return [y_h, y_e]

    def _target_count(self, task_id=0) -> float:
        """sum(target_mask[task]) of the staged batch (chem_tensorflow.py:358-360)."""
        tmask = np.asarray(self.placeholders["target_mask"], np.float64)
        return float(tmask[self.params["task_ids"].index(task_id)].sum())

    def _out_keep(self) -> float:
        return float(self.placeholders.get("out_layer_dropout_keep_prob", self.params["out_layer_dropout_keep_prob"]))

    def _heads_list(self, task_id=0):
        g = self.weights["regression_gate_task%i" % task_id]
        ge = self.weights["regression_gate_task_edges%i" % task_id]
        return [(g["weights"][0], g["biases"][0]), (ge["weights"][0], ge["biases"][0])]

    def train_buffer(self) -> FlatTrainBuffer:
        """The flat gradient / lookup-norm / loss buffer of train_step.  The
        output heads' gradients and the losses come first (one bucket, final
        before the propagation backward); with world_size > 1 and
        params['sparse_embedding_reduce'] the word table's gradient sits past
        the dense part: it is reduced as IndexedSlices (_sparse_reduce)."""
        if self._flat is None:
            params = self.trainable_variables()
            ids = {id(p): i for i, p in enumerate(params)}
            first = [ids[id(t)] for tid in self.params["task_ids"] for hw in self._heads_list(tid) for t in hw]
            sparse = [ids[id(self.weights["word_embeddings"])]] if self._sparse_reduce_on() else []
            self._flat = FlatTrainBuffer(params, n_sq=4, n_loss=2, device=self.device, first=first, sparse=sparse)
        return self._flat

    def _sparse_reduce_on(self) -> bool:
        return self.world_size > 1 and bool(self.params.get("sparse_embedding_reduce", True))

    def _lookup_rows(self):
        """The word segment's per-lookup gradient rows and ids of this rank's
        batch (persistent buffers of capacity batch_size * bucket_max_nodes,
        the same on every rank: what the ranks all-gather)."""
        if self._rows is None:
            cap = int(self.params["batch_size"]) * int(self.bucket_max_nodes)
            w = self.weights["word_embeddings"].shape[1]
            self._rows = (torch.zeros((cap, w), dtype=torch.float32, device=self.device),
                          torch.full((cap,), -1, dtype=torch.int32, device=self.device))
        return self._rows

    @staticmethod
    def _sparse_call(fl, reducer) -> bool:
        """Whether THIS step reduces the word table as IndexedSlices: the
        buffer has the sparse region and the reducer can gather (a
        dist.Reducer).  Without a reducer (a local step) or with a plain
        callable, the word table's gradient is written densely into its view
        of the buffer (and a plain callable all-reduces the whole buffer)."""
        return bool(fl.sparse) and reducer is not None and hasattr(reducer, "gather")

    def _reduce(self, fl, reducer, started=None) -> None:
        """The data-parallel reduction of one step's flat buffer: the dense
        part as (heads + losses) and the rest -- the first bucket possibly
        started already (``started``: its handle) -- and, with the sparse
        reduction on (_sparse_call), the word table as the union of every
        rank's lookups: the ranks' (rows, ids) all-gathered, accumulated in
        fixed point (exact, so the same bits on every rank).  A plain
        callable reducer sums the whole buffer in one blocking call (the word
        table dense, as the step wrote it)."""
        sparse = self._sparse_call(fl, reducer)
        if not hasattr(reducer, "start"):          # a plain callable: one blocking all-reduce
            reducer(fl.flat)
        else:
            b0, b1 = fl.buckets
            h0 = started if started is not None else reducer.start(b0)
            reducer(b1)
            reducer.wait(h0)
        if sparse:
            rows, ids = self._lookup_rows()
            g_rows, g_ids = reducer.gather(rows), reducer.gather(ids)
            if self._front_end is None:
                self._front_end = EmbeddingFrontEnd(self.params["hidden_size"])
            word = self.weights["word_embeddings"]
            tables = self._front_end_segments()[0]
            slot = next(i for i, t in enumerate(tables) if t is word)
            self._front_end.union_backward(word, fl.grads[fl.sparse[0]], g_rows.view(-1, word.shape[1]),
                                           g_ids.view(-1), fl.sq[slot:slot + 1])

    def train_step(self, feed_dict=None, grad_scale=1.0, all_reduce=None, target_count=None, task_id=0):
        """One training step (chem_tensorflow.py:483-506 + run_epoch's
        sess.run of train_step): front-end -> propagation -> heads -> loss,
        the backward of each, per-variable clip_by_norm, Adam.  Returns the
        loss (a device scalar).

        Every gradient lands in ONE flat fp32 buffer (``train_buffer()``: all
        trainable variables, the embedding tables' IndexedSlices norms and the
        per-head losses), written in place by the library's backward calls.

        Data parallel (``all_reduce``: a callable summing a tensor over the
        ranks; run_epoch passes it when world_size > 1): the loss of a global
        step is the reference's btb loss (chem_tensorflow.py:358-360,399-403)
        over the UNION of the ranks' batches, i.e. every rank normalises its
        cross-entropy by the global ``target_count`` (sum of target_mask over
        all ranks' graphs; the feed's ``global_target_count`` from the sharded
        iterator) + SMALL_NUMBER.  Then the per-rank gradients, lookup norms
        (sum of squared rows of the concatenated IndexedSlices) and losses
        simply add: one all-reduce of the flat buffer, and clip + Adam on the
        sums with grad_scale 1.  With dropout off this equals one process
        stepping the concatenated batch.  A feed with num_graphs == 0 (a rank
        without a batch in the last global step) contributes zeros."""
        if feed_dict is not None and int(feed_dict.get("num_graphs", 1)) == 0:
            return self._empty_train_step(all_reduce, grad_scale)
        if feed_dict is not None and self._graph_ok(feed_dict):
            loss = self._graph_step(feed_dict, True, task_id, target_count, all_reduce, grad_scale)
            if loss is not None:
                return loss
        self.graph_stats["eager"] += 1
        if feed_dict is not None:
            self.feed(feed_dict)
        if target_count is None:
            target_count = self.placeholders.get("global_target_count")
        fl = self.train_buffer()
        params = self.trainable_variables()
        started = []
        self._forward_backward(fl, params, None if target_count is None else float(target_count), task_id,
                               reducer=all_reduce, started=started)
        if all_reduce is not None:
            self._reduce(fl, all_reduce, started[0] if started else None)
        self._apply_gradients(fl, params, grad_scale)
        return fl.loss.sum()

    def _empty_train_step(self, all_reduce, grad_scale):
        fl = self.train_buffer()
        fl.zero_()
        if self._sparse_call(fl, all_reduce):   # no lookups of this rank in the union
            self._lookup_rows()[0].zero_()
            self._lookup_rows()[1].fill_(-1)
        if all_reduce is not None:
            self._reduce(fl, all_reduce)
        self._apply_gradients(fl, self.trainable_variables(), grad_scale)
        return fl.loss.sum()

    # ------------------------------------------- hipGraph capture (graphs.py)
    def _graph_ok(self, feed) -> bool:
        """Whether a feed can run as a captured step: a compact (edge-list)
        batch on the GPU, params['hip_graphs'] on."""
        return (bool(self.params.get("hip_graphs", True)) and self.device.type == "cuda"
                and feed.get("adjacency_matrix") is None and feed.get("adjacency_edges") is not None
                and "word_inputs" in feed and int(feed.get("num_graphs", 0)) > 0
                and self.args.get("--pr", "btb") == "btb")

    def _graph_step(self, feed, training, task_id=0, target_count=None, all_reduce=None, grad_scale=1.0):
        """One batch through its shape's captured step: stage the batch's
        inputs (one H2D copy), then replay the shape's graph.  Training: the
        train_step body (+ clip + Adam inside the graph when there is no
        all-reduce; otherwise the all-reduce and Adam follow eagerly).
        Evaluation: the build_loss forward.  Returns the loss (device
        scalar), or None when the batch does not fit a captured step (more
        edges than the b * v capacity).  A shape's first batch runs the body
        eagerly; its second is captured and replayed; later ones replay."""
        self.feed(feed)
        self._check_front_end_width()
        ph = self.placeholders
        b, v = int(ph["num_graphs"]), int(ph["num_vertices"])
        o, oe = self.params["output_size"], self.output_size_edges
        if v > o:
            raise ValueError("num_vertices %d > output_size %d" % (v, o))
        tables, cols = self._front_end_segments()
        wi = np.asarray(ph["word_inputs"]).astype(np.int64)
        for tb, c in zip(tables, cols):
            x = wi[..., c]
            if x.size and (x.min() < 0 or x.max() >= tb.shape[0]):
                raise IndexError("word_inputs[..., %d] holds index %d outside [0, %d)"
                                 % (c, int(x.max() if x.max() >= tb.shape[0] else x.min()), tb.shape[0]))
        edges, offs = edge_arrays(ph["adjacency_edges"], v, self.num_edge_types)
        if edges.shape[0] > b * v:
            return None
        if target_count is None:
            target_count = ph.get("global_target_count") if training else None
        count = self._target_count(task_id) if target_count is None else float(target_count)
        target_num = float(count + SMALL_NUMBER)
        keeps = (float(ph.get("emb_dropout_keep_prob", 1.0)),) + self._path_keeps() + (self._out_keep(),)
        adam = training and all_reduce is None
        # (grad_scale is baked into the captured Adam launch: part of the key)
        # (the word table's layout, dense or IndexedSlices, is captured too)
        sparse = bool(training) and self._sparse_call(self.train_buffer(), all_reduce)
        key = (bool(training), adam, b, v, wi.shape[-1], keeps, task_id, float(grad_scale) if adam else 1.0, sparse)
        if training:
            fl = self.train_buffer()
            params = self.trainable_variables()
            if self.optimizer is None:
                self.make_optimizer()
        cs = self._graphs.get(key)
        if cs is None:
            eng = PropagationEngine(self.params["hidden_size"], self.num_channels, bool(self.params["use_edge_bias"]),
                                    device=self.device, precision=self.precision)
            cs = CapturedStep(StepLayout(b, v, wi.shape[-1], o, oe), eng, OutputHeads(self.params["hidden_size"]),
                              self.device)
            self._graphs[key] = cs
        self._graphs.move_to_end(key)
        seeds = [self._seed() for _ in range(3)]
        step = 0
        if adam:
            self.optimizer.t += 1
            step = self.optimizer.t
        # stage the batch: pinned host buffer -> the step's device inputs
        L = cs.layout
        if self._ring is None:
            self._ring = PinnedRing()
        i, host = self._ring.acquire(L.nbytes)
        L.fill(host.numpy(), seeds, step, target_num, wi.astype(np.int32), edges, offs,
               np.asarray(ph["target_values_head"], np.float32), np.asarray(ph["target_values_edges"], np.float32))
        stream = torch.cuda.current_stream(self.device)
        cs.inputs.buf[:L.nbytes].copy_(host, non_blocking=True)
        self._ring.release(i, stream)
        inp = cs.inputs
        sf = _StepFeed(inp.wi, tuple(inp.seed_address(k) for k in range(3)), tuple(seeds), True, [inp.yh, inp.ye],
                       inp.target_num, cs.engine, cs.heads,
                       lambda eng: eng.set_adjacency_edges((inp.edges, inp.offs), v, self.num_edge_types), b, v,
                       target_num_value=target_num)

        def body():
            if training:
                # (the reducer only decides the word table's layout here: the
                # collectives run after the replay, RCCL is not captured)
                probs = self._forward_backward(fl, params, None, task_id, sf, reducer=None if adam else all_reduce)
                if adam:
                    self._apply_gradients(fl, params, grad_scale, step_dev=inp.step)
                loss = fl.loss.sum()
            else:
                probs, loss = self._forward_eval(sf, task_id)
            return {"loss": loss, "probs": probs}

        if cs.graph is None and cs.runs == 0:
            # a shape's first batch runs eagerly (on the same device inputs):
            # one-off shapes never pay for a capture
            out = body()
            self.graph_stats["uncaptured"] += 1
        else:
            if cs.graph is None:             # its second batch: capture, then replay
                g = torch.cuda.CUDAGraph()
                before = torch.cuda.memory_allocated(self.device)
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    cs.out = body()          # recorded, not executed
                cs.graph = g
                # the activations the captured body allocated live in the
                # graph's private pool for as long as the graph does
                cs.pool_bytes = max(torch.cuda.memory_allocated(self.device) - before, 0)
                self.graph_stats["captured"] += 1
                self._evict_graphs(keep=key)
            cs.graph.replay()
            out = cs.out
            self.graph_stats["replayed"] += 1
        cs.runs += 1
        if cs.runs == 1:
            self._evict_graphs(keep=key)
        probs = out["probs"]
        self.ops["computed_values"] = probs[0].reshape(b, v * o)
        self.ops["computed_values_edges"] = probs[1].reshape(b, v * oe)
        loss = out["loss"]
        if training and not adam:
            self._reduce(fl, all_reduce)
            self._apply_gradients(fl, params, grad_scale)
            # the union-batch loss: the graph's loss sum was taken before the
            # all-reduce (this rank's share), the eager path's after it
            loss = fl.loss.sum()
        self.ops["loss"] = loss
        return loss

    def _evict_graphs(self, keep=None) -> None:
        """Drop the least recently used captured steps (their graph, engine
        workspaces, heads workspace and input buffer) while the cache holds
        more than params['hip_graph_cache_mb'] of device memory.  Bucketed
        treebanks have a full and a tail batch shape per bucket, for training
        and evaluation; unbounded, their workspaces (~0.9 GB at hidden 400,
        b = 20, v = 120) grew to tens of GB per process."""
        budget = float(self.params.get("hip_graph_cache_mb", 16384)) * 2 ** 20
        total = sum(cs.nbytes() for cs in self._graphs.values())
        while total > budget and len(self._graphs) > 1:
            k = next(iter(self._graphs))
            if k == keep:
                self._graphs.move_to_end(k)
                k = next(iter(self._graphs))
            cs = self._graphs.pop(k)
            total -= cs.nbytes()
            cs.release()
            self.graph_stats["evicted"] += 1
        self.graph_stats["cache_bytes"] = int(total)

    def _forward_eval(self, sf, task_id=0):
        """build_loss's forward without autograd on a _StepFeed: front-end ->
        T-step forward -> heads + btb loss.  Returns (probs, loss sum)."""
        h = self.params["hidden_size"]
        tables, cols = self._front_end_segments()
        keep_e = float(self.placeholders.get("emb_dropout_keep_prob", 1.0))
        if self._front_end is None:
            self._front_end = EmbeddingFrontEnd(h)
        h0 = self._front_end.forward(list(zip(tables, cols)), sf.wi, keep_e, sf.seeds[0], seed_device=sf.seed_device)
        self.last_embed = dict(keep=keep_e, seed=sf.seed_values[0])
        T = self.params["num_timesteps"]
        eng = sf.engine
        sf.stage(eng)
        edge_keep, state_keep = self._path_keeps()
        W, gru = self.weights, self.weights["node_gru"]
        wts = {"edge_weights": W["edge_weights"],
               "edge_biases": W["edge_biases"] if self.params["use_edge_bias"] else None,
               "gates_kernel": gru["gates_kernel"], "gates_bias": gru["gates_bias"],
               "candidate_kernel": gru["candidate_kernel"], "candidate_bias": gru["candidate_bias"]}
        pack = eng.pack_weights(wts, T=T, edge_keep=edge_keep, seed=sf.seeds[1], seed_device=sf.seed_device,
                                batch=True)
        hT = eng.forward(h0, pack, T, training=False, state_keep=state_keep)
        self.last_dropout = dict(edge_keep=edge_keep, state_keep=state_keep, seed=sf.seed_values[1])
        keep_o = self._out_keep()
        probs, loss = sf.heads.forward(hT, h0, self._heads_list(task_id), sf.labels, keep_o, sf.seeds[2],
                                       sf.target_num, seed_device=sf.seed_device)
        self.last_heads = dict(keep=keep_o, seed=sf.seed_values[2], target_num=sf.target_num_value)
        return probs, loss.sum()

    def _apply_gradients(self, fl, params, grad_scale, step_dev=None):
        if self.optimizer is None:
            self.make_optimizer()
        tables = self._front_end_segments()[0]
        # the tables' squared lookup norms (first segment's slot per table)
        slot = {}
        for i, t in enumerate(tables):
            slot.setdefault(id(t), i)
        self.lookup_sqnorm = {k: fl.sq[i:i + 1] for k, i in slot.items()}
        sq = [self.lookup_sqnorm.get(id(p)) for p in params]
        for p, g in zip(params, fl.grads):
            p.grad = g
        self.optimizer.step(fl.grads, grad_scale=grad_scale, sqnorms=sq, step_dev=step_dev)

    def _eager_step_feed(self, task_id, target_count) -> "_StepFeed":
        """The staged batch's inputs as device tensors uploaded now, with
        fresh seed values (drawn in build_loss's order: front-end, path,
        heads) and the host target_num."""
        tables, cols = self._front_end_segments()
        wi = word_inputs_tensor(self.placeholders["word_inputs"], self.device,
                                {c: tb.shape[0] for tb, c in zip(tables, cols)})
        seeds = (self._seed(), self._seed(), self._seed())
        b, v = int(self.placeholders["num_graphs"]), int(self.placeholders["num_vertices"])
        labels = self._head_labels(b, v)
        count = self._target_count(task_id) if target_count is None else target_count
        if self._heads is None:
            self._heads = OutputHeads(self.params["hidden_size"])
        return _StepFeed(wi, seeds, seeds, False, labels, float(count + SMALL_NUMBER), self._engine("main"),
                         self._heads, self._stage_adjacency, b, v)

    def _check_front_end_width(self):
        width = self.loc_embedding_size * 2 + self.pos_embedding_size + self.word_embedding_size
        if width > self.params["hidden_size"]:
            raise ValueError("embedding concat width %d > hidden_size %d: the reference's tf.pad fails here "
                             "(SURVEY F7); pass smaller embedding_sizes" % (width, self.params["hidden_size"]))

    def _forward_backward(self, fl, params, target_count, task_id, sf=None, reducer=None, started=None):
        """The btb loss and every gradient of one staged batch, written into
        the flat buffer ``fl`` (no autograd: each backward of the library
        writes its outputs where the optimizer reads them).  ``sf``: the
        step's inputs (_StepFeed; default: uploaded from the placeholders).
        Returns the heads' probabilities."""
        if "word_inputs" not in self.placeholders:
            raise RuntimeError("feed() a minibatch with word_inputs first")
        if self.args.get("--pr", "btb") != "btb":
            raise NotImplementedError("only --pr btb is supported by the engine")
        self._check_front_end_width()
        if sf is None:
            sf = self._eager_step_feed(task_id, target_count)
        # the word table's reduction is decided per call: sparse
        # only when a gathering reducer follows; checked before any work or
        # collective is issued, so a rank cannot leave a step its peers wait in
        sparse = self._sparse_call(fl, reducer)
        if sparse:
            cap = self._lookup_rows()[0].shape[0]
            if sf.b * sf.v > cap:
                raise ValueError("batch of %d x %d nodes exceeds the word lookup-row capacity %d (batch_size x "
                                 "bucket_max_nodes)" % (sf.b, sf.v, cap))
        h = self.params["hidden_size"]
        gv = {id(p): g for p, g in zip(params, fl.grads)}
        # front-end (chem_tensorflow_dense.py:264-306)
        tables, cols = self._front_end_segments()
        keep_e = float(self.placeholders.get("emb_dropout_keep_prob", 1.0))
        if self._front_end is None:
            self._front_end = EmbeddingFrontEnd(h)
        segs = list(zip(tables, cols))
        h0 = self._front_end.forward(segs, sf.wi, keep_e, sf.seeds[0], seed_device=sf.seed_device)
        self.last_embed = dict(keep=keep_e, seed=sf.seed_values[0])
        self.ops["initial_node_representations"] = h0
        # propagation (chem_tensorflow_dense.py:312-340)
        T = self.params["num_timesteps"]
        eng = sf.engine
        sf.stage(eng)
        edge_keep, state_keep = self._path_keeps()
        W, gru = self.weights, self.weights["node_gru"]
        beta = W["edge_biases"] if self.params["use_edge_bias"] else None
        wts = {"edge_weights": W["edge_weights"], "edge_biases": beta, "gates_kernel": gru["gates_kernel"],
               "gates_bias": gru["gates_bias"], "candidate_kernel": gru["candidate_kernel"],
               "candidate_bias": gru["candidate_bias"]}
        pack = eng.pack_weights(wts, T=T, edge_keep=edge_keep, seed=sf.seeds[1], seed_device=sf.seed_device,
                                batch=True)
        hT = eng.forward(h0, pack, T, training=True, state_keep=state_keep)
        self.last_dropout = dict(edge_keep=edge_keep, state_keep=state_keep, seed=sf.seed_values[1])
        self.ops["final_node_representations"] = hT
        # heads + btb loss (chem_tensorflow_dense.py:439-516, chem_tensorflow.py:326-421)
        b, v, _ = hT.shape
        o, oe = self.params["output_size"], self.output_size_edges
        keep_o = self._out_keep()
        hl = self._heads_list(task_id)
        probs, _ = sf.heads.forward(hT, h0, hl, sf.labels, keep_o, sf.seeds[2], sf.target_num, loss_out=fl.loss,
                                    seed_device=sf.seed_device)
        self.last_heads = dict(keep=keep_o, seed=sf.seed_values[2], target_num=sf.target_num_value)
        self.ops["computed_values"] = probs[0].reshape(b, v * o)
        self.ops["computed_values_edges"] = probs[1].reshape(b, v * oe)
        _, _, dhT, dh0_heads = sf.heads.backward(hT, h0, hl, sf.labels, probs, sf.target_num,
                                                  dws=[gv[id(w)] for w, _ in hl], dbs=[gv[id(bb)] for _, bb in hl])
        if reducer is not None and started is not None and hasattr(reducer, "start"):
            # the heads' gradients and the losses are final: their reduction
            # runs on the collective's stream while the propagation backward runs
            started.append(reducer.start(fl.buckets[0]))
        # the path's backward (TF autodiff, chem_tensorflow.py:496)
        eg = {"h0": torch.empty_like(h0), "edge_weights": gv[id(W["edge_weights"])],
              "edge_biases": gv[id(beta)] if beta is not None else None,
              "gates_kernel": gv[id(gru["gates_kernel"])], "gates_bias": gv[id(gru["gates_bias"])],
              "candidate_kernel": gv[id(gru["candidate_kernel"])], "candidate_bias": gv[id(gru["candidate_bias"])]}
        eng.backward(dhT, eg)
        # the tables' gradients + IndexedSlices norms (h0 feeds the path and the heads)
        word = self.weights["word_embeddings"]
        dts = [None if (sparse and t is word) else gv[id(t)] for t in tables]
        self._front_end.backward(segs, sf.wi, eg["h0"], keep_e, sf.seeds[0], dh0_add=dh0_heads,
                                 dtables=dts, sq_out=fl.sq, seed_device=sf.seed_device)
        if sparse:
            # the word table as IndexedSlices (rows, ids): all-gathered by _reduce
            rows, ids = self._lookup_rows()
            self._front_end.lookup_rows(segs, next(i for i, t in enumerate(tables) if t is word), sf.wi, eg["h0"], keep_e, sf.seeds[0], rows, ids,
                                        dh0_add=dh0_heads, seed_device=sf.seed_device)
        return probs

    def make_optimizer(self) -> ClipAdam:
        """The reference's train step optimizer (chem_tensorflow.py:494-503) over
        ``trainable_variables()``: clip_by_norm(clamp_gradient_norm) + Adam."""
        self.optimizer = ClipAdam(self.trainable_variables(), learning_rate=self.params["learning_rate"],
                                  clamp_gradient_norm=self.params["clamp_gradient_norm"])
        self._graphs.clear()          # captured steps hold the old slots' addresses
        return self.optimizer

    # ------------------------------------------------- checkpoint / evaluation
    def save_progress(self, model_path: str, train_step: int, valid_step: int) -> None:
        """chem_tensorflow.py:796-809 (checkpoint.py)."""
        _ckpt.save_progress(self, model_path, train_step, valid_step)

    def restore_progress(self, model_path: str):
        """chem_tensorflow.py:816-855 (checkpoint.py); returns (train_step, valid_step)."""
        return _ckpt.restore_progress(self, model_path)

    get_las_uas = staticmethod(_eval.get_las_uas)  # chem_tensorflow_dense.py:1304-1319

    def evaluate_batch(self, feed_dict=None):
        """(LAS, UAS, label accuracy) of one batch from the heads' probabilities
        (``humanize_batch_results_btb``, chem_tensorflow_dense.py:1160-1215):
        runs the forward + heads (no dropout) and scores on the host."""
        if feed_dict is not None:
            self.feed(feed_dict)
        saved = {k: self.placeholders.get(k) for k in ("out_layer_dropout_keep_prob",)}
        self.placeholders["out_layer_dropout_keep_prob"] = 1.0
        try:
            with torch.no_grad():
                self.build_loss()
        finally:
            for k, v in saved.items():
                if v is None:
                    self.placeholders.pop(k, None)
                else:
                    self.placeholders[k] = v
        return self._score_batch()[:3]

    def _score_batch(self):
        """Host LAS/UAS of the staged batch from the last build_loss() (the
        heads' probabilities are the only device tensors fetched).  Returns
        (las, uas, label_acc, labels, probs, mask, labels_e, probs_e, mask_e)."""
        probs = self.ops["computed_values"].detach().cpu().numpy()
        probs_e = self.ops["computed_values_edges"].detach().cpu().numpy()
        return self._score_arrays(self.placeholders, probs, probs_e)

    def _score_arrays(self, ph, probs, probs_e):
        b = int(ph["num_graphs"])
        v = int(ph["num_vertices"])
        o, oe = self.params["output_size"], self.output_size_edges
        mask = np.asarray(ph["node_mask"], np.float32).reshape(b, v * o)
        mask_e = np.asarray(ph["node_mask_edges"], np.float32).reshape(b, v * oe)
        labels = np.asarray(ph["target_values_head"], np.float32).reshape(b, v * o)
        labels_e = np.asarray(ph["target_values_edges"], np.float32).reshape(b, v * oe)
        las, uas, uas_e = _eval.batch_las_uas(labels, probs, v, mask, labels_e, probs_e, mask_e, o, oe)
        return las, uas, uas_e, labels, probs, mask, labels_e, probs_e, mask_e

    def _fetch_batch(self, loss, feed):
        """Queue the device -> host copies of one batch's loss and heads'
        probabilities (page-locked buffers, one event) and keep the host arrays
        its scoring reads; _finish_batch waits for them.  run_epoch scores a
        batch after queueing the next one, so the host's LAS/UAS work overlaps
        the GPU step instead of alternating with it (the reference's sess.run
        returns every fetch before the host continues, chem_tensorflow.py:594)."""
        ph = dict(self.placeholders)
        dev = [loss.detach(), self.ops["computed_values"].detach(), self.ops["computed_values_edges"].detach()]
        p = {"b": int(feed["num_graphs"]), "feed": feed, "ph": ph}
        if dev[0].device.type != "cuda":
            p["host"], p["event"] = [t.cpu() for t in dev], None
            return p
        host = [self._pinned(i, t) for i, t in enumerate(dev)]
        for h, t in zip(host, dev):
            h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev[0].device))
        p["host"], p["event"] = host, ev
        return p

    def _pinned(self, slot, t):
        """A page-locked host tensor shaped like device tensor t for fetch slot
        `slot`, from a small pool (a pinned allocation per batch cost more than
        the copy).  Two sets alternate: run_epoch keeps one batch in flight."""
        pool = self.__dict__.setdefault("_pin_pool", {})
        self._pin_flip = getattr(self, "_pin_flip", 0)
        key = (slot, self._pin_flip)
        buf = pool.get(key)
        n = t.numel()
        if buf is None or buf.numel() < n or buf.dtype != t.dtype:
            buf = torch.empty(max(n, 1), dtype=t.dtype, pin_memory=True)
            pool[key] = buf
        if slot == 2:
            self._pin_flip ^= 1       # the last fetch of a batch: the next batch takes the other set
        return buf[:n].view(t.shape)

    def _finish_batch(self, p):
        """(loss, _score_arrays(...)) of a batch queued by _fetch_batch."""
        if p["event"] is not None:
            p["event"].synchronize()
        hl, hp, hpe = p["host"]
        # (copies: the pinned buffers are reused two batches later, and run_epoch
        # keeps the probabilities in its returned lists)
        return float(hl.sum()), self._score_arrays(p["ph"], hp.numpy().copy(), hpe.numpy().copy())

    def _check_schedule_agrees(self, sched) -> None:
        """Data parallel: every rank must draw the same epoch schedule (the
        rank-sharded iterator assumes it; the shuffles use the global numpy
        RNG, seeded by the constructor as chem_tensorflow.py:174-175 does).
        One collective per epoch compares a 62-bit digest of (bucket, sentence
        ids) of every batch across the ranks; a mismatch raises instead of
        silently training some batches twice and others never."""
        import hashlib

        def key(d):
            # the sentence id; without one (a dataset that carries none), the
            # element's own content: words, head locations and edge labels
            i = d.get("id")
            if i is not None:
                return i
            return tuple(tuple(d.get(k) or ()) for k in ("words_index", "words_head", "edges_index"))
        hsh = hashlib.blake2b(digest_size=8)
        for bidx, els in sched:
            hsh.update(repr((bidx, [key(d) for d in els])).encode())
        dg = int.from_bytes(hsh.digest(), "little") >> 2
        dev = self.device if torch.distributed.get_backend(self.group) == "nccl" else torch.device("cpu")
        t = torch.tensor([dg, -dg], dtype=torch.int64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=self.group)
        hi, lo = int(t[0].item()), -int(t[1].item())
        if hi != lo:
            raise RuntimeError("rank %d: the ranks drew different minibatch schedules (digest %d, range [%d, %d]); "
                               "seed np.random identically on every rank (params['random_seed'])"
                               % (self.rank, dg, lo, hi))

    # the reference's per-task "chemical accuracy" normalisers (chem_tensorflow.py:529-531)
    CHEMICAL_ACCURACIES = np.array([0.066513725, 0.012235489, 0.071939046, 0.033730778, 0.033486113, 0.004278493,
                                    0.001330901, 0.004165489, 0.004128926, 0.00409976, 0.004527465, 0.012292586,
                                    0.037467458])

    def run_epoch(self, epoch_name: str, data, is_training: bool, start_step: int = 0, verbose: bool = False):
        """One pass over ``data`` (the output of process_raw_graphs), as
        chem_tensorflow.py:528-667: minibatches built in a background thread
        (ThreadedIterator, max_queue_size 5), a training step (is_training) or a
        dropout-free forward per batch, host LAS/UAS from the heads'
        probabilities.  Returns the reference's tuple (loss, accuracies,
        error_ratios, instance_per_sec, steps, acc_las, acc_uas, all_labels,
        all_computed_values, all_num_vertices, all_masks, all_ids, all_adj_m,
        all_labels_e, all_computed_values_e, all_masks_e, acc_uas_e); for btb the
        task "accuracy" is the task loss (chem_tensorflow.py:411).

        Fetch diet: the reference's sess.run fetches 21 tensors per batch,
        among them the dense [b, 2E, v, v] adjacency, the final node states and
        the whole word-embedding table (:560-593); here only the loss and the
        two heads' probabilities leave the device.

        Data parallel (world_size > 1): each rank runs its share of every
        global step (make_minibatch_iterator(rank, world_size)); a training
        step all-reduces the flat gradient buffer once (train_step).  The loss,
        LAS/UAS sums and graph counts are summed over the ranks once at the
        end of the epoch, and instance_per_sec is all ranks' graphs over the
        slowest rank's epoch time; a training batch's loss is the global
        step's (union-batch) loss.  The per-batch lists (labels, computed
        values, ...) hold this rank's batches only."""
        loss = 0.0
        accuracies = []
        processed, steps = 0, 0
        acc_las = acc_uas = acc_uas_e = 0.0
        lists = {k: [] for k in ("labels", "cv", "nv", "mask", "ids", "adj", "labels_e", "cv_e", "mask_e")}

        def consume(p):
            # host side of one batch, run after the NEXT batch's step is queued
            nonlocal loss, processed, steps, acc_las, acc_uas, acc_uas_e
            b, feed = p["b"], p["feed"]
            batch_loss, scored = self._finish_batch(p)
            las, uas, uas_e, labels, cv, mask, labels_e, cv_e, mask_e = scored
            processed += b
            loss += batch_loss * b
            accuracies.append(np.array([batch_loss] * len(self.params["task_ids"])) * b)
            acc_las += las * b
            acc_uas += uas * b
            acc_uas_e += uas_e * b
            if verbose:
                print("Running %s, batch %i (has %i graphs). Loss so far: %.4f" % (
                    epoch_name, steps, b, loss / processed), end="\r")
            steps += 1
            for k, x in (("labels", labels), ("cv", cv), ("nv", int(feed["num_vertices"])), ("mask", mask),
                         ("ids", feed.get("sentences_id")), ("adj", feed.get("adjacency_matrix")),
                         ("labels_e", labels_e), ("cv_e", cv_e), ("mask_e", mask_e)):
                lists[k].append(x)

        start = time.time()
        pending = None
        world = self.world_size
        all_reduce = _dist.all_reduce_sum(self.group) if world > 1 else None
        if world > 1 and all_reduce is None:
            raise RuntimeError("world_size %d but torch.distributed is not initialised" % world)
        sched = self.minibatch_schedule(data, is_training)
        if world > 1:
            self._check_schedule_agrees(sched)
        it = self.make_minibatch_iterator(data, is_training, rank=self.rank, world_size=world, schedule=sched)
        for feed in ThreadedIterator(it, max_queue_size=5):
            if int(feed["num_graphs"]) == 0:     # no batch for this rank in the last global step
                if is_training:
                    self.train_step(feed, all_reduce=all_reduce)
                continue
            if is_training:
                feed["out_layer_dropout_keep_prob"] = self.params["out_layer_dropout_keep_prob"]
                batch_loss = self.train_step(feed, all_reduce=all_reduce)
            else:
                feed["out_layer_dropout_keep_prob"] = 1.0
                batch_loss = None
                if self._graph_ok(feed):
                    with torch.no_grad():
                        batch_loss = self._graph_step(feed, False)
                if batch_loss is None:
                    self.graph_stats["eager"] += 1
                    self.feed(feed)
                    with torch.no_grad():
                        batch_loss = self.build_loss()
            cur = self._fetch_batch(batch_loss, feed)
            # one batch in flight: the host scores batch k while the GPU runs k + 1
            if pending is not None:
                consume(pending)
            pending = cur
        if pending is not None:
            consume(pending)
        elapsed = time.time() - start
        acc_sum = np.sum(accuracies, axis=0) if accuracies else np.zeros(len(self.params["task_ids"]))
        if world > 1:
            # one reduction of the epoch's sums over the ranks (off the step loop)
            dev = self.device if torch.distributed.get_backend(self.group) == "nccl" else torch.device("cpu")
            tot = torch.tensor([processed, loss, acc_las, acc_uas, acc_uas_e, steps] + list(acc_sum),
                               dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(tot, group=self.group)
            mx = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX, group=self.group)
            t = tot.cpu().numpy()
            processed, loss, acc_las, acc_uas, acc_uas_e, steps = (float(t[0]), float(t[1]), float(t[2]), float(t[3]),
                                                                   float(t[4]), int(t[5]))
            acc_sum, elapsed = t[6:], float(mx.item())
        processed = max(processed, 1)
        accuracies = acc_sum / processed
        loss = loss / processed
        error_ratios = accuracies / self.CHEMICAL_ACCURACIES[self.params["task_ids"]]
        instance_per_sec = processed / elapsed
        return (loss, accuracies, error_ratios, instance_per_sec, steps, acc_las / processed, acc_uas / processed,
                lists["labels"], lists["cv"], lists["nv"], lists["mask"], lists["ids"], lists["adj"], lists["labels_e"],
                lists["cv_e"], lists["mask_e"], acc_uas_e / processed)
