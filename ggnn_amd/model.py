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

The arithmetic runs in libggnn.so; torch tensors only hold device memory and
carry the autograd graph around the call.
"""
from __future__ import annotations

import numpy as np
import torch

from .batching import BtbBatching
from .engine import PropagationEngine

GRU_KEYS = ("gates_kernel", "gates_bias", "candidate_kernel", "candidate_bias")


def glorot_init(shape, rng=None):
    """U(+-sqrt(6/(fan_in+fan_out))) on the last two dims (utils.py:11-14)."""
    rng = np.random if rng is None else rng
    lim = np.sqrt(6.0 / (shape[-2] + shape[-1]))
    return rng.uniform(low=-lim, high=lim, size=shape).astype(np.float32)


class _Propagate(torch.autograd.Function):
    """h_T = GGNN_T(h0; W, beta, GRU) through the HIP engine."""

    @staticmethod
    def forward(ctx, h0, W, beta, Wg, bg, Wc, bc, engine, T, edge_keep=1.0, state_keep=1.0, seed=0):
        weights = {"edge_weights": W.contiguous(), "edge_biases": beta.contiguous() if beta is not None else None,
                   "gates_kernel": Wg.contiguous(), "gates_bias": bg.contiguous(),
                   "candidate_kernel": Wc.contiguous(), "candidate_bias": bc.contiguous()}
        pack = engine.pack_weights(weights, T=T, edge_keep=edge_keep, seed=seed)
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
                 bucket_max_nodes=120, device=None, seed=None, precision="bf16"):
        self.args = dict(args or {"--pr": "btb"})
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
        self.precision = precision
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.placeholders = {}
        self.weights = {}
        self.ops = {}
        self._engines = {}
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

    def parameters(self):
        ps = [self.weights["edge_weights"], self.weights["edge_weights_fixed"]]
        if self.params["use_edge_bias"]:
            ps += [self.weights["edge_biases"], self.weights["edge_biases_fixed"]]
        ps += [self.weights["node_gru"][k] for k in GRU_KEYS]
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
        if self.args.get("--pr", "btb") not in ("btb",) or self.args.get("--old"):
            # the identity/--old variants compute the same contraction in another
            # order; only the btb layout is wired to the engine
            if self.args.get("--pr", "btb") != "btb":
                raise NotImplementedError("only --pr btb is supported by the engine")
        T = self.params["num_timesteps"] if fixed_ts is None else int(fixed_ts)
        W = self.weights["edge_weights"] if fixed_ts is None else self.weights["edge_weights_fixed"]
        beta = None
        if self.params["use_edge_bias"]:
            beta = self.weights["edge_biases"] if fixed_ts is None else self.weights["edge_biases_fixed"]
        h0 = initial_node_representations
        if not isinstance(h0, torch.Tensor):
            h0 = torch.from_numpy(np.ascontiguousarray(np.asarray(h0, dtype=np.float32)))
        h0 = h0.to(device=self.device, dtype=torch.float32)
        eng = self._engine("main" if fixed_ts is None else "fixed")
        if self.placeholders["adjacency_matrix"] is not None:
            eng.set_adjacency(self.placeholders["adjacency_matrix"])
        else:
            eng.set_adjacency_edges(self.placeholders["adjacency_edges"], int(self.placeholders["num_vertices"]),
                                    self.num_edge_types)
        gru = self.weights["node_gru"]
        # dropout as fed (chem_tensorflow_dense.py:860-861 training, :938-940 eval);
        # a fresh Philox seed per call = fresh masks per step, like TF's stateful RNG
        edge_keep = float(self.placeholders.get("edge_weight_dropout_keep_prob", 1.0))
        state_keep = float(self.placeholders.get("graph_state_keep_prob", 1.0))
        seed = int(self._rng.randint(0, 2 ** 31 - 1)) << 32 | int(self._rng.randint(0, 2 ** 31 - 1))
        out = _Propagate.apply(h0, W, beta, gru["gates_kernel"], gru["gates_bias"],
                               gru["candidate_kernel"], gru["candidate_bias"], eng, T, edge_keep, state_keep, seed)
        self.last_dropout = dict(edge_keep=edge_keep, state_keep=state_keep, seed=seed)
        self.ops["final_node_representations" if fixed_ts is None else "second_node_representations"] = out
        return out
