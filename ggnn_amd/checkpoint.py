"""The reference's checkpoint format for the drop-in model.

``save_progress`` / ``restore_progress`` (chem_tensorflow.py:796-855) pickle a
dict ``{"params", "weights", "train_step", "valid_step"}`` whose ``weights``
maps every TF global variable name to its value.  The names below restate the
TF1 graph's naming for the variables this build holds:

* ``tf.Variable`` without a name inside ``variable_scope("graph_model")``
  (chem_tensorflow.py:314-315) -> ``graph_model/Variable:0``,
  ``graph_model/Variable_1:0``, ... in creation order
  (chem_tensorflow_dense.py:202-215: edge_weights, edge_biases,
  edge_weights_fixed, edge_biases_fixed, att_weights; no biases when
  ``use_edge_bias`` is off);
* ``get_variable`` tables -> ``graph_model/<name>:0`` (:217-235);
* the GRUCell under ``variable_scope("gru_scope")`` (:237-241) ->
  ``graph_model/gru_scope/gru_cell/{gates,candidate}/{kernel,bias}:0``;
* the output MLPs (utils.py:52-55, names ``MLP_W_layer0`` / ``MLP_b_layer0``,
  uniquified ``_1`` for the second MLP of a scope) under
  ``out_layer_task<id>/regression_gate`` and ``/regression``
  (chem_tensorflow.py:329-341);
* Adam slots ``<var>/Adam:0`` (m), ``<var>/Adam_1:0`` (v) and
  ``beta1_power:0`` / ``beta2_power:0`` (tf.compat.v1.train.AdamOptimizer,
  chem_tensorflow.py:494).  The powers are float32 as in TF, and 0.9**t
  underflows float32 near t = 1000, so the integer Adam step count is also
  stored, as the top-level key ``adam_step`` (the reference's restore reads
  only ``params``/``weights``/``train_step``/``valid_step`` and ignores it).

Parity of the names is unpinned: no TF checkpoint of the reference exists here
to compare against (TensorFlow is not installed).  Round trips
through this module are exact, and restore follows the reference's tolerance
(missing names keep their initial value, unknown names are reported).  Only
open checkpoint files you trust: like the reference, ``restore_progress``
unpickles the file.
"""
from __future__ import annotations

import math
import pickle

import numpy as np
import torch


def variable_names(model) -> dict:
    """TF variable name -> the model's tensor (reference naming, see module doc)."""
    names = {}
    w = model.weights
    order = ["edge_weights"] + (["edge_biases"] if model.params["use_edge_bias"] else [])
    order += ["edge_weights_fixed"] + (["edge_biases_fixed"] if model.params["use_edge_bias"] else [])
    for i, k in enumerate(order):
        names["graph_model/Variable%s:0" % ("" if i == 0 else "_%d" % i)] = w[k]
    for tf_name, k in (("loc_embeddings", "loc_embeddings"), ("head_loc_embeddings", "head_loc_embeddings"),
                       ("pos_embedding", "pos_embeddings"), ("word_embedding", "word_embeddings"),
                       ("edge_embeddings", "edge_embeddings")):
        names["graph_model/%s:0" % tf_name] = w[k]
    gru = w["node_gru"]
    for part, key in (("gates/kernel", "gates_kernel"), ("gates/bias", "gates_bias"),
                      ("candidate/kernel", "candidate_kernel"), ("candidate/bias", "candidate_bias")):
        names["graph_model/gru_scope/gru_cell/%s:0" % part] = gru[key]
    for task_id in model.params["task_ids"]:
        for scope, first, second in (("regression_gate", "regression_gate_task%i", "regression_gate_task_edges%i"),
                                     ("regression", "regression_transform_task%i",
                                      "regression_transform_task_edges%i")):
            for suffix, key in (("", first), ("_1", second)):
                mlp = w[key % task_id]
                base = "out_layer_task%i/%s/" % (task_id, scope)
                names[base + "MLP_W_layer0%s:0" % suffix] = mlp["weights"][0]
                names[base + "MLP_b_layer0%s:0" % suffix] = mlp["biases"][0]
    return names


def _adam_slots(model, names):
    """(name -> tensor) of the Adam state, if the model has taken a step."""
    opt = getattr(model, "optimizer", None)
    out = {}
    if opt is None:
        return out, None
    by_id = {id(t): n for n, t in names.items()}
    for p, m, v in zip(opt.params, opt.m, opt.v):
        n = by_id.get(id(p))
        if n is None:
            continue
        stem = n[:-2]  # drop ":0"
        out[stem + "/Adam:0"] = m
        out[stem + "/Adam_1:0"] = v
    return out, opt


def save_progress(model, model_path: str, train_step: int, valid_step: int) -> None:
    """chem_tensorflow.py:796-809: pickle params, every variable (and Adam
    slot) by TF name, and the step counters."""
    names = variable_names(model)
    weights = {n: t.detach().cpu().numpy().copy() for n, t in names.items()}
    slots, opt = _adam_slots(model, names)
    weights.update({n: t.detach().cpu().numpy().copy() for n, t in slots.items()})
    if opt is not None:
        weights["beta1_power:0"] = np.float32(opt.b1 ** opt.t)
        weights["beta2_power:0"] = np.float32(opt.b2 ** opt.t)
    data = {"params": dict(model.params), "weights": weights, "train_step": int(train_step),
            "valid_step": int(valid_step)}
    if opt is not None:
        data["adam_step"] = int(opt.t)
    with open(model_path, "wb") as f:
        pickle.dump(data, f, pickle.HIGHEST_PROTOCOL)


def _adam_step_count(data, opt, log=print):
    """Adam's step count t: the stored integer, else recovered from the
    float32 beta powers (beta2 ** t stays a normal float32 far longer than
    beta1 ** t, which underflows near t = 1000); None if absent.

    The recovery is approximate: TF keeps the powers as a float32 running
    product, which drifts by a few steps at large t, and beta2 ** t itself
    leaves the normal float32 range near t = 87k (beyond that nothing can be
    recovered and Adam's bias correction restarts from t = 0).  Both cases
    are logged."""
    if "adam_step" in data:
        return int(data["adam_step"])
    saved = data["weights"]
    for key, beta in (("beta2_power:0", opt.b2), ("beta1_power:0", opt.b1)):
        p = float(saved.get(key, 0.0))
        if 0.0 < p < 1.0 and p >= 1.1754944e-38:
            t = int(round(math.log(p) / math.log(beta)))
            log("Adam step count recovered as %d from the float32 %s (approximate: no integer adam_step "
                "in this checkpoint)." % (t, key))
            return t
    if any(k in saved for k in ("beta1_power:0", "beta2_power:0")):
        log("Adam step count could not be recovered from the saved beta powers (float32 range exceeded); "
            "Adam's bias correction restarts from step 0.")
    return None


def restore_progress(model, model_path: str, log=print):
    """chem_tensorflow.py:816-855: load the pickle, assign every variable the
    file names (shape-checked), keep missing ones as initialised, report
    unused names.  Adam state (slots and step count) is restored when the file
    holds it, creating the model's optimizer if it has none yet, as the
    reference's restore fills the Adam slot variables of a fresh graph.
    Returns (train_step, valid_step)."""
    with open(model_path, "rb") as f:
        data = pickle.load(f)  # the reference's format is a pickle: trusted files only
    saved = data["weights"]
    names = variable_names(model)
    if getattr(model, "optimizer", None) is None and any(n.endswith("/Adam:0") for n in saved):
        model.make_optimizer()
    slots, opt = _adam_slots(model, names)
    targets = dict(names)
    targets.update(slots)
    used = set()
    with torch.no_grad():
        for n, t in targets.items():
            if n in saved:
                val = np.asarray(saved[n], dtype=np.float32)
                if tuple(val.shape) != tuple(t.shape):
                    raise ValueError("%s: saved shape %s, model shape %s" % (n, val.shape, tuple(t.shape)))
                t.copy_(torch.from_numpy(val).to(t.device))
                used.add(n)
            elif n in names:
                log("Freshly initializing %s since no saved value was found." % n)
    if opt is not None:
        t = _adam_step_count(data, opt, log)
        if t is not None:
            opt.t = t
        used.update(n for n in ("beta1_power:0", "beta2_power:0") if n in saved)
    for n in saved:
        if n not in used and not (opt is None and ("/Adam" in n or n.startswith("beta"))):
            log("Saved weights for %s not used by model." % n)
    return data["train_step"], data["valid_step"]
