"""Host LAS/UAS evaluation of the btb task.

The reference scores each evaluated batch on the host from the heads'
probabilities (``humanize_batch_results_btb``, chem_tensorflow_dense.py:1160-1215):

* ``get_results_reshaped`` (btb branch, :1054-1079) masks the head / label
  probabilities and reshapes them to [b, 1, v, o] and [b, e, v, 1];
* ``adj_mat_to_target`` (:106-131) turns a target 0/1 tensor, or a probability
  tensor (``is_probability=True``: the arg-max), into a list of
  ``[source, edge_type]`` per receiving node 1..v-1;
* ``merge_head_and_edge_graph`` (:1279-1280) joins the head list with the label
  list; ``get_las_uas`` (:1304-1319) counts exact matches (LAS) and matching
  heads (UAS, or labels with ``is_edge``).

Pure numpy; no part of the GPU path.  Pinned by the reference's own test vectors
(``tests_chem.py:9-27, 50-88``) in ``tests/test_evaluation.py``.
"""
from __future__ import annotations

import numpy as np


def adj_mat_to_target(adj_mat, is_probability=False, true_target=None):
    """[e, v, o] -> [[source, edge_type], ...] for receiving nodes 1..v-1
    (chem_tensorflow_dense.py:106-131).  A node whose slice is all zero, or
    (0/1 input) holds no exact 1, is skipped.  The first maximum in (edge type,
    source) row-major order wins, as ``np.where(...)[..][0]`` does there.
    ``true_target`` is accepted for signature parity (only used by a disabled
    diagnostic in the reference).  Vectorised over the nodes (the per-node loop
    took half of run_epoch's host time at batch 20)."""
    a = np.asarray(adj_mat)
    num_e, num_v, num_o = a.shape
    if num_v < 2:
        return []
    # row n-1 = node n's [e, o] slice flattened in (edge type, source) order
    t = np.transpose(a[:, 1:, :], (1, 0, 2)).reshape(num_v - 1, num_e * num_o)
    mx = t.max(axis=1)
    eq = t == (mx[:, None] if is_probability else 1)
    keep = (mx != 0) & eq.any(axis=1)  # (a NaN maximum matches nothing: skipped)
    first = eq.argmax(axis=1)
    e, src = np.divmod(first[keep], num_o)
    return [[int(x), int(y) + 1] for x, y in zip(src, e)]


def get_las_uas(target_graph, result_graph, is_edge=False):
    """Labelled / unlabelled attachment score of one sentence
    (chem_tensorflow_dense.py:1304-1319).  Edges are [head, label]; UAS compares
    the head (index 0), or the label (index 1) when ``is_edge``.  Divides by the
    number of predicted edges, as the reference does."""
    idx = 1 if is_edge else 0
    las = uas = 0
    for i, r in enumerate(result_graph):
        t = target_graph[i]
        if t == r:
            las += 1
            uas += 1
        elif t[idx] == r[idx]:
            uas += 1
    n = len(result_graph)
    return las / n, uas / n


def merge_head_and_edge_graph(result_graph_l, result_graph_e):
    """[[head, _]] + [[_, label]] -> [[head, label]] (chem_tensorflow_dense.py:1279-1280)."""
    return [[x[0], y[1]] for x, y in zip(result_graph_l, result_graph_e)]


def results_reshaped_btb(targets, computed_values, mask, num_vertices, output_size, output_size_edges,
                         is_edge=False):
    """btb branch of ``get_results_reshaped`` (chem_tensorflow_dense.py:1054-1079):
    returns (mask, results, targets) as [b, 1, v, o] (heads) or [b, e, v, 1]
    (labels, ``is_edge``)."""
    v, e, o = int(num_vertices), int(output_size_edges), int(output_size)
    cv, m, t = np.asarray(computed_values), np.asarray(mask), np.asarray(targets)
    if is_edge:
        res = np.transpose(np.reshape(cv * m, [-1, v, e, 1]), [0, 2, 1, 3])
        tgt = np.transpose(np.reshape(t, [-1, v, e, 1]), [0, 2, 1, 3])
        msk = np.transpose(np.reshape(m, [-1, v, e, 1]), [0, 2, 1, 3])
        return msk, res, tgt
    return np.reshape(m, [-1, 1, v, o]), np.reshape(cv * m, [-1, 1, v, o]), np.reshape(t, [-1, 1, v, o])


def _first_max(t, is_probability):
    """adj_mat_to_target's choice for a batch: t [b, n, K] (node rows 1..v-1,
    (edge type, source) flattened).  Returns (keep [b, n] bool, first [b, n])."""
    mx = t.max(axis=2)
    eq = t == (mx[..., None] if is_probability else 1)
    return (mx != 0) & eq.any(axis=2), eq.argmax(axis=2)


def batch_las_uas(labels, computed_values, num_vertices, mask, labels_e, computed_values_e, mask_edges,
                  output_size, output_size_edges):
    """Mean (LAS, UAS, label accuracy) over a batch, as
    ``humanize_batch_results_btb`` computes them (chem_tensorflow_dense.py:1160-1215,
    without its file output): heads from the arg-max of the head
    probabilities, labels from the arg-max of the label probabilities.

    Vectorised over the batch: every graph whose four node lists (target and
    result heads and labels) keep the same nodes -- the normal case, every
    real node has a target and a non-zero probability row -- is scored from
    per-node comparisons; any other graph goes through the reference's
    list-based path (get_las_uas compares the lists by POSITION).  The
    per-graph scores are added in graph order, as the reference does, so the
    result is bit-identical (tests/test_evaluation.py: fixtures of the
    reference's own functions)."""
    _, res, tgt = results_reshaped_btb(labels, computed_values, mask, num_vertices, output_size,
                                       output_size_edges)
    _, res_e, tgt_e = results_reshaped_btb(labels_e, computed_values_e, mask_edges, num_vertices, output_size,
                                           output_size_edges, is_edge=True)
    b, v, o = tgt.shape[0], tgt.shape[2], tgt.shape[3]
    if v < 2:
        return _batch_las_uas_lists(res, tgt, res_e, tgt_e)
    # node rows 1..v-1, (edge type, source) flattened: heads [b, v-1, o] (one edge
    # type), labels [b, v-1, e] (source 0)
    kt, ft = _first_max(tgt[:, 0, 1:, :], False)
    kr, fr = _first_max(res[:, 0, 1:, :], True)
    kte, fte = _first_max(np.transpose(tgt_e[:, :, 1:, 0], (0, 2, 1)), False)
    kre, fre = _first_max(np.transpose(res_e[:, :, 1:, 0], (0, 2, 1)), True)
    same = (kt == kr).all(axis=1) & (kt == kte).all(axis=1) & (kt == kre).all(axis=1)
    n = kt.sum(axis=1)
    head_ok = (ft == fr) & kt
    lab_ok = (fte == fre) & kt
    las_n = (head_ok & lab_ok).sum(axis=1)
    uas_n = head_ok.sum(axis=1)
    lab_n = lab_ok.sum(axis=1)
    acc_las = acc_uas = acc_uas_e = 0.0
    for i in range(b):
        if same[i] and n[i] > 0:
            ni = int(n[i])
            las, uas, uas_e = int(las_n[i]) / ni, int(uas_n[i]) / ni, int(lab_n[i]) / ni
        else:
            las, uas, uas_e = _graph_las_uas(res[i], tgt[i], res_e[i], tgt_e[i])
        acc_las += las
        acc_uas += uas
        acc_uas_e += uas_e
    return acc_las / b, acc_uas / b, acc_uas_e / b


def _graph_las_uas(res, tgt, res_e, tgt_e):
    """One graph through the reference's lists (chem_tensorflow_dense.py:1179-1199)."""
    tg_h = adj_mat_to_target(tgt)
    tg_e = adj_mat_to_target(tgt_e)
    target_graph = merge_head_and_edge_graph(tg_h, tg_e)
    rg_h = adj_mat_to_target(res, is_probability=True, true_target=tg_h)
    rg_e = adj_mat_to_target(res_e, is_probability=True)
    result_graph = merge_head_and_edge_graph(rg_h, rg_e)
    las, uas = get_las_uas(target_graph, result_graph)
    _, uas_e = get_las_uas(tg_e, rg_e, is_edge=True)
    return las, uas, uas_e


def _batch_las_uas_lists(res, tgt, res_e, tgt_e):
    """batch_las_uas through the reference's per-graph lists only."""
    b = tgt.shape[0]
    acc_las = acc_uas = acc_uas_e = 0.0
    for i in range(b):
        tg_h = adj_mat_to_target(tgt[i])
        tg_e = adj_mat_to_target(tgt_e[i])
        target_graph = merge_head_and_edge_graph(tg_h, tg_e)
        rg_h = adj_mat_to_target(res[i], is_probability=True, true_target=tg_h)
        rg_e = adj_mat_to_target(res_e[i], is_probability=True)
        result_graph = merge_head_and_edge_graph(rg_h, rg_e)
        las, uas = get_las_uas(target_graph, result_graph)
        _, uas_e = get_las_uas(tg_e, rg_e, is_edge=True)
        acc_las += las
        acc_uas += uas
        acc_uas_e += uas_e
    return acc_las / b, acc_uas / b, acc_uas_e / b
