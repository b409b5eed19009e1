"""Emulated MFMA precision policies against the float64 reference
(oracle.forward_operand_policy), per timestep, on configs[2]'s synthetic data
 and on dependency-tree graphs of the real label set.  Writes
profiles/r03_precision_policies.json (CPU only; tests/test_precision_policies.py
asserts the conclusions on a smaller slice).

    python tools/precision_policies.py [b]
    python tools/precision_policies.py --backward [b]   (the fp32-parity backward's
        weight-limb policies, oracle.backward_operand_policy: all seven gradients,
        max |err| / max |ref| against the 1e-3 bar; profiles/r05_backward_policies.json)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ggnn_oracle as O  # noqa: E402

POLICIES = [("bf16", "bf16"), ("f16", "f16"), ("exact", "bf16"), ("bf16", "exact"), ("exact", "f16"),
            ("f16", "exact"), ("bf16", "bf16x2"), ("f16", "f16x2"), ("bf16x2", "bf16x2"), ("f16x2", "f16x2")]


def trees(b, v, E, seed):
    rng = np.random.default_rng(seed)
    pz = 1.0 / np.arange(1, E + 1)
    pz /= pz.sum()
    A = np.zeros((b, 2 * E, v, v))
    for g in range(b):
        n = int(rng.integers(v // 2, v + 1))
        edges = [(int(rng.integers(0, i)), int(rng.choice(E, p=pz)) + 1, i) for i in range(1, n)]
        A[g] = O.graph_to_adj_mat_bd(edges, v, E)
    return A


def table(A, h0, w, Ts):
    out = {}
    ref = {T: O.forward_operand_policy(A, h0, w, T, "exact", "exact") for T in Ts}
    for act, wt in POLICIES:
        row = {}
        for T in Ts:
            d = O.forward_operand_policy(A, h0, w, T, act, wt) - ref[T]
            row["T%d" % T] = {"nrms": float(np.sqrt(np.mean(d * d) / np.mean(ref[T] ** 2))),
                              "max_abs": float(np.abs(d).max())}
        out["act=%s,weights=%s" % (act, wt)] = row
        print(act, wt, row["T%d" % Ts[-1]], flush=True)
    return out


BWD_POLICIES = [("f16x2", "f16x2", "f16x2", "f16"), ("f16x2", "f16", "f16x2", "f16"), ("f16x2", "f16x2", "f16", "f16"),
                ("f16x2", "f16", "f16", "f16"), ("f16", "f16x2", "f16x2", "f16"),
                ("f16x2", "f16", "f8corr", "f16"),  # round 6: k_prop_bwd's corrections on the fp8 MFMA
                ("f16x2", "f8lo", "f8corr", "f16")]  # round 6, shipped: + k_gru_bwd's f16 dz with W's lo on fp8


def backward_table(A, h0, w, T, seed=14):
    A, h0 = np.asarray(A, np.float64), np.asarray(h0, np.float64)
    w = {k: np.asarray(x, np.float64) for k, x in w.items()}
    out = {}
    for name, dr in (("no_dropout", None), ("dropout_0.9", dict(edge_keep=0.9, state_keep=0.9, seed=77))):
        _, caches = O.forward(A, h0, w, T, dropout=dr)
        dhT = np.random.default_rng(seed).standard_normal(h0.shape)
        ref = O.backward_operand_policy(A, dhT, caches, w, "exact", "exact", "exact", "exact")
        rows = {}
        for pol in BWD_POLICIES:
            g = O.backward_operand_policy(A, dhT, caches, w, *pol)
            e = {k: float(np.abs(g[k] - ref[k]).max() / np.abs(ref[k]).max()) for k in ref}
            rows["act=%s,gru_wt=%s,prop_wt=%s,wgrad=%s" % pol] = {"max_nmax": max(e.values()), "per_gradient": e}
            print(name, pol, "%.2e" % max(e.values()), flush=True)
        out[name] = rows
    return out


def main_backward(b):
    A, h0 = O.synthetic_batch(b, 128, 256, 8, seed=1)
    w = O.synthetic_weights(256, 8, seed=1)
    res = {"note": "the fp32-parity backward's MFMA operand roundings (oracle.backward_operand_policy): act = dzc, "
                   "dzg, dM operands of the dh / dX chain; gru_wt = Wc^T, Wg^T in k_gru_bwd's products; prop_wt = "
                   "W_c^T in k_prop_bwd's dM W_c^T; wgrad = both operands of the weight-gradient products. Forward "
                   "caches exact, accumulation float64; value = max over the seven gradients of max |err| / "
                   "max |ref| (the fp32 bar is 1e-3). Round 5 shipped gru_wt=f16, prop_wt=f16 (hi weight limbs in k_gru_bwd and k_prop_bwd); "
                   "round 6 ships gru_wt=f8lo (f16 dz x f16 W + e5m2 dz x e4m3 W_lo), prop_wt=f8corr (both limb corrections on the fp8 MFMA).",
           "configs[2]_synthetic": {"shape": "b=%d v=128 hidden=256 C=8 T=5, SURVEY §8d seed 1" % b,
                                    "policies": backward_table(A, h0, w, 5)}}
    At = trees(b, 30, 46, 3)
    h0t = np.random.default_rng(4).uniform(-0.2, 0.2, (b, 30, 256))
    wt = O.synthetic_weights(256, 92, seed=3, parity_bias=False)
    res["dependency_trees"] = {"shape": "b=%d v=30 hidden=256 E=46 (C=92) T=5, Zipf labels" % b,
                               "policies": backward_table(At, h0t, wt, 5)}
    with open(os.path.join(ROOT, "profiles", "r06_backward_policies.json"), "w") as f:
        json.dump(res, f, indent=1)


def main():
    if "--backward" in sys.argv:
        args = [a for a in sys.argv[1:] if a != "--backward"]
        return main_backward(int(args[0]) if args else 32)
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    A, h0 = O.synthetic_batch(b, 128, 256, 8, seed=1)
    w = O.synthetic_weights(256, 8, seed=1)
    res = {"note": "forward h_T of each policy vs the float64 reference; act = rounding of the activation MFMA "
                   "operands (h, M, X, r*h), weights = of W, Wg, Wc; x2 = a hi/lo limb pair; fp32 accumulation "
                   "emulated in float64",
           "configs[2]_synthetic": {"shape": "b=%d v=128 hidden=256 C=8, Bernoulli(0.1), SURVEY §8d seed 1" % b,
                                    "policies": table(A, h0, w, (1, 3, 5))}}
    E = 46
    At = trees(b, 30, E, 3)
    rng = np.random.default_rng(4)
    h0t = rng.uniform(-0.2, 0.2, (b, 30, 256))
    wt = O.synthetic_weights(256, 2 * E, seed=3, parity_bias=False)
    res["dependency_trees"] = {"shape": "b=%d v=30 hidden=256 E=46 (C=92), Zipf labels, TF-default biases" % b,
                               "policies": table(At, h0t, wt, (5,))}
    with open(os.path.join(ROOT, "profiles", "r03_precision_policies.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
