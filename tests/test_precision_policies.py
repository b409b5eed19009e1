"""north_star's 16-bit bar ("within ... 1e-2 bf16") on configs[2]'s own data,
decided on the oracle: the SURVEY §8d synthetic batch (b = 2 graphs of
config 3: v = 128, hidden 256, C = 8, T = 5, Bernoulli(0.1) adjacency, in-degree
~80, X rms ~2, a saturated GRU), forward with each MFMA precision policy's
operand roundings (oracle.forward_operand_policy) against the float64 reference.

The verdict (round 2, Missing 1) asked whether ANY 16-bit policy holds 1e-2
there.  What the emulation shows (numbers of the full table:
profiles/r03_precision_policies.json, tools/precision_policies.py):
  * nothing with a bf16 operand on either side does, in normalised RMS or
    max |err|: bf16 weights alone move h_T by > 2e-2 nrms, bf16 activations
    alone by > 1e-2; the engine's bf16 mode is therefore held to its
    rounding emulation and to 1e-2 on dependency trees (test_gpu_parity.py);
  * single f16 operands on both sides (GGNN_FP16) hold 1e-2 in normalised
    RMS but not in max |err| (a few saturated gates flip);
  * only hi/lo limbs on BOTH sides hold 1e-2 in max |err|: f16 pairs are the
    fp32-parity mode (<= 1e-3)."""
import numpy as np
import pytest

import ggnn_oracle as O

B, V, H, C, T = 2, 128, 256, 8, 5


@pytest.fixture(scope="module")
def case():
    A, h0 = O.synthetic_batch(B, V, H, C, seed=1)
    w = O.synthetic_weights(H, C, seed=1)
    ref = O.forward_operand_policy(A, h0, w, T, "exact", "exact")
    return A, h0, w, ref


def _err(case, act, wt):
    A, h0, w, ref = case
    d = O.forward_operand_policy(A, h0, w, T, act, wt) - ref
    return float(np.sqrt(np.mean(d * d) / np.mean(ref * ref))), float(np.abs(d).max())


def test_no_bf16_operand_policy_meets_1e_2(case):
    nrms_w, _ = _err(case, "exact", "bf16")      # bf16 weights, exact activations
    nrms_a, _ = _err(case, "bf16", "exact")      # bf16 activations, exact weights
    nrms_b, max_b = _err(case, "bf16", "bf16")   # the engine's bf16 mode
    assert nrms_w > 2e-2 and nrms_a > 1e-2 and nrms_b > 2e-2 and max_b > 1e-1, (nrms_w, nrms_a, nrms_b, max_b)
    # a bf16 hi/lo pair on the weights does not rescue bf16 activations
    nrms_x, _ = _err(case, "bf16", "bf16x2")
    assert nrms_x > 1e-2, nrms_x


def test_f16_operands_meet_1e_2_in_rms_not_in_max(case):
    nrms, mx = _err(case, "f16", "f16")          # GGNN_FP16
    assert nrms <= 1e-2 < mx, (nrms, mx)


def test_split_limbs_on_both_sides_meet_the_max_bar(case):
    nrms, mx = _err(case, "f16x2", "f16x2")      # GGNN_FP32_PARITY
    assert mx <= 1e-3 and nrms <= 1e-4, (nrms, mx)


# ---------------------------------------------------------------------------
# The fp32-parity BACKWARD's weight limbs (round 5): k_gru_bwd's products
# dzc Wc^T and dzg Wg^T and k_prop_bwd's dM W_c^T take the hi limb of the
# weights only (dz and dM stay hi/lo pairs).  Decided on the oracle
# (backward_operand_policy) against the 1e-3 bar of max |err| / max |ref| over
# all seven gradients; the full table is profiles/r05_backward_policies.json
# (tools/precision_policies.py --backward).
# ---------------------------------------------------------------------------
BWD_B = 4


@pytest.fixture(scope="module")
def bwd_case():
    A, h0 = O.synthetic_batch(BWD_B, V, H, C, seed=1)
    w = {k: x.astype(np.float64) for k, x in O.synthetic_weights(H, C, seed=1).items()}
    A, h0 = A.astype(np.float64), h0.astype(np.float64)
    _, caches = O.forward(A, h0, w, T)
    dhT = np.random.default_rng(14).standard_normal(h0.shape)
    ref = O.backward_operand_policy(A, dhT, caches, w, "exact", "exact", "exact", "exact")
    return A, dhT, caches, w, ref


def _bwd_err(case, *pol):
    A, dhT, caches, w, ref = case
    g = O.backward_operand_policy(A, dhT, caches, w, *pol)
    return max(float(np.abs(g[k] - ref[k]).max() / np.abs(ref[k]).max()) for k in ref)


def test_backward_policy_exact_equals_oracle_backward(bwd_case):
    A, dhT, caches, w, ref = bwd_case
    g = O.backward(A, dhT, caches, w)
    for k in ref:
        assert np.allclose(g[k], ref[k], rtol=1e-10, atol=1e-12), k


def test_backward_weight_hi_limbs_hold_the_fp32_bar(bwd_case):
    shipped_r4 = _bwd_err(bwd_case, "f16x2", "f16x2", "f16x2", "f16")
    shipped_r6 = _bwd_err(bwd_case, "f16x2", "f16", "f16x2", "f16")     # k_gru_bwd: Wc^T / Wg^T hi limbs
    r5 = _bwd_err(bwd_case, "f16x2", "f16", "f16", "f16")               # + k_prop_bwd's W_c^T hi limb (round 5)
    assert shipped_r4 <= 2.5e-4, shipped_r4
    assert shipped_r4 < shipped_r6 < r5, (shipped_r4, shipped_r6, r5)
    assert shipped_r6 <= 8e-4, shipped_r6


@pytest.mark.parametrize("seed,T", [(31, 5), (31, 8), (5, 5)])
def test_backward_policy_margin_over_seeds_and_unrolls(seed, T):
    """the round-5 backward (hi weight limbs in k_gru_bwd AND
    k_prop_bwd) was pinned at one seed and T = 5.  Over other inputs and the
    longer unroll it reaches the 1e-3 bar (seed 31: 1.07e-3 at T = 5, 1.10e-3 at
    T = 8; seed 5: 9.9e-4), so round 6 gives k_prop_bwd its W_c^T lo limb back:
    hi limbs in k_gru_bwd only, <= 7.6e-4 on every case measured (b = 8,
    T = 5..8, eight seeds)."""
    A, h0 = O.synthetic_batch(8, V, H, C, seed=seed)
    w = {k: x.astype(np.float64) for k, x in O.synthetic_weights(H, C, seed=seed).items()}
    A, h0 = A.astype(np.float64), h0.astype(np.float64)
    _, caches = O.forward(A, h0, w, T)
    dhT = np.random.default_rng(15 if seed == 31 else seed + 100).standard_normal(h0.shape)
    ref = O.backward(A, dhT, caches, w)
    case = (A, dhT, caches, w, ref)
    assert _bwd_err(case, "f16x2", "f16", "f16x2", "f16") <= 8e-4

@pytest.mark.parametrize("seed,T", [(31, 5), (5, 8)])
def test_backward_fp8_corrections_hold_the_bar(seed, T):
    """The shipped split-mode backward since round 6: k_gru_bwd's dz W^T as
    f16(dz) f16(W) + e5m2(dz) e4m3(W_lo) (gru_wt "f8lo") and k_prop_bwd's
    dM W_c^T with both limb corrections on the fp8 MFMA (prop_wt "f8corr").
    Seed 5 at T = 8 is where round 5's hi-only k_gru_bwd weights reach the bar
    (1.01e-3 at b = 8); the fp8 form brings W's lo limb back and stays below
    6e-4."""
    A, h0 = O.synthetic_batch(8, V, H, C, seed=seed)
    w = {k: x.astype(np.float64) for k, x in O.synthetic_weights(H, C, seed=seed).items()}
    A, h0 = A.astype(np.float64), h0.astype(np.float64)
    _, caches = O.forward(A, h0, w, T)
    dhT = np.random.default_rng(15 if seed == 31 else seed + 100).standard_normal(h0.shape)
    ref = O.backward(A, dhT, caches, w)
    case = (A, dhT, caches, w, ref)
    r6 = _bwd_err(case, "f16x2", "f8lo", "f8corr", "f16")
    assert r6 <= 6e-4, r6
    # the two fp8 pieces separately: prop's corrections cost nothing measurable,
    # gru's single-limb dz with W's lo limb beats round 5's dz hi/lo x W hi
    r5g = _bwd_err(case, "f16x2", "f16", "f16x2", "f16")
    assert _bwd_err(case, "f16x2", "f16", "f8corr", "f16") <= 1.1 * r5g + 2e-5
    assert r6 < r5g, (r6, r5g)


def test_f8corr_product_error_is_between_split_and_single_limb():
    """oracle.f8corr_product (k_prop_bwd's dh += dM W_c^T since round 6): the
    fp8 correction terms leave an error ~2^-15 of the product, far below a single
    f16 limb's (~2^-12) and above the 3-product split's (~2^-22)."""
    rng = np.random.default_rng(3)
    a = rng.standard_normal((64, 256)) * 2.0
    b = rng.uniform(-0.1, 0.1, (256, 96))
    ref = a @ b
    scale = np.abs(ref).max()
    e_f8 = np.abs(O.f8corr_product(a, b) - ref).max() / scale
    e_single = np.abs(O.round_f16(a) @ O.round_f16(b) - ref).max() / scale
    e_split = np.abs(O.OPERAND_ROUNDING["f16x2"](a) @ O.OPERAND_ROUNDING["f16x2"](b) - ref).max() / scale
    assert e_split < 1e-6 < e_f8 < 3e-5 < e_single, (e_split, e_f8, e_single)


def test_round_fp8_known_values():
    e4 = lambda x: O.round_fp8(x, 3, -6, 448.0)
    e5 = lambda x: O.round_fp8(x, 2, -14, 57344.0)
    assert np.array_equal(e4(np.array([1.0, 1.0625, 1.1875, 500.0, -3.3, 2.0 ** -9, 2.0 ** -11])),
                          [1.0, 1.0, 1.25, 448.0, -3.25, 2.0 ** -9, 0.0])
    assert np.array_equal(e5(np.array([1.0, 1.1, 1.4, 7e4, 2.0 ** -16])), [1.0, 1.0, 1.5, 57344.0, 2.0 ** -16])
