"""The C-ABI library builds, loads and exports every symbol include/ggnn.h
declares; host-only entry points (no GPU) validate dims.  No compute call."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "ggnn.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(ggnn_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ("ggnn_forward", "ggnn_backward", "ggnn_set_adjacency", "ggnn_pack_weights",
              "ggnn_workspace_bytes", "ggnn_last_error"):
        assert s in syms


def test_every_declared_symbol_is_exported(lib):
    from ggnn_amd import _lib
    syms = declared_symbols()
    assert set(syms) == set(_lib.EXPORTED)
    for s in syms:
        assert hasattr(lib, s), s


def test_dims_validation_and_sizes(lib):
    from ggnn_amd import _lib
    d = _lib.dims(256, 128, 256, 8, 5)
    _lib.check_dims(d)
    ws_t = _lib.workspace_bytes(d, True)
    ws_i = _lib.workspace_bytes(d, False)
    assert ws_t > ws_i > 0
    assert _lib.adjacency_bytes(d) >= 2 * 256 * 8 * 128 * 128 * 2
    assert _lib.weight_pack_bytes(d) >= 2 * 8 * 256 * 256 * 2
    for bad, code in ((_lib.dims(1, 1, 5000, 8, 5), -2), (_lib.dims(1, 129, 256, 5000, 5), -2),
                      (_lib.dims(0, 10, 256, 8, 5), -1), (_lib.dims(1, 10, 256, 8, 0), -1)):
        rc = lib.ggnn_check_dims(__import__("ctypes").byref(bad))
        assert rc == code
        assert lib.ggnn_last_error().decode()
    with pytest.raises(_lib.GGNNError):
        _lib.check_dims(_lib.dims(1, 1, 5000, 8, 5))
    # every other hidden size / vertex count is served by the general path
    for ok in (_lib.dims(1, 1, 100, 8, 5), _lib.dims(2, 198, 400, 92, 5), _lib.dims(1, 129, 256, 8, 5)):
        _lib.check_dims(ok)
        assert _lib.workspace_bytes(ok, True) > _lib.workspace_bytes(ok, False) > 0


def test_null_pointers_are_rejected_without_gpu(lib):
    import ctypes
    from ggnn_amd import _lib
    d = _lib.dims(2, 16, 128, 4, 2)
    rc = lib.ggnn_forward(ctypes.byref(d), None, None, None, 0, None, None, None)
    assert rc == -1 and b"NULL" in lib.ggnn_last_error()


def test_dropout_dims_validation_and_sizes(lib):
    """Keep probabilities must lie in (0, 1]; edge dropout holds one masked
    weight copy per timestep in the pack, and its dW problem's timestep-aligned
    K chunks (round 6) take their own split-K partial tiles."""
    import ctypes
    from ggnn_amd import _lib
    for ek, sk in ((0.0, 1.0), (1.0, 0.0), (1.5, 1.0), (1.0, -0.1), (float("nan"), 1.0)):
        d = _lib.dims(2, 16, 128, 4, 3, edge_keep=ek, state_keep=sk)
        assert lib.ggnn_check_dims(ctypes.byref(d)) == -1
        assert b"keep" in lib.ggnn_last_error()
    d1 = _lib.dims(256, 128, 256, 8, 5)
    d2 = _lib.dims(256, 128, 256, 8, 5, edge_keep=0.9, state_keep=0.9, seed=3)
    d3 = _lib.dims(256, 128, 256, 8, 5, edge_keep=1.0, state_keep=0.9, seed=3)
    p1, p2 = _lib.weight_pack_bytes(d1), _lib.weight_pack_bytes(d2)
    # (T-1) extra masked copies of W and W^T (hi + lo limbs) and of the general path's fp32 W,
    # and the general path's keep bits of every timestep (round 5: [T][C][h][h/32] words)
    assert p2 - p1 == 4 * 2 * (2 * 8 * 256 * 256 * 2) + 4 * (8 * 256 * 256 * 4) + 5 * 8 * 256 * 8 * 4
    assert _lib.weight_pack_bytes(d3) == p1                   # state dropout needs no extra pack
    # the dW problem's K chunks under edge dropout: 4 per timestep (T = 5: 20)
    # instead of 16 spanning every timestep -- 4 more 256 x 256 partial tiles
    # per channel for k_wgrad_reduce's deterministic reduction (no per-timestep
    # dW scratch since round 6: the reduce applies each timestep's mask itself)
    # (the forward's state keep bits, round 6, are laid out with or without
    # state dropout: a workspace sized for keep 1 serves keep < 1 too)
    assert (_lib.workspace_bytes(d2, True) - _lib.workspace_bytes(d1, True)
            == 8 * (5 * 4 - 16) * 256 * 256 * 4)
    assert _lib.workspace_bytes(d3, True) == _lib.workspace_bytes(d1, True)
    assert _lib.workspace_bytes(d2, False) == _lib.workspace_bytes(d1, False)
