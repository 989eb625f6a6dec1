"""CPU-only: libgrl.so loads, exports exactly what include/grl.h declares,
and its host-side entry points (argument validation, DropEdge setup) behave
as specified.  No device work is issued."""
import ctypes
import os
import re

import numpy as np
import pytest

from grl import _lib
from oracle import c_oracle

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "grl.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set(re.findall(r"\b(grl_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_the_hot_path():
    names = declared_functions()
    for required in ("grl_typed_spmm_fwd", "grl_typed_spmm_bwd", "grl_linear_fwd", "grl_dense_to_csr_rowptr",
                     "grl_csr_to_csc", "grl_dropedge_init", "grl_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    names = declared_functions()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"libgrl.so lacks {missing}"
    # and the binding describes every one of them
    assert sorted(_lib.SIGNATURES) == names


def test_version_and_error_channel():
    assert "gfx950" in _lib.version()
    lib = _lib.lib()
    rc = lib.grl_typed_spmm_fwd(None, None, 0, 0, None, None, None)
    assert rc == _lib.GRL_E_INVALID
    assert b"NULL" in lib.grl_last_error()
    with pytest.raises(_lib.GrlError, match="grl_typed_spmm_bwd"):
        _lib.call("grl_typed_spmm_bwd", None, None, 0, None, 0, None, None)


def test_shape_validation_is_host_side():
    g = _lib.GrlTypedCsr()
    g.num_rows, g.num_types = 10, 0
    rc = _lib.lib().grl_typed_spmm_fwd(ctypes.byref(g), None, 4, 4, None, None, None)
    assert rc == _lib.GRL_E_INVALID and b"num_types" in _lib.lib().grl_last_error()
    g.num_types = 6
    rc = _lib.lib().grl_typed_spmm_fwd(ctypes.byref(g), None, 2, 4, None, None, None)
    assert rc == _lib.GRL_E_INVALID and b"ldx" in _lib.lib().grl_last_error()


@pytest.mark.parametrize("p", [0.0, 1e-9, 0.2, 0.3, 0.5, 0.999, 1.0, 3.0])
def test_dropedge_init_matches_oracle(p):
    de = _lib.GrlDropEdge()
    _lib.call("grl_dropedge_init", ctypes.byref(de), p, 2024, 17, 1)
    od = c_oracle.drop(p, 2024, 17, True)
    assert (de.key, de.threshold, de.active, de.drop_self) == (od.key, od.threshold, od.active, od.drop_self)
    assert np.float32(de.scale) == np.float32(od.scale)


def test_dropedge_init_rejects_negative_p():
    de = _lib.GrlDropEdge()
    assert _lib.lib().grl_dropedge_init(ctypes.byref(de), -0.1, 0, 0, 1) == _lib.GRL_E_INVALID


def test_path_options_round_trip_and_reject_unknown_names():
    """grl_set_option / grl_get_option: the kernel-form hooks that replaced the
    per-call environment variables (nothing in libgrl reads the environment):
    defaults are the production paths, values round-trip, grl.options()
    restores them, unknown names and out-of-range values are GRL_E_INVALID."""
    import grl

    defaults = {"gemm_x6": 1, "graphconv_fused": 1, "graphconv_fused_bwd": 1, "fg_ws": 1, "spmm_wide": -1,
                "spmm_blocks_per_cu": 24, "attn_x6": 1, "attn_fwd8": 1, "attn_dh8": 1, "attn_fused_dq": 1,
                "attn_pipe": 1, "attn_dh16": 1, "attn_kq16": 1, "attn_qslab_max": 0, "ws_spin": 0, "ws_status_sync": 0}
    assert {k: grl.get_option(k) for k in defaults} == defaults
    with grl.options(gemm_x6=0, ws_spin=7, spmm_wide=1):
        assert (grl.get_option("gemm_x6"), grl.get_option("ws_spin"), grl.get_option("spmm_wide")) == (0, 7, 1)
    assert {k: grl.get_option(k) for k in defaults} == defaults
    with pytest.raises(grl.GrlError, match="unknown option"):
        grl.set_option("GRL_GEMM_X6", 0)
    with pytest.raises(grl.GrlError, match="outside"):
        grl.set_option("gemm_x6", 2)
    os.environ["GRL_GEMM_X6"] = "0"  # the round-5 variable: read by nothing now
    try:
        assert grl.get_option("gemm_x6") == 1
        from grl.ops import x6_rows_ok

        assert x6_rows_ok(1_000_000, 256, 1792)
    finally:
        del os.environ["GRL_GEMM_X6"]
