"""ctypes binding of libgrl.so (C ABI in include/grl.h).

This is the whole Python <-> native boundary: plain pointers, sizes and a
hipStream_t handle.  Tensors only appear in the callers (grl.graph,
grl.ops), which pass ``tensor.data_ptr()`` and the current torch stream.

There is deliberately no fallback: if libgrl.so is missing or a call fails,
GrlError is raised (the reference raises Python exceptions for bad inputs,
e.g. gnn/models/base_network.py:34-47; we keep that convention).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRL_LIB_PATH", os.path.join(_HERE, "libgrl.so"))


class GrlError(RuntimeError):
    """A libgrl call failed (negative GRL_E_* status)."""


GRL_OK = 0
GRL_E_INVALID = -1
GRL_E_UNSUPPORTED = -2
GRL_E_HIP = -3
GRL_E_WORKSPACE = -4
GRL_E_OVERFLOW = -5
GRL_E_TIMEOUT = -6

_c_i32 = ctypes.c_int32
_c_i64 = ctypes.c_int64
_c_u64 = ctypes.c_uint64
_c_vp = ctypes.c_void_p
_c_size = ctypes.c_size_t


class GrlSplitPlan(ctypes.Structure):
    _fields_ = [
        ("threshold", _c_i32),
        ("chunk_edges", _c_i32),
        ("num_heavy", _c_i64),
        ("num_chunks", _c_i64),
        ("heavy_seg", _c_vp),
        ("heavy_cptr", _c_vp),
        ("chunk_begin", _c_vp),
        ("chunk_end", _c_vp),
        ("partials", _c_vp),
        ("partials_capacity", _c_i64),
    ]


class GrlTypedCsr(ctypes.Structure):
    _fields_ = [
        ("num_rows", _c_i64),
        ("num_types", _c_i32),
        ("has_self", _c_i32),
        ("rowptr", _c_vp),
        ("colidx", _c_vp),
        ("vals", _c_vp),
        ("nnz", _c_i64),
        ("edge_id_base", _c_u64),
        ("self_id_base", _c_u64),
        ("split", ctypes.POINTER(GrlSplitPlan)),
        ("self_row0", _c_i64),
        ("path_rows", _c_i64),
    ]


class GrlTypedCsc(ctypes.Structure):
    _fields_ = [
        ("num_rows", _c_i64),
        ("self_rows", _c_i64),
        ("num_types", _c_i32),
        ("has_self", _c_i32),
        ("colptr", _c_vp),
        ("zrow", _c_vp),
        ("eid", _c_vp),
        ("vals", _c_vp),
        ("nnz", _c_i64),
        ("edge_id_base", _c_u64),
        ("self_id_base", _c_u64),
        ("split", ctypes.POINTER(GrlSplitPlan)),
    ]


class GrlDropEdge(ctypes.Structure):
    _fields_ = [
        ("key", _c_u64),
        ("threshold", ctypes.c_uint32),
        ("scale", ctypes.c_float),
        ("active", _c_i32),
        ("drop_self", _c_i32),
        ("seed_dev", _c_vp),
        ("call_id", _c_u64),
    ]


class GrlSynthSpec(ctypes.Structure):
    _fields_ = [
        ("kind", _c_i32),
        ("num_types", _c_i32),
        ("num_nodes", _c_i64),
        ("num_candidates", _c_i64),
        ("seed", _c_u64),
        ("row_begin", _c_i64),
        ("row_end", _c_i64),
    ]


class GrlLayoutItem(ctypes.Structure):
    _fields_ = [
        ("x1", ctypes.c_double),
        ("y1", ctypes.c_double),
        ("x2", ctypes.c_double),
        ("y2", ctypes.c_double),
        ("kind", _c_i32),
        ("has_text", _c_i32),
    ]


_P = ctypes.POINTER
# name -> (restype, argtypes); mirrors include/grl.h one for one.
SIGNATURES = {
    "grl_version": (ctypes.c_char_p, []),
    "grl_last_error": (ctypes.c_char_p, []),
    "grl_check": (_c_i32, [_c_vp]),
    "grl_set_option": (_c_i32, [ctypes.c_char_p, _c_i64]),
    "grl_get_option": (_c_i32, [ctypes.c_char_p, _P(_c_i64)]),
    "grl_trace_push": (None, [ctypes.c_char_p]),
    "grl_trace_pop": (None, []),
    "grl_dropedge_init": (_c_i32, [_P(GrlDropEdge), ctypes.c_float, _c_u64, _c_u64, _c_i32]),
    "grl_dropedge_init_device": (_c_i32, [_P(GrlDropEdge), ctypes.c_float, _c_vp, _c_u64, _c_i32]),
    "grl_dropedge_mask": (_c_i32, [_P(GrlDropEdge), _c_u64, _c_i64, _c_vp, _c_vp]),
    "grl_feature_dropout": (_c_i32, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i32, _c_i64, _P(GrlDropEdge), _c_vp]),
    "grl_typed_spmm_fwd": (_c_i32, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_vp, _P(GrlDropEdge), _c_vp]),
    "grl_typed_spmm_fwd_slice": (_c_i32, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_i64, _c_vp, _c_i64, _c_i32,
                                          _P(GrlDropEdge), _c_vp]),
    "grl_typed_spmm_bwd": (_c_i32, [_P(GrlTypedCsc), _c_vp, _c_i32, _c_vp, _c_i64, _P(GrlDropEdge), _c_vp]),
    "grl_typed_spmm_bwd_accum": (_c_i32, [_P(GrlTypedCsc), _c_vp, _c_i32, _c_vp, _c_i64, _P(GrlDropEdge), _c_vp]),
    "grl_typed_spmm_bwd_slice": (_c_i32, [_P(GrlTypedCsc), _c_vp, _c_i32, _c_i32, _c_i32, _c_vp, _c_i64,
                                          _P(GrlDropEdge), _c_vp]),
    "grl_graphconv_fwd_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32, _c_i32, _c_i32]),
    "grl_graphconv_fwd_workspace_query": (_c_size, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_vp, _c_i32]),
    "grl_graphconv_fwd_train": (_c_i32, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_vp, _c_vp, _c_i32, _c_i32, _c_vp,
                                         _c_vp, _P(GrlDropEdge), _c_vp, _c_size, _c_vp]),
    "grl_graphconv_bwd_data_workspace_query": (_c_size, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_vp, _c_i32]),
    "grl_graphconv_bwd_data": (_c_i32, [_P(GrlTypedCsr), _c_vp, _c_vp, _c_i64, _c_i64, _c_i32, _c_vp, _c_i32,
                                        _c_vp, _c_vp, _P(GrlDropEdge), _c_vp, _c_size, _c_vp]),
    "grl_graphconv_fwd": (_c_i32, [_P(GrlTypedCsr), _c_vp, _c_i64, _c_i32, _c_vp, _c_vp, _c_i32, _c_i32, _c_vp,
                                   _P(GrlDropEdge), _c_vp, _c_size, _c_vp]),
    "grl_linear_fwd_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "grl_linear_fwd": (_c_i32, [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_vp, _c_size,
                                _c_vp]),
    "grl_linear_fwd_ex_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32, _c_i64]),
    "grl_linear_fwd_ex": (_c_i32, [_c_vp, _c_i64, _c_vp, _c_i32, _c_vp, _c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_i64,
                                   _c_vp, _c_size, _c_vp]),
    "grl_linear_bwd_data_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "grl_linear_bwd_data": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64, _c_i32, _c_i32, _c_vp, _c_size,
                                     _c_vp]),
    "grl_relu_grad_workspace_size": (_c_size, [_c_i64, _c_i32]),
    "grl_relu_grad": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i32, _c_vp, _c_size, _c_vp]),
    "grl_linear_bwd_weight_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "grl_linear_bwd_weight": (_c_i32, [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i32, _c_i32, _c_vp,
                                       _c_size, _c_vp]),
    "grl_dense_to_csr_workspace_size": (_c_size, [_c_i64]),
    "grl_dense_to_csr_rowptr": (_c_i32, [_c_vp, _c_i64, _c_i64, _c_i32, _P(_c_i64), _c_vp, _c_vp, _c_size, _c_vp]),
    "grl_dense_to_csr_fill": (_c_i32, [_c_vp, _c_i64, _c_i64, _c_i32, _P(_c_i64), _c_vp, _c_vp, _c_vp, _c_vp]),
    "grl_csr_to_csc_workspace_size": (_c_size, [_c_i64, _c_i64]),
    "grl_csr_to_csc": (_c_i32, [_P(GrlTypedCsr), _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_size, _c_vp]),
    "grl_split_plan_workspace_size": (_c_size, [_c_i64]),
    "grl_split_plan_count": (_c_i32, [_c_vp, _c_i64, _c_i32, _c_i32, _c_i32, _c_vp, _c_vp, _c_size, _c_vp]),
    "grl_split_plan_build": (_c_i32, [_c_vp, _c_i64, _c_i32, _P(GrlSplitPlan), _c_vp, _c_size, _c_vp]),
    "grl_bag_linear_fwd": (_c_i32, [_c_vp, _c_i64, _c_i64, _c_i32, _c_vp, _c_i32, _c_vp, _c_i32, _c_vp, _c_vp]),
    "grl_bag_linear_bwd_weight_workspace_size": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "grl_bag_linear_bwd_weight": (_c_i32, [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i32, _c_i32, _c_vp,
                                           _c_size, _c_vp]),
    "grl_node_attention_workspace_size": (_c_size, [_c_i64, _c_i64, _c_i32, _c_i32]),
    "grl_node_attention_bwd_workspace_size": (_c_size, [_c_i64, _c_i64, _c_i32, _c_i32]),
    "grl_node_attention_fwd": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_i64,
                                        _c_i32, _c_i32, _c_vp, _c_size, _c_vp]),
    "grl_node_attention_bwd": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64,
                                        _c_i64, _c_i32, _c_i32, _c_vp, _c_size, _c_vp]),
    "grl_node_attention_fwd_rows": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64,
                                             _c_i64, _c_i32, _c_i32, _c_i64, _c_i64, _c_vp, _c_size, _c_vp]),
    "grl_node_attention_bwd_rows": (_c_i32, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                             _c_i64, _c_i64, _c_i32, _c_i32, _c_i64, _c_i64, _c_vp, _c_size, _c_vp]),
    "grl_layout_graph_size": (_c_i32, [_c_vp, _c_i32, _c_vp]),
    "grl_layout_graph_dense": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_i32, _c_vp]),
    "grl_layout_graph_edges": (_c_i32, [_c_vp, _c_i32, _c_i32, _c_vp, _c_i64, _c_vp]),
    "grl_synth_count": (_c_i32, [_P(GrlSynthSpec), _c_vp, _c_vp]),
    "grl_synth_workspace_size": (_c_size, [_P(GrlSynthSpec), _c_i64]),
    "grl_synth_degrees": (_c_i32, [_P(GrlSynthSpec), _c_vp, _c_vp]),
    "grl_synth_build": (_c_i32, [_P(GrlSynthSpec), _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_size, _c_vp]),
}

_lock = threading.Lock()
_lib = None


def lib() -> ctypes.CDLL:
    """Load libgrl.so once; raise GrlError (never fall back) if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise GrlError(
                    f"libgrl.so not found at {LIB_PATH}; build it with "
                    "`make -C graph-representation-learning_amd/csrc` or __graft_entry__.build()")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != GRL_OK:
        msg = lib().grl_last_error()
        raise GrlError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def set_option(name: str, value: int) -> None:
    """grl_set_option: one of the library's path options (test / A-B hooks
    that pick among kernel forms; include/grl.h)."""
    call("grl_set_option", name.encode(), int(value))


def get_option(name: str) -> int:
    v = _c_i64(0)
    call("grl_get_option", name.encode(), ctypes.byref(v))
    return int(v.value)


@contextlib.contextmanager
def options(**kw):
    """Set path options for the duration of a block, then restore them:
    `with grl.options(gemm_x6=0): ...`."""
    saved = {k: get_option(k) for k in kw}
    try:
        for k, v in kw.items():
            set_option(k, v)
        yield
    finally:
        for k, v in saved.items():
            set_option(k, v)


@contextlib.contextmanager
def trace(name: str):
    """roctx range (grl_trace_push / grl_trace_pop) around host-side steps,
    e.g. the halo exchange; shown by `rocprofv3 --marker-trace`."""
    lib().grl_trace_push(name.encode())
    try:
        yield
    finally:
        lib().grl_trace_pop()


def version() -> str:
    return lib().grl_version().decode()
