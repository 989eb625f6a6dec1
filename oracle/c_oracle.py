"""TEST INFRASTRUCTURE ONLY.  ctypes wrapper of oracle/libgrl_oracle.so.

numpy in, numpy out.  Builds the library on first use if it is missing and
a compiler is present (make -C oracle).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GRL_ORACLE_LIB: another build of grl_oracle.c (the ASan build of tests/test_asan.py)
LIB_PATH = os.environ.get("GRL_ORACLE_LIB", os.path.join(_HERE, "libgrl_oracle.so"))


class ODrop(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint64), ("threshold", ctypes.c_uint32), ("scale", ctypes.c_float),
                ("active", ctypes.c_int32), ("drop_self", ctypes.c_int32)]


_lib = None
_i32, _i64, _u64, _vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_void_p


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_dropedge_key.restype = _u64
        L.oracle_dropedge_key.argtypes = [_u64, _u64]
        L.oracle_dropedge_bits.restype = ctypes.c_uint32
        L.oracle_dropedge_bits.argtypes = [_u64, _u64]
        L.oracle_dropedge_init.restype = None
        L.oracle_dropedge_init.argtypes = [ctypes.POINTER(ODrop), ctypes.c_float, _u64, _u64, _i32]
        L.oracle_dropedge_mask.restype = None
        L.oracle_dropedge_mask.argtypes = [ctypes.POINTER(ODrop), _u64, _i64, _vp]
        L.oracle_spmm_fwd.restype = None
        L.oracle_spmm_fwd.argtypes = [_i64, _i32, _i32, _vp, _vp, _vp, _u64, _u64, _vp, _vp, _i64, _i32, _vp,
                                      ctypes.POINTER(ODrop), _i32, _i32, _i32]
        L.oracle_spmm_bwd.restype = None
        L.oracle_spmm_bwd.argtypes = [_i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _u64, _u64, _vp, _i32, _vp, _i64,
                                      ctypes.POINTER(ODrop), _i32, _i32, _i32]
        L.oracle_dense_to_csr.restype = _i64
        L.oracle_dense_to_csr.argtypes = [_vp, _i64, _i64, _i32, _vp, _vp, _vp, _vp]
        L.oracle_csr_to_csc.restype = None
        L.oracle_csr_to_csc.argtypes = [_i64, _i32, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp]
        L.oracle_synth.restype = _i64
        L.oracle_synth.argtypes = [_i32, _i32, _i64, _i64, _u64, _i64, _i64, _vp, _vp, _i64]
        L.oracle_synth_count.restype = _i64
        L.oracle_synth_count.argtypes = [_i32, _i32, _i64, _i64, _u64, _i64, _i64]
        L.oracle_max_threads.restype = _i32
        L.oracle_max_threads.argtypes = []
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def drop(p: float = 0.0, seed: int = 0, call: int = 0, drop_self: bool = True) -> ODrop:
    d = ODrop()
    lib().oracle_dropedge_init(ctypes.byref(d), float(p), seed, call, int(drop_self))
    return d


def dropedge_mask(d: ODrop, id_base: int, count: int) -> np.ndarray:
    keep = np.zeros(count, dtype=np.uint8)
    lib().oracle_dropedge_mask(ctypes.byref(d), id_base, count, _p(keep))
    return keep


def spmm_fwd(rowptr, colidx, X, num_types, has_self=True, vals=None, d: ODrop | None = None, edge_base=0,
             self_base=None, nthreads=0, split=None, X_self=None):
    """split = (threshold, chunk_edges) reproduces the engine's chunked
    summation order for rows heavier than threshold (GrlSplitPlan).
    X_self: own-feature rows of the CSR rows when they are a sub-range of X."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int32)
    colidx = np.ascontiguousarray(colidx, dtype=np.int32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    vals = None if vals is None else np.ascontiguousarray(vals, dtype=np.float32)
    rows = (rowptr.size - 1) // num_types
    F = X.shape[1]
    hs = 1 if has_self else 0
    if self_base is None:
        self_base = int(rowptr[-1])
    Z = np.empty((rows, (num_types + hs) * F), dtype=np.float32)
    if X_self is not None:
        X_self = np.ascontiguousarray(X_self, dtype=np.float32)
        assert X_self.shape[0] >= rows and X_self.shape[1] == F
    lib().oracle_spmm_fwd(rows, num_types, hs, _p(rowptr), _p(colidx), _p(vals), edge_base, self_base, _p(X),
                          _p(X_self), F, F,
                          _p(Z), ctypes.byref(d) if d is not None else None, nthreads,
                          *(split if split is not None else (-1, 1)))
    return Z


def csr_to_csc(rowptr, colidx, num_types, ncols, has_self=True, vals=None):
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int32)
    colidx = np.ascontiguousarray(colidx, dtype=np.int32)
    rows = (rowptr.size - 1) // num_types
    nnz = int(rowptr[-1])
    colptr = np.zeros(ncols + 1, dtype=np.int32)
    zrow = np.zeros(nnz, dtype=np.int32)
    eid = np.zeros(nnz, dtype=np.int32)
    cvals = None if vals is None else np.zeros(nnz, dtype=np.float32)
    vals = None if vals is None else np.ascontiguousarray(vals, dtype=np.float32)
    lib().oracle_csr_to_csc(rows, num_types, 1 if has_self else 0, _p(rowptr), _p(colidx), _p(vals), ncols,
                            _p(colptr), _p(zrow), _p(eid), _p(cvals))
    return colptr, zrow, eid, cvals


def spmm_bwd(colptr, zrow, eid, dZ, num_types, F, self_rows, has_self=True, cvals=None, d: ODrop | None = None,
             edge_base=0, self_base=0, nthreads=0, split=None):
    colptr = np.ascontiguousarray(colptr, dtype=np.int32)
    rows = colptr.size - 1
    dZ = np.ascontiguousarray(dZ, dtype=np.float32)
    dX = np.empty((rows, F), dtype=np.float32)
    cvals = None if cvals is None else np.ascontiguousarray(cvals, dtype=np.float32)
    lib().oracle_spmm_bwd(rows, self_rows, num_types, 1 if has_self else 0, _p(colptr),
                          _p(np.ascontiguousarray(zrow, dtype=np.int32)), _p(np.ascontiguousarray(eid, dtype=np.int32)),
                          _p(cvals), edge_base, self_base, _p(dZ), F, _p(dX), F,
                          ctypes.byref(d) if d is not None else None, nthreads,
                          *(split if split is not None else (-1, 1)))
    return dX


def dense_to_csr(A: np.ndarray, strides_elems, B: int, N: int, L: int):
    A = np.asarray(A, dtype=np.float32)
    st = np.asarray(strides_elems, dtype=np.int64)
    rowptr = np.zeros(B * N * L + 1, dtype=np.int32)
    nnz = lib().oracle_dense_to_csr(_p(A), B, N, L, _p(st), _p(rowptr), None, None)
    colidx = np.zeros(max(nnz, 1), dtype=np.int32)
    vals = np.zeros(max(nnz, 1), dtype=np.float32)
    lib().oracle_dense_to_csr(_p(A), B, N, L, _p(st), _p(rowptr), _p(colidx), _p(vals))
    return rowptr, colidx[:nnz], vals[:nnz]


def synth(kind, L, N, C, seed, row_begin=0, row_end=None):
    row_end = N if row_end is None else row_end
    cnt = lib().oracle_synth_count(kind, L, N, C, seed, row_begin, row_end)
    rowptr = np.zeros((row_end - row_begin) * L + 1, dtype=np.int32)
    colidx = np.zeros(max(cnt, 1), dtype=np.int32)
    nnz = lib().oracle_synth(kind, L, N, C, seed, row_begin, row_end, _p(rowptr), _p(colidx), cnt)
    return rowptr, colidx[:nnz], cnt


def max_threads() -> int:
    return int(lib().oracle_max_threads())
