"""TEST INFRASTRUCTURE ONLY.  numpy restatement of the engine's counter hashes.

The reference draws DropEdge masks with torch's Bernoulli sampler
(nn.Dropout at gnn/models/networks/drop_robust_gcn.py:38, applied at
:76,:80,:85).  The engine replaces that draw with a regenerable hash so the
same mask can be rebuilt in backward, across shards and on the CPU; this
module restates that hash from its specification in include/grl.h
(GrlDropEdge, GrlSynthSpec).  Vectorised over ids with uint64 wraparound.
"""
from __future__ import annotations

import numpy as np

_U = np.uint64


def mix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> _U(30))
        x = x * _U(0xBF58476D1CE4E5B9)
        x = x ^ (x >> _U(27))
        x = x * _U(0x94D049BB133111EB)
        x = x ^ (x >> _U(31))
    return x


def dropedge_key(seed: int, call: int) -> int:
    with np.errstate(over="ignore"):
        a = mix64(np.array([seed], dtype=np.uint64) ^ _U(0x6A09E667F3BCC909))
        b = np.array([call], dtype=np.uint64) * _U(0x9E3779B97F4A7C15)
        return int(mix64(a + b)[0])


def dropedge_bits(key: int, ids: np.ndarray) -> np.ndarray:
    ids = np.asarray(ids, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return (mix64(_U(key) ^ (ids * _U(0xD1B54A32D192ED03))) >> _U(32)).astype(np.uint32)


def dropedge_params(p: float):
    """(active, threshold, scale) exactly as grl_dropedge_init computes them."""
    p32 = float(np.float32(p))
    if p32 <= 0.0:
        return False, 0, np.float32(1.0)
    if p32 >= 1.0:
        return True, 0xFFFFFFFF, np.float32(0.0)
    thr = np.floor(p32 * 4294967296.0)
    thr = 0xFFFFFFFF if thr >= 4294967295.0 else int(thr)
    return True, thr, np.float32(1.0 / (1.0 - p32))


def dropedge_keep(p: float, seed: int, call: int, ids: np.ndarray) -> np.ndarray:
    """bool mask: entry with global id survives DropEdge(p, seed, call)."""
    active, thr, scale = dropedge_params(p)
    ids = np.asarray(ids, dtype=np.uint64)
    if not active:
        return np.ones(ids.shape, dtype=bool)
    if scale == 0.0:
        return np.zeros(ids.shape, dtype=bool)
    return dropedge_bits(dropedge_key(seed, call), ids) >= np.uint32(thr)


def synth_bits(seed: int, k: np.ndarray, lane: int) -> np.ndarray:
    k = np.asarray(k, dtype=np.uint64)
    with np.errstate(over="ignore"):
        s = mix64(np.array([seed], dtype=np.uint64) + _U(0x243F6A8885A308D3) * _U(lane + 1))
        return mix64(s ^ (k * _U(0x9E3779B97F4A7C15)))


_RMAT = (2448131358, 3264175144, 4080218931)  # floor((.57, .76, .95) * 2^32)


def synth_edges(kind: int, L: int, N: int, C: int, seed: int):
    """(src, type, dst) int64 arrays of the C candidate edges (no dedupe)."""
    k = np.arange(C, dtype=np.uint64)
    lo = _U(0xFFFFFFFF)
    h1 = synth_bits(seed, k, 1)
    typ = ((h1 & lo) * _U(L)) >> _U(32)
    if kind == 0:
        h0 = synth_bits(seed, k, 0)
        src = ((h0 & lo) * _U(N)) >> _U(32)
        dst = ((h0 >> _U(32)) * _U(N)) >> _U(32)
    else:
        scale = int(N).bit_length() - 1
        assert 1 << scale == N
        src = np.zeros(C, dtype=np.uint64)
        dst = np.zeros(C, dtype=np.uint64)
        for lvl in range(scale):
            h = synth_bits(seed, k, 2 + (lvl >> 1))
            r = (h >> _U(32)) if (lvl & 1) else (h & lo)
            q = np.where(r < _U(_RMAT[0]), 0, np.where(r < _U(_RMAT[1]), 1, np.where(r < _U(_RMAT[2]), 2, 3)))
            q = q.astype(np.uint64)
            src = (src << _U(1)) | (q >> _U(1))
            dst = (dst << _U(1)) | (q & _U(1))
    return src.astype(np.int64), typ.astype(np.int64), dst.astype(np.int64)


def synth_csr(kind: int, L: int, N: int, C: int, seed: int, row_begin: int = 0, row_end: int | None = None):
    """Deduped typed CSR (rowptr, colidx) of node range [row_begin, row_end)."""
    row_end = N if row_end is None else row_end
    src, typ, dst = synth_edges(kind, L, N, C, seed)
    sel = (src >= row_begin) & (src < row_end)
    keys = ((src[sel] - row_begin).astype(np.uint64) * _U(L) + typ[sel].astype(np.uint64)) * _U(N) + dst[sel].astype(
        np.uint64)
    keys = np.unique(keys)
    seg = (keys // _U(N)).astype(np.int64)
    colidx = (keys % _U(N)).astype(np.int32)
    nseg = (row_end - row_begin) * L
    rowptr = np.searchsorted(seg, np.arange(nseg + 1), side="left").astype(np.int32)
    return rowptr, colidx
