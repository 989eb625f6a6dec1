"""Document layout -> typed graph, on the native builder in libgrl.

Host-side (no GPU needed).  Mirrors how the reference's HeuristicGraphBuilder
turns a sample's text lines into Graph(...).adj
(gnn/data_generator/data_process/heuristic_graph_builder.py:23-83,
utils/graph_utils.py:425-834), but in C++ and with a typed-edge-list output
that feeds grl.TypedGraph directly.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Mapping, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import GrlLayoutItem, call

EDGE_TYPES = {"normal_binary": 0, "fc_similarity": 1, "fc_binary": 2}
EDGE_LABELS = ("lr", "rl", "tb", "bt", "child", "parent")  # graph_utils.py:434


def _items(textlines: Sequence[Mapping]) -> Tuple[ctypes.Array, int]:
    """Text lines (dicts with "polygon" or "location", "text", optional
    "label") -> GrlLayoutItem array, boxes as the builder sees them
    (heuristic_graph_builder.py:35-46: min/max of the polygon)."""
    n = len(textlines)
    arr = (GrlLayoutItem * max(n, 1))()
    for i, item in enumerate(textlines):
        loc = np.asarray(item["polygon"] if "polygon" in item else item["location"], dtype=np.float64)
        it = arr[i]
        it.x1, it.x2 = float(loc[:, 0].min()), float(loc[:, 0].max())
        it.y1, it.y2 = float(loc[:, 1].min()), float(loc[:, 1].max())
        kind = item.get("label", "other")
        it.kind = 1 if kind == "cell" else (2 if kind == "table" else 0)
        it.has_text = int(str(item.get("text", "")) != "")
    return arr, n


def layout_size(textlines: Sequence[Mapping]) -> int:
    arr, n = _items(textlines)
    out = ctypes.c_int32()
    call("grl_layout_graph_size", arr, n, ctypes.byref(out))
    return out.value


def layout_adjacency(textlines: Sequence[Mapping], edge_type: str = "normal_binary") -> np.ndarray:
    """Dense (N, 6, N) float16 adjacency, byte-identical to the reference's
    HeuristicGraphBuilder output for the same text lines."""
    if edge_type not in EDGE_TYPES:
        raise _lib.GrlError(f"Invalid edge type: {edge_type}")
    arr, n = _items(textlines)
    size = ctypes.c_int32()
    call("grl_layout_graph_size", arr, n, ctypes.byref(size))
    m = size.value
    adj = np.zeros((m, 6, m), dtype=np.uint16)
    call("grl_layout_graph_dense", arr, n, EDGE_TYPES[edge_type], m, adj.ctypes.data_as(ctypes.c_void_p))
    return adj.view(np.float16)


def layout_edges(textlines: Sequence[Mapping]) -> Tuple[np.ndarray, int]:
    """normal_binary edges as sorted unique (src, type, dst) int32 rows, and
    the node count N of the graph they live in."""
    arr, n = _items(textlines)
    size = ctypes.c_int32()
    call("grl_layout_graph_size", arr, n, ctypes.byref(size))
    m = size.value
    count = ctypes.c_int64()
    call("grl_layout_graph_edges", arr, n, m, None, 0, ctypes.byref(count))
    edges = np.zeros((max(count.value, 1), 3), dtype=np.int32)
    call("grl_layout_graph_edges", arr, n, m, edges.ctypes.data_as(ctypes.c_void_p), count.value, ctypes.byref(count))
    return edges[: count.value], m


def edges_to_typed_csr(edges: np.ndarray, num_nodes: int, num_types: int = 6,
                       node_offsets: Iterable[int] = None) -> Tuple[np.ndarray, np.ndarray]:
    """(src, type, dst) triples (sorted) -> typed CSR (rowptr over (node,
    type) segments, colidx).  Rows keyed by the edge's start node, as the
    reference's adj[start, label, end] (graph_utils.py:829)."""
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 3)
    seg = e[:, 0] * num_types + e[:, 1]
    order = np.lexsort((e[:, 2], seg))
    seg, dst = seg[order], e[order, 2]
    rowptr = np.searchsorted(seg, np.arange(num_nodes * num_types + 1), side="left").astype(np.int32)
    return rowptr, dst.astype(np.int32)
