"""Deterministic inputs shared by tests/golden/make_golden.py (which feeds
them to the reference) and the parity tests (which feed them to the engine
and the oracle).  numpy PCG64 streams only, so the bytes are identical on
every machine; large arrays are regenerated rather than committed."""
from __future__ import annotations

import numpy as np


def rng(seed: int) -> np.random.Generator:
    return np.random.default_rng(seed)


def random_adj_bnln(seed: int, B: int, N: int, L: int, edges_per_node: float = 3.0, float_vals: bool = False,
                    self_edges: bool = True) -> np.ndarray:
    """Collate-layout adjacency (B, N, L, N) like HeuristicGraphBuilder's
    output (gnn/data_generator/data_process/heuristic_graph_builder.py:56-83):
    binary (normal_binary) or weights in (0, 1] (fc_similarity-like)."""
    r = rng(seed)
    p = min(1.0, edges_per_node / (L * N))
    A = (r.random((B, N, L, N)) < p).astype(np.float32)
    if not self_edges:
        for n in range(N):
            A[:, n, :, n] = 0
    if float_vals:
        A = A * r.uniform(0.05, 1.0, size=A.shape).astype(np.float32)
    return A


def features(seed: int, *shape) -> np.ndarray:
    return rng(seed).standard_normal(shape).astype(np.float32)


def graphconv_params(seed: int, F: int, C: int, L: int):
    """(h_weights ((L+1)F, C), bias (C,)) with the reference's init scales
    (xavier_normal_, normal(1e-4, 5e-5): robust_gcn.py:29-30) but drawn from
    numpy so fixtures need not store them."""
    r = rng(seed)
    K = (L + 1) * F
    std = np.sqrt(2.0 / (K + C))
    W = (r.standard_normal((K, C)) * std).astype(np.float32)
    b = (1e-4 + 5e-5 * r.standard_normal(C)).astype(np.float32)
    return W, b


def probes(seed: int, n: int, k: int = 4) -> np.ndarray:
    """k random probe vectors of length n (used to compress large grads)."""
    return rng(seed).standard_normal((n, k)).astype(np.float32)


# Shapes of the GraphConv fixtures (SURVEY.md §8(c) golden list).
GRAPHCONV_CASES = {
    # name: (seed, B, N, L, F, C, float_vals, edges_per_node)
    "small": (11, 2, 7, 6, 16, 8, False, 3.0),
    "fc_odd": (12, 1, 9, 6, 10, 5, True, 6.0),
    "mid": (13, 2, 128, 6, 512, 256, False, 3.0),
}
DROPEDGE = {"p": 0.3, "seed": 20240601, "call": 5}


def synthetic_document(seed: int, n: int, cells: int = 0, tables: int = 0, float_coords: bool = False,
                       empty_text: float = 0.0):
    """A seeded OCR-like page: text lines in loose rows/columns with jitter,
    occasional overlaps, optional empty texts, "cell" and "table" items.
    Returns a list of region dicts in the reference's cassia layout
    ({"location": 4 points, "text", "label"})."""
    r = rng(seed)
    regions = []
    y = 10.0
    while len(regions) < n:
        x = float(r.integers(0, 60))
        h = float(r.integers(12, 40))
        for _ in range(int(r.integers(1, 6))):
            if len(regions) >= n:
                break
            w = float(r.integers(15, 300))
            jy = float(r.integers(-6, 7))
            x1, y1 = x, y + jy
            x2, y2 = x1 + w, y1 + h + float(r.integers(-3, 4))
            if float_coords:
                x1, y1, x2, y2 = (v + float(r.random()) for v in (x1, y1, x2, y2))
            else:
                x1, y1, x2, y2 = (float(int(v)) for v in (x1, y1, x2, y2))
            text = "" if r.random() < empty_text else "t%d" % len(regions)
            regions.append({"location": [[x1, y1], [x2, y1], [x2, y2], [x1, y2]], "text": text, "label": "other"})
            x = x2 + float(r.integers(-20, 80))  # may overlap the previous box
        y += h + float(r.integers(-8, 30))
    kinds = ["cell"] * cells + ["table"] * tables
    for i, kind in zip(r.choice(n, size=len(kinds), replace=False), kinds):
        regions[int(i)]["label"] = kind
    return regions


LAYOUT_CASES = {
    # name: (seed, n, cells, tables, float_coords, empty_text)
    "plain30": (41, 30, 0, 0, False, 0.0),
    "plain120": (42, 120, 0, 0, False, 0.0),
    "float80": (43, 80, 0, 0, True, 0.1),
    "cells60": (44, 60, 18, 0, False, 0.0),
    "tables40": (45, 40, 6, 3, False, 0.05),
    "tiny2": (46, 2, 0, 0, False, 0.0),
}
