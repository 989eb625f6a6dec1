"""Pad variable-size documents to one batch shape.

NumpyPadding is the reference's collate (data_collate/numpy_padding.py:8-103):
for every configured key, all arrays are padded to the shape with the largest
element count, half of the padding before and half after each axis
("symmetric"), with that key's fill value.

TypedEdgePadding is the engine's additive variant for graphs emitted as typed
edge lists (HeuristicGraphBuilder(emit="edges")): node-indexed arrays are
padded exactly like NumpyPadding, and each document's (src, type, dst) edges
are shifted by its padding offset and its batch slot (b * N_max) so the
batch becomes one block-diagonal edge list -- no (N, 6, N) matrix is built.
"""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np


class BaseCollate:
    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseCollate":
        return cls(**(config or {}))


def _symmetric(pad: np.ndarray):
    return tuple((int(s) // 2, int(s) - int(s) // 2) for s in pad)


class NumpyPadding(BaseCollate):
    def __init__(self, name_value_pairs: Dict[str, float], only_selected_items: bool = False):
        self.name_value_pairs = dict(name_value_pairs)
        self.only_selected_items = only_selected_items

    def _normalize_shape(self, inputs: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        for name, value in self.name_value_pairs.items():
            arrays = [x.get(name) for x in inputs if x.get(name) is not None]
            if not arrays or not all(isinstance(a, np.ndarray) for a in arrays):
                continue
            target = max((list(a.shape) for a in arrays), key=lambda s: int(np.prod(np.array(s))))
            for x in inputs:
                a = x.get(name)
                if isinstance(a, np.ndarray):
                    x[name] = np.pad(a, _symmetric(np.subtract(target, a.shape)), constant_values=value)
        return inputs

    def __call__(self, inputs: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        inputs = self._normalize_shape(inputs)
        if self.only_selected_items:
            inputs = [{k: v for k, v in x.items() if k in self.name_value_pairs} for x in inputs]
        return inputs


class TypedEdgePadding(NumpyPadding):
    """Returns ONE dict (already batched; put no default_collate after it):
    padded per-node arrays stacked, "typed_edges" (E, 3) int64 with global
    node ids b*N + offset_b + i, and "graph_shape" = (B, N)."""

    def __call__(self, inputs: List[Dict[str, Any]]) -> Dict[str, Any]:
        sizes = [int(x["num_nodes"]) for x in inputs]
        n_max = max(sizes) if sizes else 0
        edges = []
        for b, (x, n) in enumerate(zip(inputs, sizes)):
            e = np.asarray(x["typed_edges"], dtype=np.int64).reshape(-1, 3).copy()
            shift = b * n_max + (n_max - n) // 2  # NumpyPadding puts (n_max - n)//2 pad rows first
            e[:, 0] += shift
            e[:, 2] += shift
            edges.append(e)
        inputs = self._normalize_shape(inputs)
        out: Dict[str, Any] = {}
        for name in self.name_value_pairs:
            vals = [x[name] for x in inputs if x.get(name) is not None]
            if vals:
                out[name] = np.stack(vals)
        out["typed_edges"] = np.concatenate(edges) if edges else np.zeros((0, 3), np.int64)
        out["graph_shape"] = np.array([len(inputs), n_max], dtype=np.int64)
        if not self.only_selected_items:
            out["label"] = [x.get("label") for x in inputs]
        return out
