"""Heuristic spatial graph per document on the native builder (libgrl,
grl_layout_graph_*), the drop-in for the reference's HeuristicGraphBuilder
(data_process/heuristic_graph_builder.py:9-83 + utils/graph_utils.py).

emit = "dense" (default): sample["adjacency_matrix"] = (N, 6, N) float16,
       byte-identical to the reference (the collate / KVProcedure path).
emit = "edges": sample["typed_edges"] = sorted (src, type, dst) int32 rows
       and sample["num_nodes"]; no O(N^2) matrix -- feeds TypedGraph directly.
emit = "both": both keys.
"""
from __future__ import annotations

from typing import Any, Dict

from gnn.data_generator.data_process.base import BaseDataProcess
from grl.layout import EDGE_TYPES, layout_adjacency, layout_edges


class HeuristicGraphBuilder(BaseDataProcess):
    def __init__(self, num_edges: int, edge_type: str, emit: str = "dense"):
        if num_edges != 6:
            raise ValueError(f"the heuristic graph has 6 edge types (lr, rl, tb, bt, child, parent), got {num_edges}")
        if edge_type not in EDGE_TYPES:
            raise Exception("Invalid edge type: " + str(edge_type))
        if emit not in ("dense", "edges", "both"):
            raise ValueError(f"emit must be dense|edges|both, got {emit}")
        if emit != "dense" and edge_type != "normal_binary":
            raise ValueError("typed edge lists are emitted for normal_binary graphs only")
        self.num_edges = num_edges
        self.edge_type = edge_type
        self.emit = emit

    def process(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        if sample.get("label", None) is None:
            return sample
        lines = self.ordered_lines(sample)
        if self.emit in ("dense", "both"):
            sample["adjacency_matrix"] = layout_adjacency(lines, self.edge_type)
        if self.emit in ("edges", "both"):
            sample["typed_edges"], sample["num_nodes"] = layout_edges(lines)
        return sample
