"""grl -- MI355X (gfx950) message-passing engine for GraphCNNDropEdge.

Host side of the C ABI in include/grl.h.  The reference-facing drop-in API
lives in the sibling `gnn` package (gnn.models.GraphCNNDropEdge,
gnn.models.networks.robust_gcn.GraphConv, gnn.cl_warper.GNNLearningWarper).
"""
from ._lib import GrlError, get_option, options, set_option, version  # noqa: F401
from .graph import DropEdge, EdgeBlockedGraph, TypedGraph, device_check  # noqa: F401
from .ops import graph_linear, typed_aggregate  # noqa: F401

check = device_check  # grl.check(): surface a persistent kernel's stream-ordered failure (grl_check)

__all__ = ["GrlError", "version", "options", "set_option", "get_option", "DropEdge", "EdgeBlockedGraph", "TypedGraph", "check", "device_check",
           "graph_linear", "typed_aggregate"]
