"""Model registry: BaseNetwork._from_config({"type": ..., "args": ...})
resolves `type` with getattr on this module (gnn/models/base_network.py:33)."""
from gnn.models.base_network import BaseNetwork  # noqa: F401
from gnn.models.networks.drop_robust_gcn import GraphCNNDropEdge  # noqa: F401
from gnn.models.networks.robust_gcn import GraphConv, NodeSelfAtten  # noqa: F401

__all__ = ["BaseNetwork", "GraphCNNDropEdge", "GraphConv", "NodeSelfAtten"]
