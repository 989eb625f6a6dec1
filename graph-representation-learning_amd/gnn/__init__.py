"""Drop-in for the reference's `gnn` package, restricted to the
GraphCNNDropEdge message-passing path.

    gnn.models.GraphCNNDropEdge        gnn/models/networks/drop_robust_gcn.py:31
    gnn.models.networks.robust_gcn     GraphConv, NodeSelfAtten, make_linear_relu
    gnn.models.BaseNetwork             gnn/models/base_network.py:9

All graph aggregation runs in libgrl (hand-written gfx950 HIP kernels);
there is no CPU path.
"""
