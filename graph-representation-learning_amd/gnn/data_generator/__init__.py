"""Document -> (V, A, labels) pipeline feeding the GraphCNNDropEdge hot path
(the reference's gnn/data_generator).  The graph construction runs in the
native builder (grl.layout); everything else is light host code."""
