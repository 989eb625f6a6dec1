"""GPU: degree-ordered node relabeling (grl.graph.degree_order), the
one-time preprocessing the C5 bench applies to R-MAT graphs: the relabelled
graph is the same operator up to a permutation.
  * without DropEdge, Z' = Z[perm] bitwise (every row keeps its edge order,
    heavy rows are chunked the same way);
  * with DropEdge, Z' equals the oracle on the relabelled CSR bitwise;
  * dX' = dX[perm] within fp32 tolerance (the CSC order changes);
  * sources are numbered by descending in-degree."""
import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.graph import degree_order
from grl.ops import spmm_backward, spmm_forward
from oracle import c_oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("kind,threshold", [("rmat", None), ("rmat", 128), ("er", None)])
def test_degree_order_is_a_permutation_of_the_operator(kind, threshold):
    N, F, L = 1 << 14, 48, 6
    g = TypedGraph.synthetic(N, 24.0, L, kind=kind, seed=5, device=DEV)
    if threshold is not None:
        g.split_threshold, g.split_chunk = threshold, 64
    g2, perm = degree_order(g)
    assert g2.nnz == g.nnz and g2.split_threshold == g.split_threshold
    indeg = torch.bincount(g2.colidx.long(), minlength=N)
    assert bool((indeg[:-1] >= indeg[1:]).all())
    X = torch.randn(N, F, device=DEV)
    Z = spmm_forward(X, g)
    Xp = X[perm].contiguous()
    Z2 = spmm_forward(Xp, g2)
    assert torch.equal(Z2, Z[perm])
    de = DropEdge(0.3, 4, 1)
    Zd = spmm_forward(Xp, g2.with_dropedge(de))
    ref = c_oracle.spmm_fwd(g2.rowptr.cpu().numpy(), g2.colidx.cpu().numpy(), Xp.cpu().numpy(), L, True,
                            d=c_oracle.drop(0.3, 4, 1, True), split=(g2.split_threshold, g2.split_chunk))
    assert torch.equal(Zd.cpu(), torch.from_numpy(ref))
    dZ = torch.randn_like(Z)
    dX = spmm_backward(dZ, g, F)
    dX2 = spmm_backward(dZ[perm].contiguous(), g2, F)
    torch.testing.assert_close(dX2, dX[perm], rtol=1e-4, atol=1e-4)
