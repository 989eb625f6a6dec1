"""GPU, single process: the sharded path degenerates to the plain one at
world size 1 (no process group), through the same code the N-GPU bench runs."""
import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.dist import ShardedGraph, halo_exchange_into
from grl.ops import spmm_forward, typed_aggregate

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_world1_shard_equals_plain_graph():
    sg = ShardedGraph.synthetic(5000, 12.0, 6, seed=3, device=DEV)
    g = TypedGraph.synthetic(5000, 12.0, 6, seed=3, device=DEV)
    assert sg.halo_rows == 0 and torch.equal(sg.graph.colidx, g.colidx)
    X = torch.randn(5000, 64, device=DEV, requires_grad=True)
    de = DropEdge(0.3, 9, 1)
    Z1 = sg.aggregate(X, de)
    Z2 = typed_aggregate(X, g.with_dropedge(de))
    assert torch.equal(Z1, Z2)
    (dx1,) = torch.autograd.grad(Z1, X, torch.ones_like(Z1))
    (dx2,) = torch.autograd.grad(Z2, X, torch.ones_like(Z2))
    assert torch.equal(dx1, dx2)
    out = torch.empty_like(Z2)
    halo_exchange_into(X.detach(), X.detach(), torch.empty(0, 64, device=DEV), sg.plan)
    spmm_forward(X.detach(), sg.graph.with_dropedge(de), out=out)
    assert torch.equal(out, Z2)
