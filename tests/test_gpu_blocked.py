"""GPU: graphs with 2^31 or more typed edges (SURVEY.md §8(b) Dtypes row,
"int64 rowptr when E >= 2^31").  grl.EdgeBlockedGraph holds them as row
blocks of < 2^31 edges with 64-bit global edge ids; the forward aggregates
block by block, the backward runs the blocks' CSCs in order (the later ones
through grl_typed_spmm_bwd_accum).

  * small graphs cut into many blocks equal the one-CSR graph BITWISE:
    Z, dX (DropEdge on), a whole GraphConv's output and gradients, and the
    int64-rowptr constructor (from_csr64);
  * a real 2.2-billion-edge graph (2^22 nodes, avg_deg 520, d=16) runs forward
    and backward: sampled rows bitwise vs the oracle, sampled columns of dX
    vs a float64 sum over the column's in-edges."""
import numpy as np
import pytest
import torch

from grl import DropEdge, EdgeBlockedGraph, TypedGraph
from grl.ops import graph_conv, spmm_backward, spmm_forward
from oracle import c_oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
L = 6


def _graphs(kind, block, threshold=None):
    N = 1 << 14
    g = TypedGraph.synthetic(N, 24.0, L, kind=kind, seed=3, device=DEV)
    gb = EdgeBlockedGraph.synthetic(N, 24.0, L, kind=kind, seed=3, device=DEV, max_block_edges=block)
    g64 = EdgeBlockedGraph.from_csr64(g.rowptr.to(torch.int64), g.colidx, L, max_block_edges=block)
    if threshold is not None:  # R-MAT hub rows / columns as chunk items
        for graph in (g, *gb.blocks, *g64.blocks):
            graph.split_threshold, graph.split_chunk = threshold, 32
    return g, gb, g64


@pytest.mark.parametrize("threshold", [None, 64])
@pytest.mark.parametrize("kind,block", [("er", 60_000), ("rmat", 90_000), ("er", 10**9)])
def test_blocks_equal_one_csr(kind, block, threshold):
    F = 40
    torch.manual_seed(kind == "er")
    g, gb, g64 = _graphs(kind, block, threshold)
    N = g.num_rows
    assert gb.nnz == g.nnz == g64.nnz and (len(gb.blocks) > 1) == (block < g.nnz)
    for graph in (gb, g64):  # blocks cover the rows in order; ids continue across them
        assert graph.row_bounds[0] == 0 and graph.row_bounds[-1] == N
        assert [b.edge_id_base for b in graph.blocks] == list(np.cumsum([0] + [b.nnz for b in graph.blocks])[:-1])
        assert all(b.nnz <= block for b in graph.blocks)
    de = DropEdge(0.3, 5, 2)
    X = torch.randn(N, F, device=DEV)
    Z = spmm_forward(X, g.with_dropedge(de))
    for graph in (gb, g64):
        assert torch.equal(spmm_forward(X, graph.with_dropedge(de)), Z)
    dZ = torch.randn_like(Z)
    dX = spmm_backward(dZ, g.with_dropedge(de), F)
    absum = spmm_backward(dZ.abs(), g.with_dropedge(de), F)  # sum of |terms| per element
    for graph in (gb, g64):
        dXb = spmm_backward(dZ, graph.with_dropedge(de), F)
        if kind == "er":
            assert torch.equal(dXb, dX)  # no heavy columns: the one-CSC chain exactly
        else:  # R-MAT hub columns are chunked per block: the same terms, chunk sums grouped
            # differently -- hubs sum thousands of terms with cancellation, so the bound is
            # relative to the sum of |terms| (fp32 reassociation), not to the result
            assert torch.all((dXb - dX).abs() <= 1e-5 * absum + 1e-6), float(((dXb - dX).abs() / absum).max())
    if threshold is not None:
        return
    # a whole GraphConv (autograd) on the blocked graph
    W = (torch.randn(7 * F, 24, device=DEV) / 20).requires_grad_(True)
    b = torch.randn(24, device=DEV).requires_grad_(True)
    res = []
    for graph in (g, gb):
        for t in (W, b):
            t.grad = None
        Xg = torch.randn(N, F, generator=torch.Generator(device=DEV).manual_seed(4), device=DEV).requires_grad_(True)
        out = graph_conv(Xg, graph.with_dropedge(DropEdge(0.3, 6, 0)), W, b, relu=True)
        out.square().sum().backward()
        res.append((out.detach(), Xg.grad, W.grad.clone(), b.grad.clone()))
    for i, (a, c) in enumerate(zip(*res)):
        if i == 1 and kind == "rmat":  # dX: hub columns chunked per block (as above)
            torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-4)
        else:  # out, dW, db: the same Z, so the same bits
            assert torch.equal(a, c)


def test_two_billion_edges():
    N, deg, F = 1 << 22, 520.0, 16
    gb = EdgeBlockedGraph.synthetic(N, deg, L, seed=1, device=DEV)
    E = gb.nnz
    print(f"  [{E} typed edges in {len(gb.blocks)} blocks]", flush=True)
    assert E >= 2**31 and len(gb.blocks) >= 2
    X = torch.randn(N, F, generator=torch.Generator(device=DEV).manual_seed(2), device=DEV)
    de = DropEdge(0.3, 7, 0)
    Z = spmm_forward(X, gb.with_dropedge(de))
    torch.cuda.synchronize()
    Xh = X.cpu().numpy()
    d = c_oracle.drop(0.3, 7, 0, True)
    rng = np.random.default_rng(0)
    # rows from every block, including each block's first and last rows
    for blk, r0, r1 in zip(gb.blocks, gb.row_bounds[:-1], gb.row_bounds[1:]):
        for a in (0, int(rng.integers(1, r1 - r0 - 64)), r1 - r0 - 64):
            rp = blk.rowptr[a * L: (a + 64) * L + 1].cpu().numpy()
            e0 = int(rp[0])
            ci = blk.colidx[e0: int(rp[-1])].cpu().numpy()
            Zc = c_oracle.spmm_fwd(rp - e0, ci, Xh, L, True, d=d, edge_base=blk.edge_id_base + e0,
                                   self_base=blk.self_id_base + a, X_self=Xh[r0 + a:])
            assert np.array_equal(Z[r0 + a: r0 + a + 64].cpu().numpy(), Zc), (r0, a)
    print("  [forward: sampled rows of every block bitwise vs oracle]", flush=True)
    # backward: dX columns vs a float64 sum over each column's in-edges (all blocks)
    dZ = torch.randn(N, 7 * F, generator=torch.Generator(device=DEV).manual_seed(3), device=DEV)
    dX = spmm_backward(dZ, gb.with_dropedge(de), F)
    torch.cuda.synchronize()
    cols = rng.choice(N, size=4, replace=False)
    scale = np.float32(1.0 / 0.7)
    for m in cols.tolist():
        acc = np.zeros(F, np.float64)
        keep_self = c_oracle.dropedge_mask(d, E + m, 1)[0]
        if keep_self:
            acc += float(scale) * dZ[m, :F].double().cpu().numpy()
        for blk, r0 in zip(gb.blocks, gb.row_bounds[:-1]):
            pos = (blk.colidx == m).nonzero().flatten()
            if pos.numel() == 0:
                continue
            seg = torch.searchsorted(blk.rowptr, pos.to(torch.int32), right=True) - 1  # (row, type) segment
            rows, types = seg // L, seg % L
            keep = torch.from_numpy(np.array([c_oracle.dropedge_mask(d, blk.edge_id_base + int(p), 1)[0]
                                              for p in pos.cpu().tolist()], dtype=bool)).to(DEV)
            zr = dZ.view(N, 7, F)[r0 + rows[keep], 1 + types[keep]].double()
            acc += float(scale) * zr.sum(0).cpu().numpy()
        got = dX[m].double().cpu().numpy()
        assert np.abs(got - acc).max() <= 1e-4 * max(1.0, np.abs(acc).max()), (m, got, acc)
    print("  [backward: sampled dX columns vs float64 in-edge sums]", flush=True)
