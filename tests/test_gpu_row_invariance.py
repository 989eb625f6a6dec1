"""GPU: row results independent of the row count (verdict r4 item 2,
robust_gcn.py:50-51, drop_robust_gcn.py:36-58, robust_gcn.py:78-96), and
the hash-keyed feature dropout (verdict r4 item 3, drop_robust_gcn.py:64,
77, 81, 86, 100).

A node-range shard computes its rows in calls with fewer rows than the
one-GPU model's; every row-local op must give those rows the same bits:
  * the fp32 GEMM sums K in fixed chunks added in chunk order (slabs) for
    calls of fewer than 256 output tiles and in one pass for larger ones:
    the rows of an M-row call equal the same rows of any other call made
    for M rows (path_rows), bitwise;
  * path_rows makes a smaller call take the bigger call's path (x6, fp32
    one pass or fp32 slabs);
  * NodeSelfAtten's key split depends on N only: a query range's rows equal
    the whole-range call's;
  * feature dropout's mask is the hash of (seed, call, global element id)."""
import numpy as np
import pytest
import torch

from grl import DropEdge
from grl.ops import feature_dropout, linear_fwd, linear_fwd_ex, node_attention_forward, row_linear

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("K,C", [(448, 64), (1792, 256), (512, 128), (128, 1280), (1280, 53), (100, 30)])
@pytest.mark.parametrize("M", [60000, 8000])
def test_fp32_gemm_rows_do_not_depend_on_m(K, C, M):
    """grl_linear_fwd_ex on the fp32 path (below the x6 size floor), the
    path chosen for M rows (path_rows = M): the rows of calls of 74 .. M rows
    are bitwise the same rows of the M-row call -- on the one-pass kernel
    (M's calls of >= 256 output tiles) and on the chunk slabs (fewer tiles);
    within 1e-5 of float64."""
    from grl.ops import x6_rows_ok

    g = torch.Generator(device=DEV).manual_seed(K + C)
    X = torch.randn(M, K, generator=g, device=DEV)
    W = torch.randn(K, C, generator=g, device=DEV) / K ** 0.5
    b = torch.randn(C, generator=g, device=DEV)
    if x6_rows_ok(M, C, K):
        M = 8192  # keep the reference call on the fp32 path too
        X = X[:M].contiguous()
        assert not x6_rows_ok(M, C, K)
    full = linear_fwd_ex(X, W, 0, b, True, path_rows=M)
    ref = torch.relu(X.double() @ W.double() + b.double())
    assert float((full.double() - ref).abs().max()) <= 1e-5 * max(1.0, float(ref.abs().max()))
    for r0, r1 in ((0, 74), (5, 301), (1000, 3500), (777, 8000), (0, M // 2), (M // 3, M)):
        r1 = min(r1, M)
        part = linear_fwd_ex(X[r0:r1].contiguous(), W, 0, b, True, path_rows=M)
        assert torch.equal(part, full[r0:r1]), (r0, r1, float((part - full[r0:r1]).abs().max()))


@pytest.mark.parametrize("M", [40_000, 3000])  # both widths below the x6 size: one pass, slabs
@pytest.mark.parametrize("K,C", [(1280, 56), (128, 160), (100, 30)])
def test_narrow_tiles_give_the_wide_tiles_bits(M, K, C):
    """Outputs of C columns with C mod 128 in 1..64 run on 64-column tiles;
    the same columns computed inside a 128-multiple-wide call (128-column
    tiles) are bitwise equal: the tile width never changes an element's
    accumulation (one pass and chunk slabs alike)."""
    g = torch.Generator(device=DEV).manual_seed(K + C + M)
    X = torch.randn(M, K, generator=g, device=DEV)
    Cw = -(-C // 128) * 128
    Ww = torch.randn(K, Cw, generator=g, device=DEV) / K ** 0.5
    bw = torch.randn(Cw, generator=g, device=DEV)
    wide = linear_fwd_ex(X, Ww, 0, bw, True, path_rows=M)
    narrow = linear_fwd_ex(X, Ww[:, :C].contiguous(), 0, bw[:C].contiguous(), True, path_rows=M)
    assert torch.equal(narrow, wide[:, :C])


@pytest.mark.parametrize("K,C", [(512, 128), (1792, 256)])
def test_path_rows_pin_the_gemm_path(K, C):
    """A shard-sized call given the whole graph's row count takes the whole
    call's x6 path: its rows bitwise the whole call's (without path_rows the
    small call takes the fp32 path: other bits, same values to 1e-5)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    M = 1 << 18
    X = torch.randn(M, K, generator=g, device=DEV)
    W = torch.randn(K, C, generator=g, device=DEV) / K ** 0.5
    full = linear_fwd_ex(X, W, 0, None, False)
    for r0, r1 in ((0, 1000), (4096, 9000), (100_000, 130_000)):
        pinned = linear_fwd_ex(X[r0:r1].contiguous(), W, 0, None, False, path_rows=M)
        assert torch.equal(pinned, full[r0:r1])
        free = linear_fwd_ex(X[r0:r1].contiguous(), W, 0, None, False)
        assert float((free - full[r0:r1]).abs().max()) <= 1e-5 * max(1.0, float(full.abs().max()))


def test_row_linear_is_nn_linear():
    """row_linear (nn.Linear layout on the libgrl GEMM, ReLU fused) against
    float64 torch: forward, dX, dW, db; and its rows M-invariant."""
    g = torch.Generator(device=DEV).manual_seed(9)
    M, K, C = 5000, 512, 128
    lin = torch.nn.Linear(K, C).to(DEV)
    X = torch.randn(M, K, generator=g, device=DEV, requires_grad=True)
    out = row_linear(X, lin.weight, lin.bias, relu=True)
    G = torch.randn(M, C, generator=g, device=DEV)
    out.backward(G)
    Xd = X.detach().double().requires_grad_(True)
    Wd = lin.weight.detach().double().requires_grad_(True)
    bd = lin.bias.detach().double().requires_grad_(True)
    ref = torch.relu(Xd @ Wd.t() + bd)
    ref.backward(G.double())
    for a, r in ((out, ref), (X.grad, Xd.grad), (lin.weight.grad, Wd.grad), (lin.bias.grad, bd.grad)):
        assert float((a.double() - r).abs().max()) <= 1e-5 * max(1.0, float(r.abs().max()))
    with torch.no_grad():
        part = row_linear(X[1234:3456].detach(), lin.weight, lin.bias, relu=True)
    assert torch.equal(part, out.detach()[1234:3456])


@pytest.mark.parametrize("N,dk,dv", [(7500, 4, 32), (6000, 16, 128), (20000, 16, 128)])
def test_attention_query_range_rows_equal_whole(N, dk, dv):
    """grl_node_attention_fwd_rows over a query range uses the whole call's
    key split: its rows (out, o_norm, row max / sum) bitwise the whole-range
    call's rows; rows outside the range stay 0 (row sum 1)."""
    g = torch.Generator(device=DEV).manual_seed(N)
    Q = torch.relu(torch.randn(1, N, dk, generator=g, device=DEV))
    K = torch.relu(torch.randn(1, N, dk, generator=g, device=DEV))
    H = torch.relu(torch.randn(1, N, dv, generator=g, device=DEV))
    V = torch.randn(1, N, dv, generator=g, device=DEV)
    gm = torch.randn(dv, generator=g, device=DEV)
    whole = node_attention_forward(Q, K, H, V, gm, stats=True)
    for q0, q1 in ((0, N // 3), (N // 3, 2 * N // 3 + 5), (N - 777, N)):
        part = node_attention_forward(Q, K, H, V, gm, stats=True, q_range=(q0, q1))
        for a, b in zip(part, whole):
            assert torch.equal(a[0, q0:q1], b[0, q0:q1]), (q0, q1)
        assert float(part[0][0, :q0].abs().sum()) == 0.0 and float(part[0][0, q1:].abs().sum()) == 0.0


@pytest.mark.parametrize("rows,cols,row0,p", [(1000, 256, 0, 0.5), (777, 1280, 4321, 0.5), (300, 53, 12, 0.3),
                                              (64, 128, 0, 0.0)])
def test_feature_dropout_is_the_hash_mask(rows, cols, row0, p):
    """feature_dropout: out = x * 1/(1-p) where the hash of (seed, call,
    (row0 + r) * cols + c) keeps the element, else 0 (the oracle's
    restatement of the counter hash), forward and backward; a row block
    masked on its own equals the same rows of the whole tensor."""
    from oracle import hash as ohash

    seed, call = 77, (1 << 48) + 3
    x = torch.randn(rows, cols, device=DEV, requires_grad=True)
    de = DropEdge(p, seed, call)
    out = feature_dropout(x, de, row0)
    ids = (np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row0)) * np.uint64(cols) \
        + np.arange(cols, dtype=np.uint64)[None, :]
    keep = torch.from_numpy(ohash.dropedge_keep(p, seed, call, ids.reshape(-1)).reshape(rows, cols)).to(DEV)
    _, _, scale = ohash.dropedge_params(p)
    want = torch.where(keep, x.detach() * float(scale), torch.zeros((), device=DEV))
    assert torch.equal(out.detach(), want)
    g = torch.randn(rows, cols, device=DEV)
    out.backward(g)
    assert torch.equal(x.grad, torch.where(keep, g * float(scale), torch.zeros((), device=DEV)))
    if p > 0:
        kept = float(keep.float().mean())
        assert abs(kept - (1 - p)) < 0.05
    with torch.no_grad():
        part = feature_dropout(x.detach()[rows // 3:], de, row0 + rows // 3)
    assert torch.equal(part, out.detach()[rows // 3:])


def test_feature_dropout_module_shard_rows_equal_one_gpu():
    """The model's FeatureDropout on a shard's rows (row0 = the shard's first
    global row) draws the one-GPU model's mask for those rows; eval and p = 0
    are the identity."""
    from gnn.models.networks.drop_robust_gcn import FeatureDropout

    fd = FeatureDropout(0.5, seed=5).train()
    x = torch.randn(3000, 256, device=DEV)
    whole = fd(x)
    fd.reset_calls()
    fd.row0 = 1000
    part = fd(x[1000:2000])
    assert torch.equal(part, whole[1000:2000])
    fd.eval()
    assert fd(x) is x
