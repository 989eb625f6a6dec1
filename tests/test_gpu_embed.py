"""GPU: emb1 as a sparse-row gather (grl_bag_linear_fwd + MFMA backward)
against float64 torch, on bag-of-characters rows like TextlineEncoding's
(textline_encoding.py:23-42) and on fully dense rows."""
import numpy as np
import pytest
import torch

from grl import _lib
from grl.ops import bag_linear

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _bag_rows(M, K, seed, nnz=7):
    rng = np.random.default_rng(seed)
    V = np.zeros((M, K), np.float32)
    for m in range(M):
        cols = rng.choice(K - 4, size=min(nnz, K - 4), replace=False)
        V[m, cols] = rng.integers(1, 4, len(cols))
    V[:, -4:] = rng.random((M, 4)).astype(np.float32)  # box features (dense)
    return torch.from_numpy(V).to(DEV)


@pytest.mark.parametrize("M,K,C", [(74, 4369, 256), (296, 4369, 256), (1, 70, 100), (130, 64, 64), (50, 200, 512),
                                   (9, 4369, 16)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
def test_forward_backward_match_fp64(M, K, C, relu, bias):
    V = _bag_rows(M, K, seed=M + C)
    g = torch.Generator().manual_seed(K)
    W = (torch.randn(C, K, generator=g) / np.sqrt(K)).to(DEV).requires_grad_(True)
    b = torch.randn(C, generator=g).to(DEV).requires_grad_(True) if bias else None
    Vg = V.clone().requires_grad_(True)
    out = bag_linear(Vg, W, b, relu)
    ref_in = [V.double().clone().requires_grad_(True), W.detach().double().clone().requires_grad_(True)]
    ref_b = b.detach().double().clone().requires_grad_(True) if bias else None
    ref = ref_in[0] @ ref_in[1].T + (ref_b if bias else 0.0)
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5)
    dout = torch.randn(out.shape, generator=torch.Generator().manual_seed(1)).to(DEV)
    out.backward(dout)
    ref.backward(dout.double())
    torch.testing.assert_close(W.grad.double(), ref_in[1].grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(Vg.grad.double(), ref_in[0].grad, rtol=1e-5, atol=1e-4)
    if bias:
        torch.testing.assert_close(b.grad.double(), ref_b.grad, rtol=1e-5, atol=1e-4)


def test_dense_rows_and_batched_shape():
    V = torch.randn(3, 20, 300, device=DEV)
    W = torch.randn(48, 300, device=DEV) / 17
    b = torch.randn(48, device=DEV)
    out = bag_linear(V, W, b, relu=True)
    assert out.shape == (3, 20, 48)
    ref = torch.relu(V.double() @ W.double().T + b.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


def test_model_emb1_sparse_equals_dense():
    from gnn.models import GraphCNNDropEdge

    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 64).to(DEV).eval()
    V = _bag_rows(30, 4369, seed=3)[None]
    with torch.no_grad():
        a = model._embed(V)
        model.sparse_emb1 = False
        d = model._embed(V)
    torch.testing.assert_close(a, d, rtol=1e-5, atol=1e-5)


def test_errors():
    V = torch.zeros(2, 8, device=DEV)
    with pytest.raises(_lib.GrlError, match="output width"):
        bag_linear(V, torch.zeros(600, 8, device=DEV), None)
    with pytest.raises(_lib.GrlError):
        bag_linear(V.cpu(), torch.zeros(4, 8), None)


def _dw_ref(V, g, relu_out):
    """float64 dWt, db and the Sigma|terms| bound per element."""
    gd = g.double()
    if relu_out is not None:
        gd = torch.where(relu_out > 0, gd, torch.zeros((), dtype=gd.dtype, device=gd.device))
    Vd = V.double()
    return Vd.T @ gd, gd.sum(0), Vd.abs().T @ gd.abs(), gd.abs().sum(0)


@pytest.mark.parametrize("M,K,C,relu", [(20_000, 4369, 256, False), (5_000, 4369, 53, True), (3_100, 300, 512, True),
                                        (1, 17, 8, False)])
def test_bag_weight_gradient_sparse_kernel(M, K, C, relu):
    """grl_bag_linear_bwd_weight (emb1's dW / db, one row of g' per nonzero of V)
    against float64 within 1e-5 of sum|terms|, on bag rows (the 4 dense box
    columns make the heaviest column block), several row ranges (M > 1536),
    the fused ReLU mask, C > 256; run to run bitwise."""
    from grl.ops import bag_linear_bwd_weight

    V = _bag_rows(M, K, seed=M) if K > 8 else torch.randn(M, K, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(5)
    g = torch.randn(M, C, generator=gen, device=DEV)
    relu_out = torch.relu(torch.randn(M, C, generator=gen, device=DEV)) if relu else None
    dWt, db = bag_linear_bwd_weight(V, g, relu_out, True)
    rW, rb, aW, ab = _dw_ref(V, g, relu_out)
    assert float(((dWt.double() - rW).abs() - 1e-5 * aW).max()) <= 1e-30
    assert float(((db.double() - rb).abs() - 1e-5 * ab).max()) <= 1e-30
    dWt2, db2 = bag_linear_bwd_weight(V, g, relu_out, True)
    assert torch.equal(dWt, dWt2) and torch.equal(db, db2)
    dWt3, none = bag_linear_bwd_weight(V, g, relu_out, False)
    assert none is None and torch.equal(dWt, dWt3)


def test_bag_weight_gradient_dense_rows_and_strided_V():
    """Every entry nonzero (the list holds whole chunks) and V a column slice
    of a wider tensor (ldv > K)."""
    from grl.ops import bag_linear_bwd_weight

    big = torch.randn(700, 130, device=DEV)
    V = big[:, :100]
    g = torch.randn(700, 40, device=DEV)
    dWt, db = bag_linear_bwd_weight(V, g, None, True)
    rW, rb, aW, ab = _dw_ref(V, g, None)
    assert float(((dWt.double() - rW).abs() - 1e-5 * aW).max()) <= 1e-30
    assert float(((db.double() - rb).abs() - 1e-5 * ab).max()) <= 1e-30


def test_model_path_routes_large_bags_to_the_sparse_gradient():
    """bag_linear's backward at M >= BAG_DW_SPARSE_ROWS takes the sparse dW
    kernel and still matches float64 (1e-5 of sum|terms|)."""
    from grl.ops import BAG_DW_SPARSE_ROWS

    M, K, C = BAG_DW_SPARSE_ROWS + 100, 4369, 64
    V = _bag_rows(M, K, seed=11)
    W = (torch.randn(C, K, generator=torch.Generator().manual_seed(2)) / 8).to(DEV).requires_grad_(True)
    b = torch.zeros(C, device=DEV, requires_grad=True)
    out = bag_linear(V, W, b, relu=True)
    dout = torch.randn(out.shape, generator=torch.Generator(device=DEV).manual_seed(3), device=DEV)
    out.backward(dout)
    gref = torch.where(out.detach() > 0, dout, torch.zeros((), device=DEV)).double()
    rW = (V.double().T @ gref).T
    aW = (V.double().abs().T @ gref.abs()).T
    assert float(((W.grad.double() - rW).abs() - 1e-5 * aW).max()) <= 1e-30
    torch.testing.assert_close(b.grad.double(), gref.sum(0), rtol=1e-5, atol=1e-4)


def test_bag_weight_gradient_edges():
    """No rows: zero gradients; one output column; all-zero V (no entries)."""
    from grl.ops import bag_linear_bwd_weight

    dWt, db = bag_linear_bwd_weight(torch.zeros(0, 30, device=DEV), torch.zeros(0, 7, device=DEV), None, True)
    assert dWt.shape == (30, 7) and not dWt.any() and not db.any()
    V = _bag_rows(3000, 100, seed=4)
    g = torch.randn(3000, 1, device=DEV)
    dWt, db = bag_linear_bwd_weight(V, g, None, True)
    torch.testing.assert_close(dWt.double(), V.double().T @ g.double(), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db.double(), g.double().sum(0), rtol=1e-5, atol=1e-4)
    dWt, db = bag_linear_bwd_weight(torch.zeros(2000, 50, device=DEV), torch.randn(2000, 9, device=DEV), None, False)
    assert db is None and not dWt.any()
