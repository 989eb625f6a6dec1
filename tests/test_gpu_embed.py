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
