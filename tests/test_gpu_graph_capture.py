"""GPU: the C1 training step (kv_procedure.py:143-164 in the reference:
forward, cross-entropy, backward, clip, Adam) captured as ONE HIP graph.

The DropEdge seed lives in device memory (GrlDropEdge.seed_dev, written by
a device RNG kernel captured with the step), so replays draw fresh masks
without a host round trip.  Checks:
  * a device-resident seed gives exactly the host seed's mask and Z;
  * replays of a captured step equal eager steps (fixed DropEdge stream,
    feature dropout off, capturable Adam on both sides);
  * with device seeds each replay draws a new mask and the model trains."""
import copy

import numpy as np
import pytest
import torch

from grl import DropEdge, TypedGraph
from grl.ops import spmm_forward

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_device_seed_equals_host_seed():
    g = TypedGraph.synthetic(4096, 20.0, 6, seed=2, device=DEV)
    X = torch.randn(4096, 64, device=DEV)
    for seed, call in ((12345, 0), (2**61 + 7, 3)):
        t = torch.tensor([seed], dtype=torch.int64, device=DEV)
        Zh = spmm_forward(X, g.with_dropedge(DropEdge(0.3, seed, call)))
        Zd = spmm_forward(X, g.with_dropedge(DropEdge(0.3, 0, call, seed_tensor=t)))
        assert torch.equal(Zh, Zd)
        mh = g.dropedge_mask(DropEdge(0.3, seed, call), 0, 1000)
        md = g.dropedge_mask(DropEdge(0.3, 0, call, seed_tensor=t), 0, 1000)
        assert torch.equal(mh, md)
    # the seed is read at launch: rewriting it changes the next launch's mask
    t = torch.tensor([1], dtype=torch.int64, device=DEV)
    de = DropEdge(0.3, 0, 0, seed_tensor=t)
    Z1 = spmm_forward(X, g.with_dropedge(de)).clone()
    t.fill_(2)
    Z2 = spmm_forward(X, g.with_dropedge(de))
    assert not torch.equal(Z1, Z2)
    assert torch.equal(Z2, spmm_forward(X, g.with_dropedge(DropEdge(0.3, 2, 0))))


def _batch(B=4, N=40, F=64, L=6, C=15, seed=3):
    rng = np.random.default_rng(seed)
    V = torch.from_numpy((rng.random((B, N, F)) < 0.1).astype(np.float32)).to(DEV)
    A = torch.from_numpy((rng.random((B, N, L, N)) < 3.0 / (L * N)).astype(np.float32)).to(DEV)
    y = torch.from_numpy(rng.integers(0, C, (B, N))).to(DEV)
    return V, A, y


def _make(dropedge_seed, feat_p):
    from gnn.models import GraphCNNDropEdge

    torch.manual_seed(0)
    m = GraphCNNDropEdge(64, 15, 6, net_size=32, dropedge_seed=dropedge_seed).to(DEV)
    m.dropout.p = feat_p
    m.train()
    return m


def _step(model, opt, V, graph, y):
    logits = model.forward([V, graph])
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1))
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0)
    opt.step()
    return loss


def _capture(model, opt, V, graph, y, warm=3, before=None):
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        for _ in range(warm):
            if before:
                before()
            opt.zero_grad(set_to_none=True)
            _step(model, opt, V, graph, y)
    torch.cuda.current_stream(DEV).wait_stream(side)
    hg = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=True)
    if before:
        before()
    with torch.cuda.graph(hg):
        static_loss = _step(model, opt, V, graph, y)
    return hg, static_loss


def test_captured_train_step_equals_eager():
    V, A, y = _batch()
    model = _make(dropedge_seed=11, feat_p=0.0)
    ref = copy.deepcopy(model)
    graph = model.to_graph(A)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)
    opt_r = torch.optim.Adam(ref.parameters(), lr=1e-3, capturable=True)
    hg, static_loss = _capture(model, opt, V, graph, y, before=model.edge_dropout.reset_calls)
    for _ in range(3):  # the eager twin takes the same warm-up steps
        ref.edge_dropout.reset_calls()
        opt_r.zero_grad(set_to_none=True)
        _step(ref, opt_r, V, graph, y)
    for i in range(5):
        hg.replay()
        ref.edge_dropout.reset_calls()
        opt_r.zero_grad(set_to_none=True)
        loss_r = _step(ref, opt_r, V, graph, y)
        torch.cuda.synchronize()
        torch.testing.assert_close(static_loss, loss_r, rtol=1e-6, atol=1e-6, msg=f"replay {i}")
        for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-6, msg=f"replay {i}: {n}")


def test_captured_train_step_redraws_masks_and_trains():
    V, A, y = _batch(seed=5)
    model = _make(dropedge_seed=None, feat_p=0.5)  # production: device-seeded DropEdge + feature dropout
    graph = model.to_graph(A)
    opt = torch.optim.Adam(model.parameters(), lr=3e-3, capturable=True)
    hg, static_loss = _capture(model, opt, V, graph, y)
    losses = []
    for _ in range(40):
        hg.replay()
        losses.append(float(static_loss.detach()))
    assert all(np.isfinite(losses))
    assert len(set(losses[:5])) == 5  # new masks every replay
    assert np.mean(losses[-5:]) < np.mean(losses[:5])
