"""GPU: grl_graphconv_fwd, one GraphConv layer forward in one call
(robust_gcn.py:45-51): bitwise equal to the two-op path (typed SpMM then the
linear), for whole-graph and row-chunked workspaces, and within fp32
tolerance of the oracle's aggregation times W in fp64."""
import numpy as np
import pytest
import torch

from grl import DropEdge, TypedGraph, _lib
from grl.ops import graph_conv, graph_conv_infer, linear_fwd, typed_aggregate, x6_rows_ok
from oracle import c_oracle
from oracle import hash as ohash

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _two_op(X, g, W, b, relu):
    Z = typed_aggregate(X, g)
    return linear_fwd(Z, W, b, relu)


def _planes_bytes(K, C):
    return 3 * ((C + 255) // 256 * 256) * K * 2 + 256 + 256


@pytest.mark.parametrize("N,L,deg,F,C,has_self", [(300, 6, 16.0, 256, 64, True), (129, 6, 8.0, 10, 7, True),
                                                   (200, 3, 12.0, 100, 36, False), (74, 6, 3.0, 256, 256, True)])
@pytest.mark.parametrize("relu,bias", [(True, True), (False, False)])
@pytest.mark.parametrize("di", [0, 1])
def test_graphconv_small_matches_two_ops_and_oracle(N, L, deg, F, C, has_self, relu, bias, di):
    rowptr, colidx = ohash.synth_csr(0, L, N, int(N * deg), 11)
    de = [None, DropEdge(0.3, 7, 1, True)][di]
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV, has_self=has_self).with_dropedge(de)
    rng = np.random.default_rng(N + F)
    X = rng.standard_normal((N, F)).astype(np.float32)
    K = (L + (1 if has_self else 0)) * F
    W = (rng.standard_normal((K, C)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32) if bias else None
    Xt, Wt = torch.from_numpy(X).to(DEV), torch.from_numpy(W).to(DEV)
    bt = torch.from_numpy(b).to(DEV) if bias else None
    out = graph_conv_infer(Xt, g, Wt, bt, relu)
    ref = _two_op(Xt, g, Wt, bt, relu)
    assert torch.equal(out, ref)
    with torch.no_grad():  # graph_conv routes here when no gradient is wanted
        assert torch.equal(graph_conv(Xt, g, Wt, bt, relu), out)
    d = None if de is None else c_oracle.drop(de.p, de.seed, de.call, de.drop_self)
    Z = c_oracle.spmm_fwd(rowptr, colidx, X, L, has_self, d=d).astype(np.float64)
    o = Z @ W.astype(np.float64) + (b.astype(np.float64) if bias else 0.0)
    if relu:
        o = np.maximum(o, 0.0)
    scale = np.abs(Z) @ np.abs(W.astype(np.float64)) + (np.abs(b.astype(np.float64)) if bias else 0.0)
    assert np.all(np.abs(out.cpu().numpy() - o) <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("di,strided", [(0, False), (1, False), (2, True)])
def test_graphconv_row_chunks_bitwise(di, strided, monkeypatch, grl_option):
    """Bounded workspace on the two-kernel path: rows in chunks (here 12
    chunks, the last partial) give the whole-graph bits, which are the
    two-op bits (also with X a column slice of a wider matrix, and DropEdge
    sparing the self loops)."""
    grl_option("graphconv_fused", 0)
    N, L, F, C = 100_003, 6, 256, 256
    de = [None, DropEdge(0.3, 2, 0, True), DropEdge(0.2, 5, 3, False)][di]
    g = TypedGraph.synthetic(N, 16.0, L, seed=0, device=DEV).with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(1)
    X = torch.randn(N, F + 64 if strided else F, device=DEV, generator=gen)[:, :F]
    assert X.stride(0) == (F + 64 if strided else F)
    K = (L + 1) * F
    W = torch.randn(K, C, device=DEV, generator=gen) / K ** 0.5
    b = torch.randn(C, device=DEV, generator=gen)
    full = graph_conv_infer(X, g, W, b, True)
    chunked = graph_conv_infer(X, g, W, b, True, max_workspace_bytes=_planes_bytes(K, C) + 8704 * K * 4)
    assert torch.equal(full, chunked)
    assert torch.equal(full, _two_op(X, g, W, b, True))


def test_graphconv_workspace_errors():
    """Chunking needs the x6 GEMM shape and no heavy-row split plan: else a
    too-small workspace is an error, never a silent fallback."""
    rowptr, colidx = ohash.synth_csr(0, 6, 300, 4800, 3)
    g = TypedGraph.from_csr_host(rowptr, colidx, 6, DEV)
    X = torch.randn(300, 64, device=DEV)
    W = torch.randn(7 * 64, 32, device=DEV)
    with pytest.raises(_lib.GrlError, match="workspace"):
        graph_conv_infer(X, g, W, None, False, max_workspace_bytes=4096)
    # power-law graph whose heavy rows are split: whole-graph workspace only
    N, L, F, C = 1 << 16, 6, 256, 256
    rp, ci = ohash.synth_csr(1, L, N, N * 16, 21)
    gr = TypedGraph.from_csr_host(rp, ci, L, DEV)
    gr.split_threshold, gr.split_chunk = 256, 128
    Xr = torch.randn(N, F, device=DEV)
    Wr = torch.randn(7 * F, C, device=DEV) / (7 * F) ** 0.5
    out = graph_conv_infer(Xr, gr, Wr, None, False)
    assert gr.split_stats()["csr"]["heavy_segments"] > 0
    assert torch.equal(out, _two_op(Xr, gr, Wr, None, False))
    with pytest.raises(_lib.GrlError, match="split plan"):
        graph_conv_infer(Xr, gr, Wr, None, False, max_workspace_bytes=_planes_bytes(7 * F, C) + 4096 * 7 * F * 4)


@pytest.mark.parametrize("relu", [True, False])
def test_recompute_z_gives_the_same_gradients_with_less_memory(relu):
    """graph_conv(recompute=True) keeps X, not Z = A_drop X, between the
    passes and re-aggregates Z in the backward (same DropEdge record): out,
    dX, dW and db bitwise equal to the saved-Z path, and the memory held
    across the passes drops by about Z's size."""
    N, F, C = 60_000, 128, 96
    g = TypedGraph.synthetic(N, 16.0, 6, seed=6, device=DEV).with_dropedge(DropEdge(0.3, 8, 1))
    X0 = torch.randn(N, F, device=DEV)
    W0 = torch.randn(7 * F, C, device=DEV) / 30
    b0 = torch.randn(C, device=DEV)
    R = torch.randn(N, C, device=DEV)
    res, held = {}, {}
    for rc in (False, True):
        X, W, b = (t.clone().requires_grad_(True) for t in (X0, W0, b0))
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(DEV)
        out = graph_conv(X, g, W, b, relu=relu, recompute=rc)
        torch.cuda.synchronize()
        held[rc] = torch.cuda.memory_allocated(DEV) - base
        (out * R).sum().backward()
        res[rc] = (out.detach(), X.grad, W.grad, b.grad)
        del out
    for a, c in zip(res[False], res[True]):
        assert torch.equal(a, c)
    z_bytes = N * 7 * F * 4
    assert held[False] - held[True] >= 0.9 * z_bytes, held
    # auto mode keeps Z for graphs below RECOMPUTE_Z_BYTES
    from grl import ops

    assert z_bytes < ops.RECOMPUTE_Z_BYTES


def _ws_query(X, g, W, C):
    csr = g.csr_c(X.shape[1])
    import ctypes
    return _lib.lib().grl_graphconv_fwd_workspace_query(ctypes.byref(csr), X.data_ptr(), X.stride(0), X.shape[1],
                                                        W.data_ptr(), C)


# sizes just above the x6 GEMM's 1.6e10-flop threshold (below it the linear,
# hence the two-kernel reference, is the fp32-MFMA kernel and no fusion runs);
# avg_deg 120 puts ~160 edges in a gather wave's segment list (more than one
# 64-entry fetch), L = 7 fills the wave's rowptr window (8 rows x 7 + 1)
@pytest.mark.parametrize("N,L,F,C,has_self,deg", [(20_011, 6, 256, 256, True, 16.0), (50_000, 6, 256, 96, True, 9.0),
                                                  (40_007, 6, 128, 256, True, 16.0), (70_001, 6, 64, 256, True, 12.0),
                                                  (60_001, 3, 256, 200, False, 20.0), (20_000, 6, 256, 256, True, 120.0),
                                                  (18_001, 7, 256, 256, True, 14.0),
                                                  # wide: F = 512 / 1024 as 256-column virtual segments (gcn3's
                                                  # 2C input, C5's d = 512), C > 256 on 4 gather + 8 MFMA waves
                                                  (20_011, 6, 512, 256, True, 10.0), (20_011, 6, 512, 512, True, 10.0),
                                                  (24_001, 6, 256, 512, True, 12.0), (10_007, 6, 1024, 512, True, 8.0),
                                                  (30_001, 6, 128, 384, True, 12.0), (20_000, 6, 256, 512, True, 120.0),
                                                  (18_001, 7, 512, 500, True, 14.0), (40_003, 3, 512, 260, False, 9.0)])
@pytest.mark.parametrize("variant", ["plain", "drop_bias_relu", "drop_spare_self", "strided_relu"])
@pytest.mark.parametrize("kernel", ["ws", "phases"])
def test_fused_graphconv_bitwise_equals_two_kernels(N, L, F, C, has_self, deg, variant, kernel, monkeypatch, grl_option):
    """The one-kernel GraphConv (graphconv.hip; both kernels: the
    warp-specialized default and the phase-alternating fg_ws = 0 one)
    gives the two-kernel bits (typed SpMM, then the x6 GEMM): the same fmaf
    chain per Z element, the same split, K order and product order; and it
    runs in a workspace of only W's planes (Z never reaches HBM)."""
    grl_option("fg_ws", int("1" if kernel == "ws" else "0"))
    de = {"plain": None, "drop_bias_relu": DropEdge(0.3, 3, 2, True), "drop_spare_self": DropEdge(0.25, 9, 0, False),
          "strided_relu": None}[variant]
    bias = variant == "drop_bias_relu"
    relu = variant in ("drop_bias_relu", "strided_relu")
    g = TypedGraph.synthetic(N, deg, L, seed=N % 7, device=DEV)
    if not has_self:
        g = TypedGraph(g.rowptr, g.colidx, L, has_self=False, num_cols=N)
    g = g.with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(N + F)
    wide = F + 64 if variant == "strided_relu" else F
    X = torch.randn(N, wide, device=DEV, generator=gen)[:, :F]
    K = (L + (1 if has_self else 0)) * F
    W = torch.randn(K, C, device=DEV, generator=gen) / K ** 0.5
    b = torch.randn(C, device=DEV, generator=gen) if bias else None
    if deg > 64:  # no heavy-row split plan on this graph: the fused path applies
        assert g.split_stats()["csr"]["heavy_segments"] == 0
    ws = _ws_query(X, g, W, C)
    assert ws < 3 * (256 if C <= 256 else 512) * K * 2 + 4096 < N * K * 4, ws  # W planes only: the fused path
    out = graph_conv_infer(X, g, W, b, relu)
    ref = _two_op(X, g, W, b, relu)
    assert torch.equal(out, ref)
    grl_option("graphconv_fused", 0)
    assert _ws_query(X, g, W, C) >= N * K * 4
    assert torch.equal(graph_conv_infer(X, g, W, b, relu), out)


def test_fused_graphconv_edge_values_and_oracle():
    """fc_similarity-style edge values (vals != NULL) through the fused
    kernel: bitwise the two-kernel result, and within 1e-5 sum|terms| of the
    oracle's Z times W in fp64 on sampled rows."""
    N, L, F, C = 20_480, 6, 256, 256
    rowptr, colidx = ohash.synth_csr(0, L, N, N * 12, 5)
    rng = np.random.default_rng(3)
    vals = rng.random(len(colidx)).astype(np.float32)
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV, vals=vals).with_dropedge(DropEdge(0.3, 1, 4, True))
    X = rng.standard_normal((N, F)).astype(np.float32)
    K = 7 * F
    W = (rng.standard_normal((K, C)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32)
    Xt, Wt, bt = (torch.from_numpy(a).to(DEV) for a in (X, W, b))
    assert _ws_query(Xt, g, Wt, C) < N * K * 4
    out = graph_conv_infer(Xt, g, Wt, bt, True)
    assert torch.equal(out, _two_op(Xt, g, Wt, bt, True))
    de = g.dropedge
    Z = c_oracle.spmm_fwd(rowptr, colidx, X, L, True, vals=vals,
                          d=c_oracle.drop(de.p, de.seed, de.call, de.drop_self)).astype(np.float64)
    rows = np.r_[0:64, N - 64:N, rng.integers(0, N, 512)]
    o = np.maximum(Z[rows] @ W.astype(np.float64) + b, 0.0)
    scale = np.abs(Z[rows]) @ np.abs(W.astype(np.float64)) + np.abs(b)
    assert np.all(np.abs(out.cpu().numpy()[rows] - o) <= 1e-5 * scale + 1e-6)


@pytest.mark.parametrize("de", [None, DropEdge(0.3, 4, 2, True)])
@pytest.mark.parametrize("recompute", [False, True])
def test_training_forward_one_kernel_same_bits(de, recompute, monkeypatch, grl_option):
    """The training GraphConv (graph_conv with gradients) runs its forward as
    one kernel that also writes Z for the backward (grl_graphconv_fwd_train),
    or -- recompute=True -- as the inference kernel; out, Z and every
    gradient are bitwise those of the two-kernel path (graphconv_fused = 0)."""
    from grl.ops import graph_conv_fwd_train, spmm_forward

    N, L, F, C = 20_011, 6, 256, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=3, device=DEV).with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(5)
    X0 = torch.randn(N, F, device=DEV, generator=gen)
    W0 = torch.randn(7 * F, C, device=DEV, generator=gen) / 40
    b0 = torch.randn(C, device=DEV, generator=gen)
    R = torch.randn(N, C, device=DEV, generator=gen)
    out_f, Z_f = graph_conv_fwd_train(X0, g, W0, b0, True)
    assert torch.equal(Z_f, spmm_forward(X0, g))
    grl_option("graphconv_fused_bwd", 0)  # dX by the chain (the reassociated one: test below)
    res = {}
    for fused in ("1", "0"):
        grl_option("graphconv_fused", int(fused))
        X, W, b = (t.clone().requires_grad_(True) for t in (X0, W0, b0))
        out = graph_conv(X, g, W, b, relu=True, recompute=recompute)
        (out * R).sum().backward()
        res[fused] = (out.detach(), X.grad, W.grad, b.grad)
    assert torch.equal(res["1"][0], out_f)
    for a, c in zip(res["1"], res["0"]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("F,C", [(512, 256), (512, 512), (256, 512), (1024, 512)])
@pytest.mark.parametrize("de", [None, DropEdge(0.3, 4, 2, True)])
def test_wide_training_forward_one_kernel_same_bits(F, C, de):
    """The training forward at gcn3's F = 2C and at d = 512 (C5): the one
    kernel (256-column virtual segments; 8 MFMA waves for C > 256) writes
    out and Z bitwise those of the two-kernel path, and the layer's
    gradients through graph_conv equal the chain's (dX within fp32 rounding
    of the one-kernel reassociation, dW / db bitwise)."""
    from grl.ops import graph_conv_fwd_train, spmm_forward

    N, L = (12_007 if F == 1024 else 20_011), 6
    g = TypedGraph.synthetic(N, 10.0, L, seed=2, device=DEV).with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(F + C)
    X = torch.randn(N, F, device=DEV, generator=gen)
    W = torch.randn(7 * F, C, device=DEV, generator=gen) / (7 * F) ** 0.5
    b = torch.randn(C, device=DEV, generator=gen)
    out, Z = graph_conv_fwd_train(X, g, W, b, True)
    Zr = spmm_forward(X, g)
    assert torch.equal(Z, Zr)
    assert torch.equal(out, linear_fwd(Zr, W, b, True))
    assert torch.equal(graph_conv_infer(X, g, W, b, True), out)


@pytest.mark.parametrize("N,L,F,C,has_self,deg", [(20_011, 6, 256, 256, True, 16.0), (100_003, 6, 96, 128, True, 9.0),
                                                  (80_000, 6, 256, 64, True, 12.0), (60_001, 3, 200, 256, False, 20.0),
                                                  (20_000, 6, 256, 256, True, 120.0), (18_001, 7, 256, 256, True, 14.0),
                                                  (20_011, 6, 512, 256, True, 10.0), (40_011, 6, 260, 256, True, 8.0),
                                                  (20_011, 6, 512, 512, True, 10.0), (20_011, 6, 256, 512, True, 10.0),
                                                  (10_007, 6, 1024, 512, True, 8.0), (18_001, 7, 384, 512, True, 12.0)])
@pytest.mark.parametrize("variant", ["plain", "drop_self", "drop_spare_self_vals"])
def test_bwd_data_one_kernel(N, L, F, C, has_self, deg, variant, monkeypatch, grl_option):
    """grl_graphconv_bwd_data: dX = sum_s (A_drop,s^T G) W_s^T in one kernel
    over the typed transpose (DropEdge ids through eid, so the forward's
    mask) against the autograd chain dZ = G W^T, dX = A_drop^T dZ: within
    1e-5 of the chain run on |G|, |W| (fp32-level: the same products summed
    in another order), deterministic, and what graph_conv's backward returns
    (dW / db unchanged, bitwise)."""
    from grl.ops import graph_conv_bwd_data, linear_bwd_data, spmm_backward

    de = {"plain": None, "drop_self": DropEdge(0.3, 3, 2, True), "drop_spare_self_vals": DropEdge(0.25, 9, 0, False)}
    de = de[variant]
    g = TypedGraph.synthetic(N, deg, L, seed=N % 5, device=DEV)
    if variant.endswith("vals"):
        vals = torch.rand(g.nnz, generator=torch.Generator(device=DEV).manual_seed(2), device=DEV)
        g = TypedGraph(g.rowptr, g.colidx, L, vals=vals, has_self=has_self, num_cols=N)
    elif not has_self:
        g = TypedGraph(g.rowptr, g.colidx, L, has_self=False, num_cols=N)
    g = g.with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(N + F)
    K = g.segments * F
    G = torch.randn(N, C, device=DEV, generator=gen)
    W = torch.randn(K, C, device=DEV, generator=gen) / K ** 0.5
    dX = graph_conv_bwd_data(G, g, W, F)
    assert dX is not None, "shape should take the one-kernel path"
    assert torch.equal(graph_conv_bwd_data(G, g, W, F), dX)  # deterministic
    chain = spmm_backward(linear_bwd_data(G, None, W), g, F)
    bound = spmm_backward(linear_bwd_data(G.abs(), None, W.abs()), g.with_dropedge(de), F)
    err = (dX - chain).abs()
    assert bool((err <= 1e-5 * bound + 1e-6).all()), float((err / (bound + 1e-30)).max())
    # through autograd (ReLU on): X.grad is the one-kernel dX of g * [out > 0]; dW, db the chain's bits
    X0 = torch.randn(N, F, device=DEV, generator=gen)
    b0 = torch.randn(C, device=DEV, generator=gen)
    res = {}
    for fb in ("1", "0"):
        grl_option("graphconv_fused_bwd", int(fb))
        X, Wp, b = (t.clone().requires_grad_(True) for t in (X0, W, b0))
        out = graph_conv(X, g, Wp, b, relu=True)
        (out * G).sum().backward()
        res[fb] = (out.detach(), X.grad, Wp.grad, b.grad)
    grl_option("graphconv_fused_bwd", 1)
    assert torch.equal(res["1"][1], graph_conv_bwd_data(G, g, W, F, res["1"][0]))
    assert torch.equal(res["1"][0], res["0"][0]) and torch.equal(res["1"][2], res["0"][2])
    assert torch.equal(res["1"][3], res["0"][3])
    Gm = torch.where(res["1"][0] > 0, G, torch.zeros((), device=DEV))
    bound = spmm_backward(linear_bwd_data(Gm.abs(), None, W.abs()), g, F)
    assert bool(((res["1"][1] - res["0"][1]).abs() <= 1e-5 * bound + 1e-6).all())


def test_bwd_data_falls_back_outside_its_shapes():
    """Small graphs, C outside {64, 128, 256} or a non-square shard: None (the
    caller runs the chain); the C entry refuses with GRL_E_UNSUPPORTED."""
    import ctypes

    from grl.ops import graph_conv_bwd_data

    g = TypedGraph.synthetic(2000, 8.0, 6, seed=1, device=DEV)
    assert graph_conv_bwd_data(torch.randn(2000, 256, device=DEV), g, torch.randn(7 * 256, 256, device=DEV), 256) is None
    g = TypedGraph.synthetic(30_000, 8.0, 6, seed=1, device=DEV)
    assert graph_conv_bwd_data(torch.randn(30_000, 96, device=DEV), g, torch.randn(7 * 256, 96, device=DEV), 256) is None
    gt, eid = g.typed_transpose()
    csr = gt.csr_c(96)
    G = torch.randn(30_000, 96, device=DEV)
    rc = _lib.lib().grl_graphconv_bwd_data(ctypes.byref(csr), eid.data_ptr(), G.data_ptr(), 96, 30_000, 96,
                                           torch.empty(7 * 256, 96, device=DEV).data_ptr(), 256,
                                           torch.empty(30_000, 256, device=DEV).data_ptr(), None, None, None, 0, None)
    assert rc == _lib.GRL_E_UNSUPPORTED


@pytest.mark.parametrize("de", [None, DropEdge(0.3, 4, 2, True)])
def test_recompute_takes_weight_gradient_from_the_aggregate(de):
    """recompute=True on a one-kernel-eligible layer: X is kept, not Z, and
    the backward re-aggregates nothing -- the data-gradient kernel also
    writes G_s = A_drop,s^T g and dW_s = X^T G_s.  out and dX bitwise the
    saved-Z path's; dW and db the same products in another order (within
    1e-5 of the sums of |terms|); the held memory drops by Z."""
    from grl.ops import linear_bwd_weight, spmm_forward

    N, L, F, C = 20_011, 6, 256, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=3, device=DEV).with_dropedge(de)
    gen = torch.Generator(device=DEV).manual_seed(5)
    X0 = torch.randn(N, F, device=DEV, generator=gen)
    W0 = torch.randn(7 * F, C, device=DEV, generator=gen) / 40
    b0 = torch.randn(C, device=DEV, generator=gen)
    R = torch.randn(N, C, device=DEV, generator=gen)
    res, held = {}, {}
    for rc in (False, True):
        X, W, b = (t.clone().requires_grad_(True) for t in (X0, W0, b0))
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(DEV)
        out = graph_conv(X, g, W, b, relu=True, recompute=rc)
        torch.cuda.synchronize()
        held[rc] = torch.cuda.memory_allocated(DEV) - base
        (out * R).sum().backward()
        res[rc] = (out.detach(), X.grad, W.grad, b.grad)
        del out
    assert torch.equal(res[True][0], res[False][0]) and torch.equal(res[True][1], res[False][1])
    assert held[False] - held[True] >= 0.9 * N * 7 * F * 4, held
    ge = torch.where(res[False][0] > 0, R, torch.zeros((), device=DEV))
    Z = spmm_forward(X0, g)
    bound_w, _ = linear_bwd_weight(Z.abs(), ge.abs(), None, False)
    assert bool(((res[True][2] - res[False][2]).abs() <= 1e-5 * bound_w + 1e-6).all())
    bound_b = ge.abs().sum(0)
    assert bool(((res[True][3] - res[False][3]).abs() <= 1e-5 * bound_b + 1e-6).all())


def test_persistent_kernel_timeout_is_an_error(monkeypatch, grl_option):
    """graphconv_ws_kernel's bounded waits: with a one-sleep bound
    (ws_spin = 1) the MFMA waves give up before the gather waves fill the
    ring.  The calls stay stream-ordered (no host sync): a follow-up kernel
    fills each failed call's outputs with NaN and records the entry point in
    the sticky device word, and grl.check() -- at the caller's next sync
    point -- raises GrlError(GRL_E_TIMEOUT) naming every failed entry point,
    then clears the word.  Replays of a captured call fail the same way.
    ws_status_sync = 1 keeps the per-call check (the call itself raises).
    With the normal bound the next call is correct again."""
    import grl
    from grl.ops import graph_conv_bwd_data

    N, L, F, C = 20_011, 6, 256, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=3, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(9)
    X = torch.randn(N, F, device=DEV, generator=gen)
    W = torch.randn(7 * F, C, device=DEV, generator=gen) / 40
    b = torch.randn(C, device=DEV, generator=gen)
    ref = graph_conv_infer(X, g, W, b, True)
    assert torch.equal(ref, _two_op(X, g, W, b, True))  # the one-kernel shape
    G = torch.randn(N, C, device=DEV, generator=gen)
    dX_ref = graph_conv_bwd_data(G, g, W, F)
    assert dX_ref is not None
    grl.check()  # nothing pending
    grl_option("ws_spin", 1)
    out = graph_conv_infer(X, g, W, b, True)  # no raise, no sync: the failure is stream-ordered
    with pytest.raises(_lib.GrlError, match=r"grl_graphconv_fwd: a wave .* gave up waiting"):
        grl.check()
    assert bool(torch.isnan(out).all())
    grl.check()  # cleared
    Xg = X.clone().requires_grad_(True)
    out_t = graph_conv(Xg, g, W, b, relu=True)
    dX = graph_conv_bwd_data(G, g, W, F)
    with pytest.raises(_lib.GrlError, match="grl_graphconv_fwd_train, grl_graphconv_bwd_data"):
        grl.check()
    assert bool(torch.isnan(out_t).all()) and bool(torch.isnan(dX).all())
    grl_option("ws_status_sync", 1)  # debug aid: every eager call checks itself
    with pytest.raises(_lib.GrlError, match="gave up waiting"):
        graph_conv_infer(X, g, W, b, True)
    grl_option("ws_status_sync", 0)
    # inside a capture: the replay's outputs are NaN and grl.check() reports it
    hg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(hg):
        out_c = graph_conv_infer(X, g, W, b, True)
    hg.replay()
    with pytest.raises(_lib.GrlError, match="grl_graphconv_fwd"):
        grl.check()
    assert bool(torch.isnan(out_c).all())
    grl_option("ws_spin", 0)
    assert torch.equal(graph_conv_infer(X, g, W, b, True), ref)
    assert torch.equal(graph_conv_bwd_data(G, g, W, F), dX_ref)
    grl.check()
    hg.replay()  # the captured call reads the bound at capture: it still times out
    torch.cuda.synchronize()
    assert bool(torch.isnan(out_c).all())
    with pytest.raises(_lib.GrlError):
        grl.check()


def test_timeout_report_is_never_lost_between_checks(monkeypatch, grl_option):
    """grl_check takes the sticky word with ONE atomic exchange (its old value
    written to a pinned host word): a poisoned call on another stream that
    lands while checks run on this stream is reported by exactly one check
    -- never lost between a read and a separate clear, never twice."""
    import grl

    N, L, F, C = 20_011, 6, 256, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=3, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(9)
    X = torch.randn(N, F, device=DEV, generator=gen)
    W = torch.randn(7 * F, C, device=DEV, generator=gen) / 40
    b = torch.randn(C, device=DEV, generator=gen)
    graph_conv_infer(X, g, W, b, True)
    grl.check()
    grl_option("ws_spin", 1)
    reports = 0
    for delay in (0, 2_000_000, 20_000_000):  # the poison lands before, during, after the checks below
        side = torch.cuda.Stream(DEV)
        side.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(side):
            if delay:
                torch.cuda._sleep(delay)
            out = graph_conv_infer(X, g, W, b, True)
        for _ in range(50):
            try:
                grl.check()
            except _lib.GrlError:
                reports += 1
        side.synchronize()
        try:
            grl.check()
        except _lib.GrlError:
            reports += 1
        assert bool(torch.isnan(out).all())
    assert reports == 3  # one per poisoned call
    grl_option("ws_spin", 0)
    grl.check()


def test_bench_surfaces_a_poisoned_timed_region(monkeypatch, grl_option):
    """bench.py checks after every timed region (bench.surface): a poisoned
    run exits non-zero naming the section and the entry point instead of
    being reported as a timing."""
    import bench

    N, L, F, C = 20_011, 6, 256, 256
    g = TypedGraph.synthetic(N, 16.0, L, seed=3, device=DEV)
    X = torch.randn(N, F, device=DEV)
    W = torch.randn(7 * F, C, device=DEV) / 40
    bench.surface("clean", DEV)
    grl_option("ws_spin", 1)
    graph_conv_infer(X, g, W, None, True)
    with pytest.raises(SystemExit, match=r"bench.py: extras \(layers\): .*grl_graphconv_fwd"):
        bench.surface("extras (layers)", DEV)
    grl_option("ws_spin", 0)
    bench.surface("clean again", DEV)


@pytest.mark.parametrize("N,F,C,p,cuts", [(40_000, 256, 256, 0.3, (0, 17_500, 25_000, 40_000)),
                                          (20_000, 512, 256, 0.3, (0, 9999, 20_000)),
                                          (3000, 64, 64, 0.0, (0, 1000, 1001, 3000))])
def test_row_views_forward_equals_whole_graph(N, F, C, p, cuts):
    """TypedGraph.rows_view (GrlTypedCsr.self_row0: the sharded inference's
    row blocks, grl.dist ShardedGraph._graphconv_streamed): the aggregation of
    a row range is bitwise the whole graph's rows, DropEdge included; the
    GraphConv forward over a row range equals the whole-graph call bitwise
    when both take the split-bf16 GEMM (ops.x6_rows_ok: a 17.5k-row view of
    the F = 256 layer, both 10k-row halves at F = 512 -- the one-kernel form
    with self_row0) and within 1e-5 otherwise (the fp32 linear picks its
    split-K by row count)."""
    g = TypedGraph.synthetic(N, 12.0, 6, kind="er", seed=3, device=DEV)
    gd = g.with_dropedge(DropEdge(p=p, seed=9, call=2) if p else None)
    gen = torch.Generator().manual_seed(N + F)
    X = torch.randn(N, F, generator=gen).to(DEV)
    W = (torch.randn(7 * F, C, generator=gen) * 0.05).to(DEV)
    b = torch.randn(C, generator=gen).to(DEV)
    Z = typed_aggregate(X, gd)
    whole = graph_conv_infer(X, gd, W, b, relu=True)
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        v = gd.rows_view(r0, r1)
        assert v.num_rows == r1 - r0 and v.self_row0 == r0 and (r0 == 0 or not v.transpose_ok)
        assert torch.equal(typed_aggregate(X, v), Z[r0:r1])
        part = graph_conv_infer(X, v, W, b, relu=True)
        if x6_rows_ok(r1 - r0, C, 7 * F) and x6_rows_ok(N, C, 7 * F):
            assert torch.equal(part, whole[r0:r1])
        else:
            assert float((part - whole[r0:r1]).abs().max()) <= 1e-5 * max(1.0, float(whole.abs().max()))
    with pytest.raises(_lib.GrlError):
        gd.rows_view(5, 10).typed_transpose()
