"""GPU parity: every libgrl kernel against the CPU oracle on identical inputs.

The aggregation kernels sum each row in CSR order with one fmaf per edge,
exactly like oracle/grl_oracle.c, so forward and backward are required to be
BITWISE equal to the oracle (integer/index work: bitwise as well).  The fp32
MFMA linear is checked against float64 numpy at 1e-5 relative (north_star
tolerance is 1e-4) and bitwise on exact integer data (fragment-layout check).
"""
import numpy as np
import pytest
import torch

from grl import DropEdge, TypedGraph, _lib
from grl.graph import current_stream_handle
from grl.ops import linear_fwd, typed_aggregate
from oracle import c_oracle
from oracle import hash as ohash

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def host_graph(N, L, deg, seed, hub=0, vals=False, empty_rows=True):
    """ER typed CSR (oracle generator) + optional hub row with `hub` extra
    edges spread over types, + optional float values."""
    rowptr, colidx = ohash.synth_csr(0, L, N, int(N * deg), seed)
    if hub:
        rng = np.random.default_rng(seed + 1)
        rows = [colidx[rowptr[s]:rowptr[s + 1]] for s in range(N * L)]
        for t in range(L):
            extra = rng.integers(0, N, size=hub // L + 1)
            rows[t] = np.unique(np.concatenate([rows[t], extra])).astype(np.int32)
        colidx = np.concatenate(rows).astype(np.int32)
        rowptr = np.concatenate([[0], np.cumsum([r.size for r in rows])]).astype(np.int32)
    v = np.random.default_rng(seed + 2).uniform(0.1, 2.0, colidx.size).astype(np.float32) if vals else None
    return rowptr, colidx, v


def to_dev(a, dtype=None):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV) if dtype is None else torch.as_tensor(
        a, dtype=dtype).to(DEV)


def assert_bitwise(gpu, ref, what):
    gpu = np.asarray(gpu)
    if not np.array_equal(gpu, ref):
        d = np.abs(gpu.astype(np.float64) - ref.astype(np.float64))
        raise AssertionError(f"{what}: not bitwise equal, max|d|={d.max():.3e} at {np.unravel_index(d.argmax(), d.shape)}")


CASES = [
    # N, L, deg, F, hub, vals, has_self
    (300, 6, 16.0, 256, 0, False, True),
    (300, 6, 16.0, 512, 0, True, True),
    (257, 6, 4.0, 16, 0, False, True),
    (129, 6, 8.0, 10, 0, True, True),     # F % 4 != 0 -> scalar-lane path
    (200, 3, 12.0, 100, 0, False, False),  # VEC=1, NV=2; no identity block
    (90, 6, 6.0, 1000, 0, False, True),    # 2 column blocks of 512
    (500, 6, 2.0, 256, 700, False, True),  # hub row: > 64 edges in one segment
    (64, 7, 0.0, 64, 0, False, True),      # no edges at all
]
DROPS = [None, DropEdge(0.3, 7, 1, True), DropEdge(0.2, 99, 4, False), DropEdge(1.0, 5, 0, True)]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("di", range(len(DROPS)))
def test_spmm_fwd_bwd_bitwise(case, di):
    N, L, deg, F, hub, vals, hs = case
    de = DROPS[di]
    rowptr, colidx, v = host_graph(N, L, deg, 1000 + N, hub, vals)
    X = np.random.default_rng(N + F).standard_normal((N, F)).astype(np.float32)
    ebase, sbase = 1234, 10 ** 9 + 7
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV, vals=v, has_self=hs, edge_id_base=ebase,
                                 self_id_base=sbase).with_dropedge(de)
    Xt = to_dev(X).requires_grad_(True)
    Z = typed_aggregate(Xt, g)
    d = None if de is None else c_oracle.drop(de.p, de.seed, de.call, de.drop_self)
    Zref = c_oracle.spmm_fwd(rowptr, colidx, X, L, hs, vals=v, d=d, edge_base=ebase, self_base=sbase)
    assert_bitwise(Z.detach().cpu().numpy(), Zref, "forward")
    dZ = np.random.default_rng(N + F + 1).standard_normal(Zref.shape).astype(np.float32)
    Z.backward(to_dev(dZ))
    colptr, zrow, eid, cvals = c_oracle.csr_to_csc(rowptr, colidx, L, N, hs, v)
    dXref = c_oracle.spmm_bwd(colptr, zrow, eid, dZ, L, F, N, hs, cvals, d=d, edge_base=ebase, self_base=sbase)
    assert_bitwise(Xt.grad.cpu().numpy(), dXref, "backward")


def test_spmm_strided_input_rows():
    """X given as a column slice (ldx > F), as torch.cat views produce."""
    N, L, F = 150, 6, 128
    rowptr, colidx, _ = host_graph(N, L, 10.0, 5)
    big = np.random.default_rng(0).standard_normal((N, 3 * F)).astype(np.float32)
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV)
    Z = typed_aggregate(to_dev(big)[:, F:2 * F], g)
    Zref = c_oracle.spmm_fwd(rowptr, colidx, big[:, F:2 * F].copy(), L, True)
    assert_bitwise(Z.cpu().numpy(), Zref, "strided forward")


@pytest.mark.parametrize("N,deg,hub", [(1500, 9.0, 300),  # > 8192 edges: the radix-sort transpose
                                       (120, 3.0, 40),     # a page
                                       (64, 0.0, 0),       # no edges at all
                                       (8192, 1.0, 0)])    # 8192 columns and edges
def test_csc_matches_oracle(N, deg, hub):
    L = 6
    rowptr, colidx, v = host_graph(N, L, deg, 77, hub=hub, vals=True)
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV, vals=v)
    c = g.csc()
    colptr, zrow, eid, cvals = c_oracle.csr_to_csc(rowptr, colidx, L, N, True, v)
    np.testing.assert_array_equal(c["colptr"].cpu().numpy(), colptr)
    np.testing.assert_array_equal(c["zrow"].cpu().numpy()[:colidx.size], zrow)
    np.testing.assert_array_equal(c["eid"].cpu().numpy()[:colidx.size], eid)
    np.testing.assert_array_equal(c["cvals"].cpu().numpy()[:colidx.size], cvals)


@pytest.mark.parametrize("layout", ["bnln", "bnnl", "pre"])
@pytest.mark.parametrize("float_vals", [False, True])
@pytest.mark.parametrize("B,N", [(3, 37), (4, 400)])  # a page and > 8191 row segments
def test_dense_to_csr_matches_oracle(layout, float_vals, B, N):
    import inputs as gi

    L = 6
    A = gi.random_adj_bnln(4, B, N, L, 5.0, float_vals=float_vals)
    if layout == "bnln":
        At = to_dev(A)
        rp, ci, va = c_oracle.dense_to_csr(A, [N * L * N, L * N, N, 1], B, N, L)
        Lx = L
    elif layout == "bnnl":
        At = to_dev(A).permute(0, 1, 3, 2)  # non-contiguous view, as GraphConv receives it
        rp, ci, va = c_oracle.dense_to_csr(A, [N * L * N, L * N, N, 1], B, N, L)
        Lx = L
    else:
        from oracle import dense_ref
        pre = dense_ref.preprocess_adj(np.transpose(A, (0, 1, 3, 2))).astype(np.float32)
        At = to_dev(pre)
        Lx = L + 1
        rp, ci, va = c_oracle.dense_to_csr(pre.reshape(B, N, Lx, N), [N * Lx * N, Lx * N, N, 1], B, N, Lx)
    g = TypedGraph.from_dense(At, layout=layout)
    assert g.num_types == Lx and g.has_self == (layout != "pre")
    np.testing.assert_array_equal(g.rowptr.cpu().numpy(), rp)
    np.testing.assert_array_equal(g.colidx.cpu().numpy(), ci)
    if float_vals:
        np.testing.assert_array_equal(g.vals.cpu().numpy(), va)
    else:
        assert g.vals is None


@pytest.mark.parametrize("kind,N,deg,rng_", [(0, 5000, 16.0, None), (0, 3001, 7.0, (1000, 2500)),
                                             (1, 1 << 13, 12.0, None), (1, 1 << 12, 20.0, (100, 3000))])
def test_synth_matches_oracle(kind, N, deg, rng_):
    rb, re = (0, N) if rng_ is None else rng_
    g = TypedGraph.synthetic(N, deg, 6, kind=["er", "rmat"][kind], seed=11, row_range=rng_, device=DEV)
    rp, ci = ohash.synth_csr(kind, 6, N, int(round(N * deg)), 11, rb, re)
    np.testing.assert_array_equal(g.rowptr.cpu().numpy(), rp)
    np.testing.assert_array_equal(g.colidx.cpu().numpy(), ci)


@pytest.mark.parametrize("p", [0.0, 0.2, 0.3, 1.0])
def test_dropedge_mask_matches_oracle(p):
    g = TypedGraph.from_csr_host(np.zeros(7, np.int32), np.zeros(0, np.int32), 6, DEV)
    de = DropEdge(p, 31337, 2)
    keep = g.dropedge_mask(de, 2**33 + 5, 100_000).cpu().numpy()
    ref = ohash.dropedge_keep(p, 31337, 2, np.arange(2**33 + 5, 2**33 + 5 + 100_000, dtype=np.uint64))
    np.testing.assert_array_equal(keep.astype(bool), ref)


@pytest.mark.parametrize("M,K,C", [(1, 8, 4), (74, 1792, 256), (300, 3584, 256), (129, 10, 5), (517, 36, 200),
                                   (1000, 1792, 128),
                                   # one pass (>= 256 output tiles) on 64-column tiles: aligned, unaligned, 3 tiles
                                   (40_000, 100, 56), (33_000, 64, 30), (20_000, 128, 160)])
@pytest.mark.parametrize("relu,bias", [(False, True), (True, True), (False, False)])
def test_linear_matches_fp64(M, K, C, relu, bias):
    rng = np.random.default_rng(M * 7 + K)
    Z = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((K, C)) / np.sqrt(K)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32) if bias else None
    out = linear_fwd(to_dev(Z), to_dev(W), to_dev(b) if bias else None, relu).cpu().numpy()
    ref = Z.astype(np.float64) @ W.astype(np.float64) + (b if bias else 0.0)
    if relu:
        ref = np.maximum(ref, 0)
    scale = np.abs(Z).astype(np.float64) @ np.abs(W).astype(np.float64) + 1.0
    assert np.all(np.abs(out - ref) <= 1e-5 * scale)


def test_linear_fragment_layout_exact():
    """Exact small-integer data: any row/col/k mapping error shows up bitwise.
    B is asymmetric (guide: 'A=I-check with ASYMMETRIC B')."""
    M, K, C = 160, 64, 136
    I = np.zeros((M, K), np.float32)
    I[np.arange(M), np.arange(M) % K] = 1.0
    Wt = (np.arange(K * C).reshape(K, C) % 97 - 48).astype(np.float32)
    out = linear_fwd(to_dev(I), to_dev(Wt), None, False).cpu().numpy()
    np.testing.assert_array_equal(out, I @ Wt)
    rng = np.random.default_rng(1)
    Zi = rng.integers(-8, 9, (M, K)).astype(np.float32)
    Wi = rng.integers(-8, 9, (K, C)).astype(np.float32)
    bi = rng.integers(-8, 9, C).astype(np.float32)
    out = linear_fwd(to_dev(Zi), to_dev(Wi), to_dev(bi), False).cpu().numpy()
    np.testing.assert_array_equal(out, Zi @ Wi + bi)
    # the one-pass form (>= 256 output tiles) on 64-column tiles (136 = 128 + 8) and on 128-column ones
    for Mb, Cb in ((33_000, 136), (33_000, 128)):
        Zb = rng.integers(-8, 9, (Mb, K)).astype(np.float32)
        Wb = rng.integers(-8, 9, (K, Cb)).astype(np.float32)
        out = linear_fwd(to_dev(Zb), to_dev(Wb), None, False).cpu().numpy()
        np.testing.assert_array_equal(out, Zb @ Wb)


def test_errors_raise_not_fallback():
    g = TypedGraph.from_csr_host(np.zeros(13, np.int32), np.zeros(0, np.int32), 6, DEV)
    with pytest.raises(_lib.GrlError, match="rows"):
        typed_aggregate(torch.zeros(3, 8, device=DEV), g)
    with pytest.raises(_lib.GrlError, match="float32"):
        typed_aggregate(torch.zeros(2, 8, device=DEV, dtype=torch.float16), g)
    assert current_stream_handle(DEV) is not None


SPLITS = [(64, 24), (300, 128), (2048, 1024)]


@pytest.mark.parametrize("split", SPLITS)
@pytest.mark.parametrize("di", [0, 1])
@pytest.mark.parametrize("F,vals", [(256, False), (512, True), (10, False)])
def test_split_rows_bitwise_rmat(split, di, F, vals):
    """Power-law (R-MAT) graph: rows/columns heavier than the threshold are
    summed in chunks by separate wavefronts + an ordered fixup; must equal the
    oracle restating that chunk order bitwise, forward and backward."""
    N, L = 1 << 12, 6
    rowptr, colidx = ohash.synth_csr(1, L, N, N * 40, 21)
    deg = np.diff(rowptr[::L])
    assert deg.max() > split[0] or split[0] == 2048  # the small thresholds really split rows
    v = np.random.default_rng(3).uniform(0.1, 2.0, colidx.size).astype(np.float32) if vals else None
    de = [None, DropEdge(0.3, 7, 1, True)][di]
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV, vals=v).with_dropedge(de)
    g.split_threshold, g.split_chunk = split
    X = np.random.default_rng(F).standard_normal((N, F)).astype(np.float32)
    Xt = to_dev(X).requires_grad_(True)
    Z = typed_aggregate(Xt, g)
    d = None if de is None else c_oracle.drop(de.p, de.seed, de.call, de.drop_self)
    Zref = c_oracle.spmm_fwd(rowptr, colidx, X, L, True, vals=v, d=d, split=split)
    assert_bitwise(Z.detach().cpu().numpy(), Zref, "forward (split)")
    dZ = np.random.default_rng(F + 1).standard_normal(Zref.shape).astype(np.float32)
    Z.backward(to_dev(dZ))
    colptr, zrow, eid, cvals = c_oracle.csr_to_csc(rowptr, colidx, L, N, True, v)
    dXref = c_oracle.spmm_bwd(colptr, zrow, eid, dZ, L, F, N, True, cvals, d=d, self_base=int(rowptr[-1]),
                              split=split)
    assert_bitwise(Xt.grad.cpu().numpy(), dXref, "backward (split)")
    st = g.split_stats()
    if split[0] < 300:
        assert st["csr"]["heavy_segments"] > 0 and st["csc"]["heavy_segments"] > 0
    # and within fp32 tolerance of the unsplit summation order
    Zplain = c_oracle.spmm_fwd(rowptr, colidx, X, L, True, vals=v, d=d)
    assert np.allclose(Zref, Zplain, rtol=1e-5, atol=1e-4)


def test_split_plan_matches_definition():
    N, L = 1 << 11, 6
    rowptr, colidx = ohash.synth_csr(1, L, N, N * 30, 4)
    g = TypedGraph.from_csr_host(rowptr, colidx, L, DEV)
    g.split_threshold, g.split_chunk = 100, 40
    g._split("csr", 8)
    sp = g._shared["split_csr"]
    heavy_rows = np.nonzero(np.diff(rowptr[::L]) > 100)[0]
    exp_seg = (heavy_rows[:, None] * L + np.arange(L)[None]).ravel()
    np.testing.assert_array_equal(sp["tensors"]["heavy_seg"].cpu().numpy()[:exp_seg.size], exp_seg)
    begins, ends, cptr = [], [], [0]
    for s in exp_seg:
        for e in range(rowptr[s], rowptr[s + 1], 40):
            begins.append(e)
            ends.append(min(e + 40, rowptr[s + 1]))
        cptr.append(len(begins))
    assert sp["plan"].num_chunks == len(begins)
    np.testing.assert_array_equal(sp["tensors"]["chunk_begin"].cpu().numpy()[:len(begins)], begins)
    np.testing.assert_array_equal(sp["tensors"]["chunk_end"].cpu().numpy()[:len(ends)], ends)
    np.testing.assert_array_equal(sp["tensors"]["heavy_cptr"].cpu().numpy()[:len(cptr)], cptr)


@pytest.mark.parametrize("kind,N", [(0, 3000), (1, 1 << 12)])
def test_synth_degrees_match_oracle(kind, N):
    deg = TypedGraph.synthetic_degrees(N, 11.0, 6, kind=["er", "rmat"][kind], seed=5, device=DEV).cpu().numpy()
    src, _, _ = ohash.synth_edges(kind, 6, N, int(round(N * 11.0)), 5)
    np.testing.assert_array_equal(deg, np.bincount(src, minlength=N))


@pytest.mark.parametrize("M,K,C", [(1, 8, 4), (74, 1792, 256), (3000, 3584, 256), (129, 10, 5), (517, 36, 200),
                                   (70000, 1792, 128)])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_backward_matches_fp64(M, K, C, relu):
    from grl.ops import linear_bwd_data, linear_bwd_weight

    rng = np.random.default_rng(M + K + C)
    Z = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((K, C)) / np.sqrt(K)).astype(np.float32)
    g = rng.standard_normal((M, C)).astype(np.float32)
    out = rng.standard_normal((M, C)).astype(np.float32) if relu else None
    gm = g.astype(np.float64) * ((out > 0) if relu else 1.0)
    dZ = linear_bwd_data(to_dev(g), to_dev(out) if relu else None, to_dev(W)).cpu().numpy()
    ref = gm @ W.T.astype(np.float64)
    scale = np.abs(gm) @ np.abs(W.T).astype(np.float64) + 1.0
    assert np.all(np.abs(dZ - ref) <= 1e-5 * scale)
    dW, db = linear_bwd_weight(to_dev(Z), to_dev(g), to_dev(out) if relu else None, True)
    refW = Z.T.astype(np.float64) @ gm
    scaleW = np.abs(Z.T).astype(np.float64) @ np.abs(gm) + 1.0
    assert np.all(np.abs(dW.cpu().numpy() - refW) <= 1e-5 * scaleW)
    np.testing.assert_allclose(db.cpu().numpy(), gm.sum(0), rtol=1e-5, atol=1e-4 * np.sqrt(M))


@pytest.mark.parametrize("M,C", [(65536, 256), (100003, 200), (70000, 7)])
def test_relu_grad_one_pass(M, C):
    """grl_relu_grad (the layer backward's ReLU mask + db, M >= PREMASK_ROWS):
    g_eff bitwise torch.where(out > 0, g, 0) (NaN outputs masked, -0.0 / NaN
    gradients passed), db bitwise linear_bwd_weight's db on g_eff."""
    from grl.ops import PREMASK_ROWS, linear_bwd_weight, relu_grad

    assert M >= PREMASK_ROWS
    rng = np.random.default_rng(M + C)
    g = rng.standard_normal((M, C)).astype(np.float32)
    out = rng.standard_normal((M, C)).astype(np.float32)
    out[::97, 0] = np.nan
    out[1::89, -1] = 0.0
    g[2::101, 0] = -0.0
    g[3::103, -1] = np.nan
    gd, od = to_dev(g), to_dev(out)
    g_eff, mask, db = relu_grad(gd, od, True)
    assert mask is None
    ref = torch.where(od > 0, gd, torch.zeros((), device=gd.device))
    assert torch.equal(g_eff.view(torch.int32), ref.view(torch.int32))
    Z = to_dev(rng.standard_normal((M, 8)).astype(np.float32))
    _, db_gemm = linear_bwd_weight(Z, ref, None, True)
    assert torch.equal(db.view(torch.int32), db_gemm.view(torch.int32))
    g2, _, none = relu_grad(gd, od, False)
    assert none is None and torch.equal(g2.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(gd.cpu().view(torch.int32), torch.from_numpy(g).view(torch.int32))  # g untouched


def test_linear_backward_deterministic():
    from grl.ops import linear_bwd_weight

    rng = np.random.default_rng(0)
    Z = to_dev(rng.standard_normal((50000, 1792)).astype(np.float32))
    g = to_dev(rng.standard_normal((50000, 256)).astype(np.float32))
    a = linear_bwd_weight(Z, g, g, True)
    b = linear_bwd_weight(Z, g, g, True)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.parametrize("M,K,C", [(74, 1792, 256), (296, 3584, 256), (517, 36, 200)])
def test_small_m_split_k_deterministic(M, K, C):
    """Small graphs split K over workgroups (fp32 slabs, ordered reduce):
    repeated calls are bitwise identical, forward and data gradient, and a
    strided Z (ldz > K) reads the same values."""
    from grl import _lib
    from grl.ops import linear_bwd_data

    assert _lib.lib().grl_linear_fwd_workspace_size(M, K, C) > 0  # the split path is what runs
    # large M takes the x6 path: only W's bf16 planes (3 x 256-padded C x K); off the x6 shape the fp32
    # GEMM in one pass (the call fills the chip: no slabs)
    big = _lib.lib().grl_linear_fwd_workspace_size(1_000_000, K, C)
    if K % 16 == 0:
        assert big == 3 * (-(-C // 256) * 256) * K * 2 + 256
    else:
        assert big == 0
    # below the x6 size and the one-pass tile count: the chunk slabs, in row blocks of at most 256 MB
    mid = _lib.lib().grl_linear_fwd_workspace_size(20_000, 1280, 16)
    assert 0 < mid <= (256 << 20) + 256
    rng = np.random.default_rng(M)
    Zw = to_dev(rng.standard_normal((M, K + 8)).astype(np.float32))
    Z = Zw[:, :K]
    W = to_dev((rng.standard_normal((K, C)) / np.sqrt(K)).astype(np.float32))
    b = to_dev(rng.standard_normal(C).astype(np.float32))
    a1 = linear_fwd(Z, W, b, True)
    a2 = linear_fwd(Z, W, b, True)
    a3 = linear_fwd(Z.contiguous(), W, b, True)
    assert torch.equal(a1, a2) and torch.equal(a1, a3)
    g = to_dev(rng.standard_normal((M, C)).astype(np.float32))
    d1 = linear_bwd_data(g, a1, W)
    d2 = linear_bwd_data(g, a1, W)
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("x6", ["1", "0"])
@pytest.mark.parametrize("M,K,C", [(300_000, 1792, 256), (70_003, 3584, 256), (131_072, 512, 128), (65_600, 256, 1792),
                                   (45_001, 1792, 200)])
def test_large_tile_gemms_match_fp64(M, K, C, x6, monkeypatch, grl_option):
    """Shapes that take the large-M paths (>= 16 GFLOP, aligned, K % 16 == 0):
    x6 = "1" the split-bf16 kernel (gemm_x6_kernel), "0" the fp32 256x256
    LDS-DMA tile (gemm256p_kernel).  Forward with bias+ReLU, dZ and dW/db
    (pre-masked g) against float64 on sampled rows / the full dW; ragged M
    tails and a C that is not a multiple of the 256-column tile included."""
    from grl.ops import linear_bwd_data, linear_bwd_weight

    grl_option("gemm_x6", int(x6))

    gen = torch.Generator(device=DEV).manual_seed(M % 1000)
    Z = torch.randn(M, K, device=DEV, generator=gen)
    W = torch.randn(K, C, device=DEV, generator=gen) / np.sqrt(K)
    b = torch.randn(C, device=DEV, generator=gen)
    out = linear_fwd(Z, W, b, True)
    rows = torch.randint(0, M, (512,), device=DEV, generator=gen)
    rows[0], rows[1] = 0, M - 1
    ref = torch.relu(Z[rows].double() @ W.double() + b.double())
    scale = Z[rows].double().abs() @ W.double().abs() + 1.0
    assert ((out[rows].double() - ref).abs() <= 1e-5 * scale).all()
    g = torch.randn(M, C, device=DEV, generator=gen) * (out > 0)
    dZ = linear_bwd_data(g, None, W)
    refz = g[rows].double() @ W.double().T
    scz = g[rows].double().abs() @ W.double().abs().T + 1.0
    assert ((dZ[rows].double() - refz).abs() <= 1e-5 * scz).all()
    dW, db = linear_bwd_weight(Z, g, None, True)
    refw = Z.double().T @ g.double()
    scw = Z.double().abs().T @ g.double().abs() + 1.0
    assert ((dW.double() - refw).abs() <= 1e-5 * scw).all()
    torch.testing.assert_close(db.double(), g.double().sum(0), rtol=1e-5, atol=1e-3)
    assert torch.equal(linear_fwd(Z, W, b, True), out)  # deterministic


def test_x6_split_is_exact_on_wide_dynamic_range(monkeypatch, grl_option):
    """The x6 GEMM splits every fp32 value into three bf16 parts exactly: rows
    of Z scaled over 2^-60 .. 2^60 and W columns over 2^-30 .. 2^30 keep the
    per-element error at the fp32 level (<= 1e-6 of sum |terms|), the same
    bound the fp32-MFMA kernel meets; integer data is exact."""
    from grl.ops import linear_bwd_data

    grl_option("gemm_x6", 1)
    M, K, C = 40_000, 1792, 256
    gen = torch.Generator(device=DEV).manual_seed(7)
    rs = torch.pow(2.0, torch.randint(-60, 61, (M, 1), device=DEV, generator=gen).float())
    cs = torch.pow(2.0, torch.randint(-30, 31, (1, C), device=DEV, generator=gen).float())
    Z = torch.randn(M, K, device=DEV, generator=gen) * rs
    W = torch.randn(K, C, device=DEV, generator=gen) * cs
    out = linear_fwd(Z, W, None, False)
    rows = torch.randint(0, M, (1024,), device=DEV, generator=gen)
    ref = Z[rows].double() @ W.double()
    scale = Z[rows].double().abs() @ W.double().abs()
    assert ((out[rows].double() - ref).abs() <= 1e-6 * scale).all()
    Zi = torch.randint(-64, 65, (M, K), device=DEV, generator=gen).float()
    Wi = torch.randint(-64, 65, (K, C), device=DEV, generator=gen).float()
    assert torch.equal(linear_fwd(Zi, Wi, None, False), (Zi.double() @ Wi.double()).float())
    gi = torch.randint(-64, 65, (M, C), device=DEV, generator=gen).float()
    assert torch.equal(linear_bwd_data(gi, None, Wi), (gi.double() @ Wi.double().T).float())


@pytest.mark.parametrize("wide", ["1", "0"])
def test_spmm_wide_rows_bitwise(wide, monkeypatch, grl_option):
    """F in (256, 512]: one wave per whole row (spmm_wide = 1, the choice for
    gathered tables above 12 GB) or 256-column waves along grid.y ("0"); both
    bitwise equal to the oracle, forward and backward, with DropEdge, float
    edge values and split heavy rows."""
    grl_option("spmm_wide", int(wide))
    test_spmm_fwd_bwd_bitwise((300, 6, 16.0, 512, 0, True, True), 1)
    test_spmm_fwd_bwd_bitwise((200, 6, 8.0, 384, 0, False, True), 2)
    test_split_rows_bitwise_rmat((300, 128), 1, 512, True)


def test_x6_strided_z_matches_contiguous(monkeypatch, grl_option):
    """The x6 forward reads Z through its row stride (ldz > K, as a column
    slice of a wider buffer gives): bitwise the same as on a contiguous copy."""
    grl_option("gemm_x6", 1)
    M, K, C = 40_000, 1792, 256
    gen = torch.Generator(device=DEV).manual_seed(11)
    big = torch.randn(M, K + 32, device=DEV, generator=gen)
    Z = big[:, 16:16 + K]
    W = torch.randn(K, C, device=DEV, generator=gen) / np.sqrt(K)
    b = torch.randn(C, device=DEV, generator=gen)
    assert Z.stride(0) == K + 32
    assert torch.equal(linear_fwd(Z, W, b, True), linear_fwd(Z.contiguous(), W, b, True))
