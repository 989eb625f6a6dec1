"""CPU-only: pin the oracle against the reference's own outputs
(tests/golden/*.npz from make_golden.py) and check the oracle's C and numpy
halves against each other.  No GPU, no libgrl compute calls."""
import numpy as np
import pytest

import inputs as gi
from oracle import c_oracle, dense_ref
from oracle import hash as ohash


def _close(a, b, tol):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(1.0, float(np.abs(b).max()) if b.size else 1.0)
    err = float(np.abs(a - b).max()) if a.size else 0.0
    assert err <= tol * scale, f"max|d|={err:.3e} > {tol:.0e} * {scale:.3g}"


def _case_inputs(name, g):
    seed, B, N, L, F, C, fv, epn = gi.GRAPHCONV_CASES[name]
    A = gi.random_adj_bnln(seed, B, N, L, epn, float_vals=fv)
    V = gi.features(seed + 1, B, N, F)
    W, b = gi.graphconv_params(seed + 2, F, C, L)
    dout = gi.features(seed + 3, B, N, C)
    if "A" in g:  # small fixtures also carry the inputs: check regeneration
        np.testing.assert_array_equal(A, g["A"])
        np.testing.assert_array_equal(V, g["V"])
        np.testing.assert_array_equal(W, g["W"])
    return seed, A, V, W, b, dout


@pytest.mark.parametrize("name", list(gi.GRAPHCONV_CASES))
@pytest.mark.parametrize("tag", ["eval", "drop"])
def test_dense_oracle_matches_reference_graphconv(golden, name, tag):
    """oracle/dense_ref.py == reference GraphConv fwd+bwd (robust_gcn.py:32-72)."""
    g = golden(f"graphconv_{name}.npz")
    seed, A, V, W, b, dout = _case_inputs(name, g)
    A_pre = dense_ref.preprocess_adj(np.transpose(A, (0, 1, 3, 2)).astype(np.float64))
    if tag == "drop":
        de = gi.DROPEDGE
        mult = dense_ref.dropedge_weights_pre(A, de["p"], de["seed"], de["call"])
        A_pre = dense_ref.apply_dropedge(A_pre, mult).astype(np.float64)
    out, Z = dense_ref.graphconv_forward(V.astype(np.float64), A_pre, W.astype(np.float64), b.astype(np.float64))
    dV, dW, db = dense_ref.graphconv_backward(V.astype(np.float64), A_pre, W.astype(np.float64), Z,
                                              dout.astype(np.float64))
    _close(out, g[f"{tag}_out"], 1e-5)
    _close(dV, g[f"{tag}_dV"], 1e-5)
    _close(db, g[f"{tag}_db"], 1e-5)
    _close(dW @ gi.probes(seed + 4, dW.shape[1]).astype(np.float64), g[f"{tag}_dW_probe"], 1e-5)
    if f"{tag}_dW" in g:
        _close(dW, g[f"{tag}_dW"], 1e-5)


@pytest.mark.parametrize("name", list(gi.GRAPHCONV_CASES))
@pytest.mark.parametrize("tag", ["eval", "drop"])
def test_csr_oracle_matches_reference_graphconv(golden, name, tag):
    """Typed-CSR restatement (grl_oracle.c) + linear == reference GraphConv."""
    g = golden(f"graphconv_{name}.npz")
    seed, A, V, W, b, dout = _case_inputs(name, g)
    B, N, L, _ = A.shape
    F = V.shape[-1]
    rowptr, colidx, vals = c_oracle.dense_to_csr(A, [N * L * N, L * N, N, 1], B, N, L)
    d = None
    if tag == "drop":
        de = gi.DROPEDGE
        d = c_oracle.drop(de["p"], de["seed"], de["call"], True)
    Z = c_oracle.spmm_fwd(rowptr, colidx, V.reshape(B * N, F), L, True, vals=vals, d=d)
    out = Z.astype(np.float64) @ W.astype(np.float64) + b
    _close(out.reshape(g[f"{tag}_out"].shape), g[f"{tag}_out"], 1e-5)
    # backward: dZ = dout W^T, dV = A_drop^T dZ through the CSC
    dZ = (dout.reshape(B * N, -1).astype(np.float64) @ W.T.astype(np.float64)).astype(np.float32)
    colptr, zrow, eid, cvals = c_oracle.csr_to_csc(rowptr, colidx, L, B * N, True, vals)
    dV = c_oracle.spmm_bwd(colptr, zrow, eid, dZ, L, F, B * N, True, cvals, d=d, self_base=int(rowptr[-1]))
    _close(dV.reshape(g[f"{tag}_dV"].shape), g[f"{tag}_dV"], 1e-5)


def test_dense_to_csr_orders_and_values():
    A = gi.random_adj_bnln(5, 3, 11, 4, 5.0, float_vals=True)
    B, N, L, _ = A.shape
    rowptr, colidx, vals = c_oracle.dense_to_csr(A, [N * L * N, L * N, N, 1], B, N, L)
    b, n, t, m = np.nonzero(A)  # C order == (b, n, t, m) ascending
    np.testing.assert_array_equal(colidx, (b * N + m).astype(np.int32))
    np.testing.assert_array_equal(vals, A[b, n, t, m])
    seg = (b * N + n) * L + t
    np.testing.assert_array_equal(rowptr, np.searchsorted(seg, np.arange(B * N * L + 1)).astype(np.int32))
    # the permuted (B,N,N,L) view addresses the same operator
    Ap = np.ascontiguousarray(np.transpose(A, (0, 1, 3, 2)))
    r2, c2, v2 = c_oracle.dense_to_csr(Ap, [N * N * L, N * L, 1, L], B, N, L)
    np.testing.assert_array_equal(r2, rowptr)
    np.testing.assert_array_equal(c2, colidx)


def test_csr_to_csc_is_stable_transpose():
    rng = np.random.default_rng(3)
    N, L = 50, 6
    A = gi.random_adj_bnln(9, 1, N, L, 8.0)
    rowptr, colidx, _ = c_oracle.dense_to_csr(A, [N * L * N, L * N, N, 1], 1, N, L)
    colptr, zrow, eid, _ = c_oracle.csr_to_csc(rowptr, colidx, L, N, True)
    order = np.argsort(colidx, kind="stable")
    np.testing.assert_array_equal(eid, order.astype(np.int32))
    seg = np.searchsorted(rowptr, np.arange(colidx.size), side="right") - 1
    np.testing.assert_array_equal(zrow, ((seg // L) * (L + 1) + 1 + seg % L)[order].astype(np.int32))
    np.testing.assert_array_equal(colptr, np.searchsorted(colidx[order], np.arange(N + 1)).astype(np.int32))
    del rng


def test_hash_numpy_equals_c():
    ids = np.concatenate([np.arange(5000, dtype=np.uint64), np.array([2**32 - 1, 2**32, 2**63 + 5], np.uint64)])
    for seed, call in [(0, 0), (7, 3), (2**63 + 11, 2**40)]:
        key = ohash.dropedge_key(seed, call)
        assert key == c_oracle.lib().oracle_dropedge_key(seed, call)
        bits = ohash.dropedge_bits(key, ids)
        cb = np.array([c_oracle.lib().oracle_dropedge_bits(key, int(i)) for i in ids[:200]], dtype=np.uint32)
        np.testing.assert_array_equal(bits[:200], cb)
    for p in (0.0, 0.2, 0.3, 0.5, 1.0):
        d = c_oracle.drop(p, 99, 1)
        keep_c = c_oracle.dropedge_mask(d, 1000, 20000).astype(bool)
        np.testing.assert_array_equal(keep_c, ohash.dropedge_keep(p, 99, 1, np.arange(1000, 21000)))
        act, thr, scale = ohash.dropedge_params(p)
        assert (d.active, d.threshold) == (int(act), thr) and np.float32(d.scale) == scale


@pytest.mark.parametrize("p", [0.2, 0.3, 0.5])
def test_dropedge_keep_rate(p):
    keep = ohash.dropedge_keep(p, 1234, 0, np.arange(2_000_000))
    # Bernoulli(1-p): 6 sigma band
    sigma = np.sqrt(p * (1 - p) / keep.size)
    assert abs(keep.mean() - (1 - p)) < 6 * sigma
    # independent streams per call: masks of two calls agree ~ p^2 + (1-p)^2
    k2 = ohash.dropedge_keep(p, 1234, 1, np.arange(2_000_000))
    agree = (keep == k2).mean()
    assert abs(agree - (p * p + (1 - p) ** 2)) < 0.005


@pytest.mark.parametrize("kind,N,deg", [(0, 997, 16.0), (0, 4096, 5.0), (1, 1024, 12.0)])
def test_synth_numpy_equals_c(kind, N, deg):
    L, seed = 6, 42
    C = int(round(N * deg))
    r_np, c_np = ohash.synth_csr(kind, L, N, C, seed)
    r_c, c_c, _ = c_oracle.synth(kind, L, N, C, seed)
    np.testing.assert_array_equal(r_np, r_c)
    np.testing.assert_array_equal(c_np, c_c)
    # a node-range shard is exactly the rows of the full graph
    rb, re = N // 3, (2 * N) // 3
    r_s, c_s, _ = c_oracle.synth(kind, L, N, C, seed, rb, re)
    np.testing.assert_array_equal(c_s, c_np[r_np[rb * L]:r_np[re * L]])
    np.testing.assert_array_equal(r_s, r_np[rb * L:re * L + 1] - r_np[rb * L])


def test_rmat_is_skewed():
    N, L = 1 << 12, 6
    r, c = ohash.synth_csr(1, L, N, N * 16, 3)
    deg = np.diff(r[::L])
    assert deg.max() > 20 * max(1.0, np.median(deg))


def test_oracle_model_matches_reference_eval(golden):
    """Full GraphCNNDropEdge(4369,53,6,256) eval logits on debug.json
    (drop_robust_gcn.py:61-103): numpy restatement vs reference output,
    with the reference's init reproduced by torch.manual_seed(0)."""
    import torch

    from gnn.models import GraphCNNDropEdge

    g = golden("model_debug.npz")
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256)
    P = {k: v.detach().double().numpy() for k, v in model.state_dict().items()}
    V = np.zeros(tuple(g["V_shape"]), dtype=np.float32)
    V[g["V_rows"], g["V_cols"]] = g["V_vals"]
    A = np.unpackbits(g["A_bits"])[: int(np.prod(g["A_shape"]))].reshape(tuple(g["A_shape"])).astype(np.float32)
    logits = dense_ref.graph_cnn_dropedge_forward(P, V[None], A[None])[0]
    _close(logits, g["logits"], 1e-5)


def test_torch_fp32_restatement_matches_reference_eval(golden):
    """oracle/dense_torch.py (the fp32 torch-CPU restatement timed as the C1
    CPU baseline) reproduces the reference's eval logits on debug.json, and
    its train step runs (dense Bernoulli masks over A_pre, Adam)."""
    import torch

    from gnn.models import GraphCNNDropEdge
    from oracle import dense_torch

    g = golden("model_debug.npz")
    torch.manual_seed(0)
    model = GraphCNNDropEdge(4369, 53, 6, 256)
    P = {k: v.detach().float() for k, v in model.state_dict().items()}
    V = np.zeros(tuple(g["V_shape"]), dtype=np.float32)
    V[g["V_rows"], g["V_cols"]] = g["V_vals"]
    A = np.unpackbits(g["A_bits"])[: int(np.prod(g["A_shape"]))].reshape(tuple(g["A_shape"])).astype(np.float32)
    with torch.no_grad():
        logits = dense_torch.forward(P, torch.from_numpy(V)[None], torch.from_numpy(A)[None])[0].double().numpy()
    _close(logits, g["logits"], 1e-4)
    step = dense_torch.TrainStep(model.state_dict())
    y = torch.randint(0, 53, (2, V.shape[0]), generator=torch.Generator().manual_seed(1))
    V2, A2 = torch.from_numpy(V)[None].expand(2, -1, -1), torch.from_numpy(A)[None].expand(2, -1, -1, -1)
    l0 = step(V2, A2, y)
    assert np.isfinite(l0)


def test_oracle_model_matches_reference_train_masks(golden):
    g = golden("model_small_train.npz")
    P = {k[len("init::"):]: v.astype(np.float64) for k, v in g.items() if k.startswith("init::")}
    de = gi.DROPEDGE
    mults = [dense_ref.dropedge_weights_pre(g["A"], de["p"], de["seed"], c) for c in range(3)]
    logits = dense_ref.graph_cnn_dropedge_forward(P, g["V"], g["A"], edge_mults=mults)
    _close(logits, g["logits"], 1e-5)


@pytest.mark.parametrize("tag,att", [("att", True), ("noatt", False)])
def test_oracle_model_variants_eval(golden, tag, att):
    """Padded B=2 batch, float (fc_similarity-style) adjacency, with and
    without NodeSelfAtten: numpy restatement vs the reference's logits."""
    g = golden("model_variants.npz")
    P = {k[len(f"{tag}::init::"):]: v.astype(np.float64) for k, v in g.items() if k.startswith(f"{tag}::init::")}
    logits = dense_ref.graph_cnn_dropedge_forward(P, g["V"], g["A"], use_attention=att)
    _close(logits, g[f"{tag}::logits"], 1e-5)


def test_oracle_model_efficient_mode_false(golden):
    """efficient_mode=False: the edge masks hit raw A and the identity is
    never dropped (drop_self=False multipliers)."""
    g = golden("model_variants.npz")
    P = {k[len("effF::init::"):]: v.astype(np.float64) for k, v in g.items() if k.startswith("effF::init::")}
    de = gi.DROPEDGE
    mults = [dense_ref.dropedge_weights_pre(g["effF::A"], de["p"], de["seed"], c, drop_self=False) for c in range(3)]
    logits = dense_ref.graph_cnn_dropedge_forward(P, g["V"], g["effF::A"], edge_mults=mults)
    _close(logits, g["effF::logits"], 1e-5)


def test_oracle_model_matches_reference_procedure_first_loss(golden):
    """procedure_train.npz (the reference KVProcedure's three steps): the
    float64 oracle model, from the fixture's initial weights with the eager
    step's injected DropEdge masks, gives the reference's first-step loss
    (CrossEntropyLoss over the non-ignored nodes, kv_procedure.py:127 /
    cross_entropy_loss.py:23-35) -- the fixture's batches, masks and init are
    consistent with the restated model."""
    g = golden("procedure_train.npz")
    touched = g["emb1_touched_cols"]
    P = {k[len("init::"):]: g[k].astype(np.float64) for k in g.keys() if k.startswith("init::") and "emb1.0.weight" not in k}
    Vs, As = tuple(g["V_shape"]), tuple(g["A_shape"])
    W1 = np.zeros((P["emb1.0.bias"].shape[0], Vs[-1]))
    W1[:, touched] = g["init::emb1.0.weight::touched"]
    P["emb1.0.weight"] = W1  # V is zero on every other column
    V = np.zeros(Vs, dtype=np.float32)
    V[tuple(g["batch0::V_idx"])] = g["batch0::V_vals"]
    A = np.unpackbits(g["batch0::A_bits"])[: int(np.prod(As))].reshape(As).astype(np.float32)
    y = g["batch0::labels"]
    mults = [dense_ref.dropedge_weights_pre(A, 0.3, 5, c) for c in range(3)]
    logits = dense_ref.graph_cnn_dropedge_forward(P, V, A, edge_mults=mults)
    keep = y != -100
    z = logits[keep]
    lse = np.log(np.exp(z - z.max(-1, keepdims=True)).sum(-1)) + z.max(-1)
    loss = float((lse - z[np.arange(len(z)), y[keep]]).mean())
    assert abs(loss - float(g["eager::losses"][0])) <= 1e-5 * abs(loss), (loss, g["eager::losses"][0])
