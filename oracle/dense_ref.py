"""TEST INFRASTRUCTURE ONLY.  numpy restatement of the reference's dense path.

Restates, operation for operation, the math of
  gnn/models/networks/robust_gcn.py:14-99   (GraphConv, NodeSelfAtten)
  gnn/models/networks/drop_robust_gcn.py:13-103 (RanPACLayer, GraphCNNDropEdge)
in float64 (the "true" value the fp32 reference and the fp32 engine are both
compared against).  DropEdge masks are supplied explicitly (the reference's
Bernoulli draw is replaced by oracle.hash in parity tests; see
oracle/grl_oracle.c header).  Pinned by tests/golden/*.npz.
"""
from __future__ import annotations

import numpy as np

from oracle import hash as ohash


def preprocess_adj(adj_bnnl: np.ndarray) -> np.ndarray:
    """robust_gcn.py:53-72: (B,N,N,L) -> (B,(L+1)N,N) with identity block l=0."""
    B, N, _, L = adj_bnnl.shape
    eye = np.broadcast_to(np.eye(N, dtype=adj_bnnl.dtype)[None, :, :, None], (B, N, N, 1))
    adj = np.concatenate([eye, adj_bnnl], axis=-1)  # B,N,N,L+1
    adj = adj.reshape(B * N, N, L + 1)
    return np.ascontiguousarray(adj.transpose(0, 2, 1)).reshape(B, (L + 1) * N, N)


def graphconv_forward(V, A_pre, W, bias):
    """robust_gcn.py:39-51 (preprocess_A=False): returns (out, new_V)."""
    B, N, F = V.shape
    L1 = W.shape[0] // F
    Z = np.matmul(A_pre, V.reshape(-1, N, F)).reshape(-1, N, L1 * F)
    out = np.matmul(Z, W) + bias[None]
    return out.reshape(B, N, W.shape[1]), Z


def graphconv_backward(V, A_pre, W, Z, dout):
    """Autograd of robust_gcn.py:45-50: (dV, dW, dbias)."""
    B, N, F = V.shape
    K, C = W.shape
    d2 = dout.reshape(-1, C)
    dW = Z.reshape(-1, K).T @ d2
    db = d2.sum(0)
    dZ = (d2 @ W.T).reshape(B, -1, F)  # (B, (L+1)N, F): view of (B, N, (L+1)F)
    dV = np.matmul(np.swapaxes(A_pre, 1, 2), dZ)
    return dV, dW, db


def dense_edge_ids(A_bnln: np.ndarray, self_base=None):
    """Global DropEdge ids of A_pre's nonzeros, in the engine's id scheme:
    typed edges numbered in CSR order (b, n, t, m ascending); the self loop of
    global node b*N+n gets self_base + b*N + n, self_base = E by default (a
    captured training step's static graph starts them at its edge capacity,
    step_graph.py).  Returns (ids_pre, E) where ids_pre has A_pre's shape and
    is -1 on structural zeros."""
    B, N, L, _ = A_bnln.shape
    nz = A_bnln != 0
    E = int(nz.sum())
    ids = np.full(A_bnln.shape, -1, dtype=np.int64)
    ids[nz] = np.arange(E, dtype=np.int64)  # C-order == (b, n, t, m) ascending
    ids_pre = np.full((B, N, L + 1, N), -1, dtype=np.int64)
    ids_pre[:, :, 1:, :] = ids
    g = np.arange(B * N, dtype=np.int64).reshape(B, N)
    sb = E if self_base is None else int(self_base)
    for n in range(N):
        ids_pre[:, n, 0, n] = sb + g[:, n]
    return ids_pre.reshape(B, N * (L + 1), N), E


def dropedge_weights_pre(A_bnln, p, seed, call, drop_self=True, self_base=None):
    """Multiplier applied to each A_pre entry by the fused DropEdge:
    keep * float(1/(1-p)) (0 for dropped; 1 on the identity when
    drop_self is False)."""
    ids_pre, _ = dense_edge_ids(A_bnln, self_base)
    active, _, scale = ohash.dropedge_params(p)
    mult = np.zeros(ids_pre.shape, dtype=np.float32)
    valid = ids_pre >= 0
    keep = ohash.dropedge_keep(p, seed, call, ids_pre[valid].astype(np.uint64))
    mult[valid] = np.where(keep, scale, np.float32(0.0)) if active else np.float32(1.0)
    if not drop_self:
        B, R, N = ids_pre.shape
        L1 = R // N
        for n in range(N):
            mult[:, n * L1, n] = 1.0
    return mult


def apply_dropedge(A_pre_f32: np.ndarray, mult: np.ndarray) -> np.ndarray:
    """fp32 A_drop entries as torch forms them: (a * mask) * scale."""
    return (A_pre_f32.astype(np.float32) * mult).astype(np.float32)


# ---------------------------- full model -----------------------------------
def _relu(x):
    return np.maximum(x, 0.0)


def _linear(x, w, b=None):
    y = x @ w.T
    return y + b if b is not None else y


def _softmax(x, axis=-1):
    x = x - x.max(axis=axis, keepdims=True)
    e = np.exp(x)
    return e / e.sum(axis=axis, keepdims=True)


def node_self_atten(P, prefix, x):
    """robust_gcn.py:90-96."""
    f = _relu(_linear(x, P[prefix + "f.0.weight"], P[prefix + "f.0.bias"]))
    g = _relu(_linear(x, P[prefix + "g.0.weight"], P[prefix + "g.0.bias"]))
    h = _relu(_linear(x, P[prefix + "h.0.weight"], P[prefix + "h.0.bias"]))
    s = _softmax(np.matmul(f, np.swapaxes(g, 1, 2)), -1)
    return P[prefix + "gamma"] * np.matmul(s, h) + x


def graph_cnn_dropedge_forward(P: dict, V, A_bnln, edge_mults=None, use_attention=True):
    """drop_robust_gcn.py:61-103 with feature dropout as identity (eval, or
    p=0) and optional explicit DropEdge multipliers for the three
    edge_dropout calls.  P: state_dict as float64 numpy arrays."""
    V = V.astype(np.float64)
    A = np.transpose(A_bnln, (0, 1, 3, 2)).astype(np.float64)
    emb = _relu(_linear(V, P["emb1.0.weight"], P["emb1.0.bias"]))
    A_pre = preprocess_adj(A)

    def drop(i):
        return A_pre if edge_mults is None else A_pre * edge_mults[i].astype(np.float64)

    g1 = _relu(graphconv_forward(emb, drop(0), P["gcn1.h_weights"], P["gcn1.bias"])[0])
    g2 = _relu(graphconv_forward(g1, drop(1), P["gcn2.h_weights"], P["gcn2.bias"])[0])
    g3 = _relu(graphconv_forward(np.concatenate([g1, g2], -1), drop(2), P["gcn3.h_weights"], P["gcn3.bias"])[0])
    x = _relu(_linear(np.concatenate([g1, g3], -1), P["emb2.0.weight"], P["emb2.0.bias"]))
    if use_attention:
        x = node_self_atten(P, "self_atten.", x)
    x = _relu(_linear(x, P["w_rand.projection.weight"]))
    return _linear(x, P["classifier.weight"], P["classifier.bias"])
