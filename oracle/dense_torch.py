"""TEST INFRASTRUCTURE ONLY (CPU baseline).  fp32 torch-CPU restatement of
the reference's dense GraphCNNDropEdge, operation for operation, for timing
the reference's own CPU path on the GPU box's host (the reference cannot
travel there; SURVEY.md §8(d) "C1: dense restatement of a2-a5 (exact
reference math, incl. dense dropout) and the whole model forward").

  gnn/models/networks/robust_gcn.py:39-51   GraphConv.forward (bmm + mm)
  gnn/models/networks/robust_gcn.py:53-72   preprocess_adj (dense A_pre)
  gnn/models/networks/robust_gcn.py:78-99   NodeSelfAtten
  gnn/models/networks/drop_robust_gcn.py:61-103  GraphCNNDropEdge.forward,
      with edge_dropout = nn.Dropout(0.3) drawing a dense Bernoulli mask over
      A_pre on every call and nn.Dropout(0.5) on node features (train mode)

Parameters come as a state_dict of fp32 CPU tensors (the engine model's, so
both sides start from the same weights).  Never imported by the product.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def preprocess_adj(A_bnnl: torch.Tensor) -> torch.Tensor:
    """(B, N, N, L) -> (B, (L+1)N, N), identity block l = 0."""
    B, N, _, L = A_bnnl.shape
    eye = torch.eye(N, dtype=A_bnnl.dtype).view(1, N, N, 1).expand(B, N, N, 1)
    adj = torch.cat([eye, A_bnnl], dim=-1).view(B * N, N, L + 1).permute(0, 2, 1).contiguous()
    return adj.view(B, (L + 1) * N, N)


def graph_conv(V, A_pre, W, b):
    B, N, Fd = V.shape
    L1 = W.shape[0] // Fd
    new_v = torch.matmul(A_pre, V).view(B, N, L1 * Fd)
    return torch.matmul(new_v, W) + b


def forward(P: dict, V: torch.Tensor, A_bnln: torch.Tensor, train: bool = False, p_edge: float = 0.3,
            p_feat: float = 0.5, edge_mults=None) -> torch.Tensor:
    """edge_mults: optional three (B, (L+1)N, N) multipliers over A_pre
    injected in place of the three edge_dropout draws (parity tests; feature
    dropout is then whatever `train` / p_feat say)."""
    drop = (lambda x, p: F.dropout(x, p, True)) if train else (lambda x, p: x)
    A_pre = preprocess_adj(A_bnln.permute(0, 1, 3, 2))
    it = iter(edge_mults) if edge_mults is not None else None

    def edrop(A):
        return A * next(it) if it is not None else drop(A, p_edge)

    emb = drop(F.relu(F.linear(V, P["emb1.0.weight"], P["emb1.0.bias"])), p_feat)
    g1 = drop(F.relu(graph_conv(emb, edrop(A_pre), P["gcn1.h_weights"], P["gcn1.bias"])), p_feat)
    g2 = drop(F.relu(graph_conv(g1, edrop(A_pre), P["gcn2.h_weights"], P["gcn2.bias"])), p_feat)
    g3 = drop(F.relu(graph_conv(torch.cat([g1, g2], -1), edrop(A_pre), P["gcn3.h_weights"], P["gcn3.bias"])),
              p_feat)
    x = F.relu(F.linear(torch.cat([g1, g3], -1), P["emb2.0.weight"], P["emb2.0.bias"]))
    if "self_atten.gamma" in P:
        f = F.relu(F.linear(x, P["self_atten.f.0.weight"], P["self_atten.f.0.bias"]))
        g = F.relu(F.linear(x, P["self_atten.g.0.weight"], P["self_atten.g.0.bias"]))
        h = F.relu(F.linear(x, P["self_atten.h.0.weight"], P["self_atten.h.0.bias"]))
        s = torch.softmax(torch.matmul(f, g.transpose(1, 2)), -1)
        x = P["self_atten.gamma"] * torch.matmul(s, h) + x
    x = drop(F.relu(F.linear(x, P["w_rand.projection.weight"])), p_feat)
    return F.linear(x, P["classifier.weight"], P["classifier.bias"])


class TrainStep:
    """One Adam training step of the dense model (kv_procedure.py:143-164 in
    the reference: forward in train mode, cross-entropy, backward, step)."""

    def __init__(self, state_dict: dict, lr: float = 1e-3):
        self.P = {k: v.detach().float().cpu().clone() for k, v in state_dict.items()}
        params = [v.requires_grad_(True) for k, v in self.P.items() if k != "w_rand.projection.weight"]
        self.opt = torch.optim.Adam(params, lr=lr)

    def __call__(self, V, A, y) -> float:
        self.opt.zero_grad(set_to_none=True)
        logits = forward(self.P, V, A, train=True)
        loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1))
        loss.backward()
        self.opt.step()
        return float(loss.detach())
