"""GraphConv on the MI355X engine (drop-in for gnn/models/networks/robust_gcn.py).

Reference semantics (robust_gcn.py:14-75): for V (B, N, F) and the
preprocessed adjacency A_pre (B, (L+1)N, N),
    new_V = (A_pre @ V).view(B, N, (L+1)F)          # aggregation, :45-47
    out   = new_V @ h_weights + bias                # dense linear, :50-51
Here A_pre is a TypedGraph (typed CSR, identity block implicit) and the two
steps are libgrl kernels: grl_typed_spmm_fwd (HBM-bound gather) and
grl_linear_fwd (fp32 MFMA).  Parameters, their shapes, creation order and
init RNG use are the reference's, so state_dicts load both ways and
torch.manual_seed reproduces the reference's weights bit for bit.
"""
from __future__ import annotations

from typing import Optional, Union

import torch
from torch import nn

from grl import TypedGraph
from grl.dist import ShardedGraph, sharded_node_attention
from grl.ops import graph_conv, node_self_attention, row_linear


def make_linear_relu(input_dim: int, output_dim: int) -> nn.Sequential:
    """Linear + ReLU block (robust_gcn.py:10-11); state_dict keys `0.weight`, `0.bias`."""
    return nn.Sequential(nn.Linear(input_dim, output_dim), nn.ReLU())


# Row count from which the row-local linears run on the libgrl GEMM (whose row
# results do not depend on the row count: what a node-range shard needs to
# reproduce the one-GPU model's rows bitwise).  Below it -- document pages
# such as debug.json's 74 nodes, graphs far too small to shard -- torch's
# single-launch GEMM is faster (tools/probe_row_linear.py).  The choice is
# made on the WHOLE graph's rows (path_rows), so a shard and its one-GPU
# model always take the same one.
ROW_LINEAR_MIN_ROWS = 4096


def _on_grl(x: torch.Tensor, path_rows: int) -> bool:
    return x.is_cuda and max(x.numel() // max(x.shape[-1], 1), path_rows) > ROW_LINEAR_MIN_ROWS


def apply_linear(mod: nn.Module, x: torch.Tensor, relu: bool = False, path_rows: int = 0) -> torch.Tensor:
    """An nn.Linear (or a make_linear_relu block, its ReLU fused) over the rows
    of x: on the libgrl GEMM (grl.ops.row_linear, rows independent of the row
    count; path_rows: a node-range shard's whole-graph row count) from
    ROW_LINEAR_MIN_ROWS rows, else torch."""
    lin = mod[0] if isinstance(mod, nn.Sequential) else mod
    if isinstance(mod, nn.Sequential):
        relu = True
    return linear_rows(x, lin.weight, lin.bias, relu, path_rows)


def linear_rows(x: torch.Tensor, W: torch.Tensor, b, relu: bool, path_rows: int = 0) -> torch.Tensor:
    if _on_grl(x, path_rows):
        return row_linear(x.float(), W, b, relu=relu, path_rows=path_rows)
    y = torch.nn.functional.linear(x, W, b)
    return torch.relu(y) if relu else y


AdjLike = Union[TypedGraph, torch.Tensor]


class GraphConv(nn.Module):
    """Multi-edge-type graph convolution, `num_edges` (L) edge types plus the
    identity block; h_weights rows are grouped by type: rows [l*F, (l+1)*F)
    multiply segment l (l = 0 is the node itself)."""

    def __init__(self, input_dim: int, output_dim: int, num_edges: int, with_bias: bool = True):
        super().__init__()
        self.C = output_dim
        self.L = num_edges
        self.F = input_dim
        self.gpu = torch.cuda.is_available()
        # training memory: None = keep Z = A_pre V for the weight gradient unless it
        # exceeds grl.ops.RECOMPUTE_Z_BYTES, True = always re-aggregate it in the
        # backward (saves (L+1)F floats per node), False = always keep it
        self.recompute_aggregation: Optional[bool] = None
        # Same allocation + init sequence as robust_gcn.py:22-30 (xavier_normal_
        # on h_weights, then normal_(1e-4, 5e-5) on bias): identical RNG draws.
        self.h_weights = nn.Parameter(torch.empty(self.F * (self.L + 1), self.C))
        if with_bias:
            self.bias = nn.Parameter(torch.empty(self.C))
        else:
            self.register_parameter("bias", None)
        nn.init.xavier_normal_(self.h_weights)
        if self.bias is not None:
            nn.init.normal_(self.bias, mean=0.0001, std=0.00005)

    # --------------------------------------------------------------- graph
    def preprocess_adj(self, adj: AdjLike) -> TypedGraph:
        """(B, N, N, L) adjacency -> TypedGraph (the sparse A_pre of
        robust_gcn.py:53-72: identity block + typed segments)."""
        if isinstance(adj, TypedGraph):
            return adj
        return TypedGraph.from_dense(self._on_device(adj), layout="bnnl")

    def _on_device(self, t: torch.Tensor) -> torch.Tensor:
        dev = self.h_weights.device
        return t if t.device == dev else t.to(dev)

    def _graph(self, A: AdjLike, preprocess_A: bool) -> TypedGraph:
        if isinstance(A, TypedGraph):
            return A
        if preprocess_A:
            return self.preprocess_adj(A)
        return TypedGraph.from_dense(self._on_device(A), layout="pre")

    # ------------------------------------------------------------- forward
    def propagate(self, V: torch.Tensor, graph, relu: bool = False, dropout=None) -> torch.Tensor:
        """Aggregate + linear (+ fused ReLU) on a ready TypedGraph, or on this
        rank's node-range shard of a graph (grl.dist.ShardedGraph: V holds the
        shard's rows; the halo exchange runs inside, the output rows are the
        shard's, every value the one-GPU layer's -- the forward bitwise).
        dropout: the feature dropout the model applies to the layer's output
        (drop_robust_gcn.py:77,81,86); on a shard in training it is fused into
        the layer, whose output rows then stream to the peers as they are
        written."""
        lead = V.shape[:-1]
        if isinstance(graph, ShardedGraph):
            V2 = V.reshape(-1, V.shape[-1])
            training = torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                                       for t in (V, self.h_weights, self.bias))
            if training:  # the one-kernel forms both ways, the reverse halo exchange pipelined over row blocks
                fd = dropout.record(V.device) if dropout is not None else None
                out = graph.graphconv(V2, self, relu=relu, pipeline="rows", fdrop=fd)
            else:
                out = graph.graphconv(V2, self, relu=relu)
                out = dropout(out) if dropout is not None else out
            return out.view(*lead, self.C)
        # new_V = A_pre V (B*N, (L+1)F) then new_V h_weights + bias, one autograd node
        out = graph_conv(V, graph, self.h_weights, self.bias, relu=relu, recompute=self.recompute_aggregation)
        out = out.view(*lead, self.C)
        return dropout(out) if dropout is not None else out

    def forward(self, V: torch.Tensor, A: AdjLike, preprocess_A: bool = True) -> torch.Tensor:
        """V: (B, N, F).  A: TypedGraph, or dense (B, N, N, L) when
        preprocess_A, or dense A_pre (B, (L+1)N, N) when not."""
        return self.propagate(V, self._graph(A, preprocess_A), relu=False)

    def __repr__(self) -> str:
        return f"GraphConv(in_dim={self.F}, out_dim={self.C}, num_edges={self.L}, bias={self.bias is not None})"


class NodeSelfAtten(nn.Module):
    """Node self-attention (robust_gcn.py:78-99): gamma * softmax(f g^T) h + V.
    The f/g/h projections are torch Linear+ReLU (as in the reference); the
    attention core is the fused flash-style libgrl kernel
    (grl_node_attention_fwd/_bwd), so the N x N scores never exist and the
    model runs at graph sizes where the reference's dense softmax cannot."""

    def __init__(self, input_dim: int):
        super().__init__()
        self.F = input_dim
        self.f = make_linear_relu(input_dim, int(self.F // 8))
        self.g = make_linear_relu(input_dim, int(self.F // 8))
        self.h = make_linear_relu(input_dim, self.F)
        self.softmax = nn.Softmax(-1)
        self.gamma = nn.Parameter(torch.empty(input_dim))
        nn.init.normal_(self.gamma)

    def forward(self, V: torch.Tensor, shard=None) -> torch.Tensor:
        """shard (additive): the grl.dist.ShardedGraph whose rows V holds --
        the softmax then runs over every node of the graph
        (grl.dist.sharded_node_attention)."""
        pr = shard.global_rows if shard is not None else 0
        if _on_grl(V, pr):
            # f, g, h read the same V: one GEMM over their concatenated weights (2 x F/8 + F columns; a
            # column's result does not depend on the others)
            lins = (self.f[0], self.g[0], self.h[0])
            W = torch.cat([m.weight for m in lins])
            b = torch.cat([m.bias for m in lins])
            fgh = linear_rows(V, W, b, True, pr)
            dk = self.f[0].out_features
            f, g, h = fgh[..., :dk], fgh[..., dk:2 * dk], fgh[..., 2 * dk:]
        else:  # small graphs: torch's three GEMMs, no concatenation or strided slices around them
            f, g, h = self.f(V), self.g(V), self.h(V)
        if shard is not None:
            return sharded_node_attention(f, g, h, V, self.gamma, shard)
        return node_self_attention(f, g, h, V, self.gamma)

    def __repr__(self) -> str:
        return f"NodeSelfAttention(input_dim={self.F})"
