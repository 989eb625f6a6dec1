"""GraphCNNDropEdge on the MI355X engine (drop-in for
gnn/models/networks/drop_robust_gcn.py).

Forward (reference :61-103):
    emb1 -> [edge_dropout -> GraphConv -> ReLU -> Dropout] x3 (skip concats)
    -> emb2 -> NodeSelfAtten -> RanPAC random projection -> ReLU -> Dropout
    -> classifier
The adjacency is converted once to a TypedGraph (the reference preprocesses
once in efficient_mode, :69); each edge_dropout call becomes a (p, seed,
call) record that the aggregation kernels expand on the fly, so no dense
A_pre and no dense mask exist.  Module names, parameter shapes and creation
order match the reference (state_dict keys, shapes and init RNG identical).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from gnn.models.base_network import BaseNetwork
from gnn.models.networks.robust_gcn import (ROW_LINEAR_MIN_ROWS, GraphConv, NodeSelfAtten, apply_linear,
                                            make_linear_relu)
from grl import DropEdge, TypedGraph, device_check
from grl.dist import ShardedGraph
from grl.ops import bag_linear, feature_dropout

RP_FACTOR = 10


class RanPACLayer(nn.Module):
    """Frozen Gaussian random projection (drop_robust_gcn.py:13-28)."""

    def __init__(self, input_dim: int, output_dim: int):
        super().__init__()
        self.projection = nn.Linear(input_dim, output_dim, bias=False)
        for p in self.projection.parameters():
            p.requires_grad = False
        nn.init.normal_(self.projection.weight, mean=0, std=1.0)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.projection(x)


class EdgeDropout(nn.Dropout):
    """nn.Dropout(p) over the preprocessed adjacency (drop_robust_gcn.py:38).

    On a TypedGraph it returns the graph tagged with a fresh DropEdge draw
    (training) or untagged (eval / p == 0): the mask is generated inside the
    aggregation kernels from (seed, call, edge id).  `seed=None` draws each
    call's seed on the graph's device (torch's CUDA generator, so
    torch.manual_seed makes runs reproducible) into a 1-element tensor the
    kernels read at launch: no host round trip, and a training step captured
    in a HIP graph redraws every mask on each replay.  A fixed `seed` numbers
    calls 0, 1, 2, ... (reset_calls()) for parity tests.  Dense tensors get
    plain nn.Dropout.
    `stream` (data-parallel rank, set by the training procedure) keeps the
    ranks' masks independent when every rank is seeded alike
    (cl_warper.py:36-40): it is the DropEdge call id under a device-drawn
    seed, and the upper 32 bits of the call id under a fixed seed (rank r's
    call c is c + r * 2^32).
    `seed_source` (a 1-element int64 device tensor, set by a training
    procedure that captures its step, KVProcedure) takes precedence: every
    call reads the seed from it at launch, with call ids numbered from
    reset_calls() -- the procedure writes a new seed before each step, so a
    replayed HIP graph draws new masks, identical to the eager step's.
    """

    STREAM_SHIFT = 32

    def __init__(self, p: float = 0.5, seed: Optional[int] = None):
        super().__init__(p=p)
        self.seed = seed
        self.stream = 0
        self.seed_source: Optional[torch.Tensor] = None
        self._calls = 0

    def reset_calls(self) -> None:
        self._calls = 0

    def forward(self, A, drop_self: bool = True):
        if not isinstance(A, (TypedGraph, ShardedGraph)):
            return super().forward(A)
        if not self.training or self.p == 0.0:
            return A.with_dropedge(None)
        if self.seed_source is not None:
            call = self._calls + (self.stream << self.STREAM_SHIFT)
            self._calls += 1
            return A.with_dropedge(DropEdge(p=float(self.p), seed=0, call=call, drop_self=drop_self,
                                            seed_tensor=self.seed_source))
        if self.seed is None:
            seed_t = torch.randint(0, 2**62, (1,), dtype=torch.int64, device=A.device)
            if isinstance(A, ShardedGraph):  # one draw for the whole graph: rank 0's seed on every rank
                seed_t = A.broadcast_seed(seed_t)
            return A.with_dropedge(DropEdge(p=float(self.p), seed=0, call=self.stream, drop_self=drop_self,
                                            seed_tensor=seed_t))
        else:
            seed, call = self.seed, self._calls + (self.stream << self.STREAM_SHIFT)
            self._calls += 1
        return A.with_dropedge(DropEdge(p=float(self.p), seed=seed, call=call, drop_self=drop_self))


class FeatureDropout(nn.Dropout):
    """nn.Dropout(p) on node-feature rows (drop_robust_gcn.py:64,77,81,86,100)
    whose mask is a counter hash of (seed, call, global row, column)
    (grl_feature_dropout): the mask of a row does not depend on where the
    row is computed, so a node-range shard draws exactly the one-GPU model's
    mask for its rows, and a row block's mask is computable on its own.
    The distribution is the reference's (i.i.d. keep(1-p), scaled by
    1/(1-p)); the draws are not torch's generator stream.

    Seeds, as EdgeDropout's: `seed_source` (a device word a captured training
    step writes) takes precedence; else a fixed `seed` with calls numbered
    0, 1, 2, ... (reset_calls()); else begin_forward() draws one device seed
    per forward (torch's CUDA generator, so torch.manual_seed reproduces
    runs; broadcast from rank 0 on a sharded graph) and numbers that
    forward's calls from 0.  `stream` (data-parallel rank) keeps the ranks'
    masks independent.  Host tensors, and graphs of at most
    ROW_LINEAR_MIN_ROWS rows that are not a shard (document pages: too small
    to shard, host-bound steps where one fused torch op beats two library
    calls), get plain nn.Dropout."""

    STREAM_SHIFT = 32
    DOMAIN = 1 << 48  # call ids apart from EdgeDropout's (which may share the seed)

    def __init__(self, p: float = 0.5, seed: Optional[int] = None):
        super().__init__(p=p)
        self.seed = seed
        self.stream = 0
        self.seed_source: Optional[torch.Tensor] = None
        self._calls = 0
        self._seed_t: Optional[torch.Tensor] = None
        self.row0 = 0
        self._hash = True

    def reset_calls(self) -> None:
        self._calls = 0

    def begin_forward(self, device, shard: Optional[ShardedGraph] = None, rows: Optional[int] = None) -> None:
        """Per-forward state: the global row of this rank's first row, the
        mask kind (the hash on shards and on graphs of more than
        ROW_LINEAR_MIN_ROWS rows), and (device-drawn seeds) the forward's
        seed."""
        self.row0 = shard.plan.row_begin if shard is not None else 0
        self._hash = shard is not None or rows is None or rows > ROW_LINEAR_MIN_ROWS
        if self.seed_source is not None or self.seed is not None or not self.training or self.p == 0.0 \
                or torch.device(device).type != "cuda" or not self._hash:
            return
        seed_t = torch.randint(0, 2**62, (1,), dtype=torch.int64, device=device)
        self._seed_t = shard.broadcast_seed(seed_t) if shard is not None else seed_t
        self._calls = 0

    def record(self, device) -> Optional[DropEdge]:
        """The next call's draw (p, seed, call id) as a DropEdge record, or
        None when the dropout is the identity (eval, p == 0) or runs on the
        host; consumes a call id.  A layer that fuses this dropout
        (GraphConv.propagate on a shard) applies it with row0."""
        if not self.training or self.p == 0.0 or torch.device(device).type != "cuda":
            return None
        call = self.DOMAIN + self._calls + (self.stream << self.STREAM_SHIFT)
        self._calls += 1
        if self.seed_source is not None:
            return DropEdge(p=float(self.p), seed=0, call=call, seed_tensor=self.seed_source)
        if self.seed is not None:
            return DropEdge(p=float(self.p), seed=self.seed, call=call)
        if self._seed_t is None or self._seed_t.device != torch.device(device):
            self.begin_forward(device)
            call = self.DOMAIN + (self.stream << self.STREAM_SHIFT)
            self._calls = 1
        return DropEdge(p=float(self.p), seed=0, call=call, seed_tensor=self._seed_t)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self.training or self.p == 0.0:
            return x
        if not x.is_cuda or not self._hash:
            return super().forward(x)
        return feature_dropout(x.float(), self.record(x.device), self.row0)


# grl_bag_linear_fwd keeps one output row per wave in registers (include/grl.h)
BAG_LINEAR_MAX_C = 512


class GraphCNNDropEdge(BaseNetwork):
    def __init__(self, input_dim: int, output_dim: int, num_edges: int, net_size: int = 256,
                 use_attention: bool = True, dropedge_seed: Optional[int] = None):
        super().__init__()
        self.output_dim = output_dim
        self.net_size = net_size
        self.emb1 = make_linear_relu(input_dim, self.net_size)
        # emb1's input is a bag-of-characters row (~7 nonzeros of 4369): run it
        # as a sparse-row gather (grl_bag_linear_fwd); False = dense torch Linear
        self.sparse_emb1 = True
        self.dropout = FeatureDropout(p=0.5, seed=dropedge_seed)
        self.edge_dropout = EdgeDropout(p=0.3, seed=dropedge_seed)
        self.gcn1 = GraphConv(self.net_size, self.net_size, num_edges)
        self.gcn2 = GraphConv(self.net_size, self.net_size, num_edges)
        self.gcn3 = GraphConv(self.net_size * 2, self.net_size, num_edges)
        half_net_size = self.net_size // 2
        self.emb2 = make_linear_relu(self.net_size * 2, half_net_size)
        self.use_attention = use_attention
        if use_attention:
            self.self_atten = NodeSelfAtten(half_net_size)
        rp_size = half_net_size * RP_FACTOR
        self.w_rand = RanPACLayer(half_net_size, rp_size)
        self.classifier = nn.Linear(rp_size, output_dim)

    def to_graph(self, A) -> TypedGraph:
        """Collate-layout dense A (B, N, L, N) -> TypedGraph on the model's
        device.  A grl.dist.ShardedGraph (additive: this rank's node-range
        shard of one large graph, V holding the shard's rows) is used as is:
        every layer then runs on the shard -- GraphConv with its halo
        exchange, NodeSelfAtten with the softmax over all nodes -- and the
        logits are the shard's rows of the one-GPU model's."""
        if isinstance(A, (TypedGraph, ShardedGraph)):
            return A
        dev = self.gcn1.h_weights.device
        return TypedGraph.from_dense(A if A.device == dev else A.to(dev), layout="bnln")

    def _embed(self, V: torch.Tensor) -> torch.Tensor:
        """emb1 (drop_robust_gcn.py:36,64): Linear + ReLU, same parameters."""
        lin = self.emb1[0]
        if self.sparse_emb1 and V.is_cuda and lin.out_features <= BAG_LINEAR_MAX_C:
            return bag_linear(V.float(), lin.weight, lin.bias, relu=True)
        return self.emb1(V)  # net_size > 512: one output row no longer fits a wave's registers

    def forward(self, inputs, efficient_mode: bool = True):
        V, A = inputs
        graph = self.to_graph(A)
        sharded = isinstance(graph, ShardedGraph)
        if sharded and any(b1 <= b0 for b0, b1 in zip(graph.plan.bounds[:-1], graph.plan.bounds[1:])):
            # every rank holds the same bounds, so every rank raises here (none is left waiting in a
            # collective): the streamed layers and the attention's row gathers assume each rank owns rows
            raise ValueError(f"GraphCNNDropEdge over node-range shards needs every shard to own at least one "
                             f"node (bounds {list(graph.plan.bounds)}): use fewer ranks than nodes")
        # row-local layers of a shard take the one-GPU model's GEMM path (bitwise its rows)
        pr = graph.global_rows if sharded else 0
        self.dropout.begin_forward(V.device, graph if sharded else None, V.numel() // max(V.shape[-1], 1))
        embedding = self.dropout(self._embed(V))
        # efficient_mode=True: dropout covers the identity block of A_pre
        # (:69,:76); False: dropout hits raw A, identity added after (:72-74).
        ds = bool(efficient_mode)
        if sharded:  # gcn3's input cat[g1, g2]: g1's halo rows already came for gcn2
            graph = graph.with_halo_memo()
        # each GraphConv's feature dropout (:77,:81,:86) rides in propagate: on a shard in training it is fused
        # into the layer, whose output rows then stream to the peers while the rest of the layer computes
        g1 = self.gcn1.propagate(embedding, self.edge_dropout(graph, ds), relu=True, dropout=self.dropout)
        if sharded:
            graph.remember(g1)
        g2 = self.gcn2.propagate(g1, self.edge_dropout(graph, ds), relu=True, dropout=self.dropout)
        x3 = torch.cat([g1, g2], dim=-1)
        if sharded:
            graph.note_concat(x3, (g1, g2))
        # (sharded inference: gcn3's rows feed no later GraphConv, so they are not streamed)
        g3 = self.gcn3.propagate(x3, self.edge_dropout(graph.without_streaming() if sharded else graph, ds),
                                 relu=True, dropout=self.dropout)
        if sharded:
            graph.clear_halo_memo()
        new_v = apply_linear(self.emb2, torch.cat([g1, g3], dim=-1), path_rows=pr)
        if self.use_attention:
            new_v = self.self_atten(new_v, shard=graph) if sharded else self.self_atten(new_v)
        new_v = self.dropout(apply_linear(self.w_rand.projection, new_v, relu=True, path_rows=pr))
        logits = apply_linear(self.classifier, new_v, path_rows=pr)
        if sharded and not torch.is_grad_enabled() and logits.is_cuda:
            # sharded inference has no procedure around it to surface a persistent kernel's stream-ordered
            # failure (grl_check): one check per forward (training: allreduce_gradients checks)
            device_check(logits.device)
        return logits
