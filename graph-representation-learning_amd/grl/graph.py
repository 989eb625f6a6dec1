"""TypedGraph: the HBM-resident sparse stand-in for the reference's A_pre.

The reference materialises A_pre = preprocess_adj(A) as a dense
(B, (L+1)N, N) tensor (gnn/models/networks/robust_gcn.py:53-72) and draws a
dense Bernoulli mask over it for every edge_dropout call
(gnn/models/networks/drop_robust_gcn.py:76,80,85).  A TypedGraph holds the
same operator as a typed CSR (rows = destination nodes, one segment per edge
type, implicit identity block) plus, lazily, its CSC for the backward pass.
DropEdge is a small (p, seed, call) record; the mask is regenerated inside
the kernels and never stored.

Layout in HBM (int32 indices, fp32 values):
  rowptr [num_rows*L + 1]   colidx [nnz]   vals [nnz] or None (all ones)
  colptr [num_cols + 1]     zrow [nnz]     eid [nnz]   cvals [nnz] (CSC)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch

from . import _lib
from ._lib import GrlDropEdge, GrlSplitPlan, GrlSynthSpec, GrlTypedCsc, GrlTypedCsr, call

# Heavy-row splitting (R-MAT hubs): rows with more edges than SPLIT_THRESHOLD
# are summed in chunks of SPLIT_CHUNK edges by separate wavefronts.
SPLIT_THRESHOLD = 2048
SPLIT_CHUNK = 1024


def current_stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def device_check(device=None) -> None:
    """Raise GrlError if a persistent one-kernel GraphConv call on `device`
    (default: the current one) gave up on its LDS ring since the last check:
    grl_check reads and clears the sticky status word those calls' follow-up
    kernels set (their outputs are NaN then).  It waits for the current
    stream, so call it where the caller syncs anyway (a loss.item())."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        return  # no device work ran there
    with torch.cuda.device(dev):  # the sticky word is per device: the library reads the current device's
        call("grl_check", current_stream_handle(dev))


def _require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise _lib.GrlError(
            f"{what} must be a ROCm device tensor (got {t.device}); the MI355X engine has no CPU path")


@dataclass(frozen=True)
class DropEdge:
    """One edge_dropout draw: nn.Dropout(p) over A_pre (drop_robust_gcn.py:38).

    seed_tensor: optional 1-element int64 device tensor holding the seed; the
    kernels read it at launch (grl_dropedge_init_device), so a HIP graph that
    captured the seed's producer (a device RNG kernel) redraws the mask on
    every replay.  `seed` is then unused."""

    p: float
    seed: int
    call: int = 0
    drop_self: bool = True  # efficient_mode=True masks the identity block too
    seed_tensor: Optional[torch.Tensor] = field(default=None, compare=False, repr=False)

    def to_c(self) -> GrlDropEdge:
        de = GrlDropEdge()
        if self.seed_tensor is not None:
            t = self.seed_tensor
            if not t.is_cuda or t.dtype != torch.int64 or t.numel() != 1:
                raise _lib.GrlError("DropEdge.seed_tensor must be a 1-element int64 device tensor")
            call("grl_dropedge_init_device", ctypes.byref(de), float(self.p), t.data_ptr(),
                 int(self.call) & (2**64 - 1), int(self.drop_self))
            return de
        call("grl_dropedge_init", ctypes.byref(de), float(self.p), int(self.seed) & (2**64 - 1),
             int(self.call) & (2**64 - 1), int(self.drop_self))
        return de


class TypedGraph:
    """Typed CSR over `num_rows` destination nodes gathering from `num_cols`
    source rows.  `batch_shape = (B, N)` records a block-diagonal batch of B
    graphs of N (padded) nodes each, row id = b*N + n."""

    def __init__(self, rowptr: torch.Tensor, colidx: torch.Tensor, num_types: int, *,
                 vals: Optional[torch.Tensor] = None, has_self: bool = True, num_cols: Optional[int] = None,
                 edge_id_base: int = 0, self_id_base: Optional[int] = None, self_rows: Optional[int] = None,
                 batch_shape: Optional[Tuple[int, int]] = None, _shared: Optional[dict] = None):
        _require_device(rowptr, "rowptr")
        if rowptr.dtype != torch.int32 or colidx.dtype != torch.int32:
            raise _lib.GrlError("rowptr/colidx must be int32")
        if (rowptr.numel() - 1) % num_types:
            raise _lib.GrlError(f"rowptr length {rowptr.numel()} is not num_rows*{num_types}+1")
        self.rowptr = rowptr.contiguous()
        self.colidx = colidx.contiguous()
        self.vals = None if vals is None else vals.contiguous().float()
        self.num_types = int(num_types)
        self.has_self = bool(has_self)
        self.num_rows = (rowptr.numel() - 1) // num_types
        self.num_cols = self.num_rows if num_cols is None else int(num_cols)
        self.nnz = int(colidx.numel())
        self.edge_id_base = int(edge_id_base)
        self.self_id_base = self.nnz if self_id_base is None else int(self_id_base)
        self.self_rows = self.num_rows if self_rows is None else int(self_rows)
        self.batch_shape = batch_shape
        self.dropedge: Optional[DropEdge] = None
        self.split_threshold = SPLIT_THRESHOLD
        self.split_chunk = SPLIT_CHUNK
        self._shared = {"csc": None} if _shared is None else _shared

    # ------------------------------------------------------------------ views
    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    @property
    def segments(self) -> int:
        """Output segments per row of Z: identity + typed (L+1 in the reference)."""
        return self.num_types + (1 if self.has_self else 0)

    def with_dropedge(self, de: Optional[DropEdge]) -> "TypedGraph":
        """Shallow copy carrying a DropEdge draw (shares all device arrays and
        the CSC cache), i.e. the reference's edge_dropout(A)."""
        g = TypedGraph.__new__(TypedGraph)
        g.__dict__.update(self.__dict__)
        g.dropedge = de
        return g

    self_row0 = 0  # X row of row 0's identity term (row-range views, rows_view)
    # rows the GEMM path is chosen for (GrlTypedCsr.path_rows; 0 = num_rows): a
    # node-range shard carries the whole graph's row count, a row-range view its
    # parent's, so their rows take the one-GPU layer's path (bitwise its rows)
    path_rows = 0

    def rows_view(self, r0: int, r1: int) -> "TypedGraph":
        """Rows [r0, r1) as a forward graph of their own: rowptr a slice
        (edge positions, hence DropEdge ids, stay absolute), colidx / vals
        shared, the identity term from X row r0 on (GrlTypedCsr.self_row0)
        and its DropEdge ids from self_id_base + r0 -- every row exactly as in
        the whole graph.  Cached per graph; carries this graph's DropEdge
        draw.  Forward entry points only (no transpose of its own)."""
        if not 0 <= r0 <= r1 <= self.num_rows:
            raise _lib.GrlError(f"rows [{r0}, {r1}) outside [0, {self.num_rows})")
        cache = self._shared.setdefault("fwd_row_views", {})
        v = cache.get((r0, r1))
        if v is None:
            L = self.num_types
            v = TypedGraph(self.rowptr[r0 * L: r1 * L + 1], self.colidx, L, vals=self.vals, has_self=self.has_self,
                           num_cols=self.num_cols, edge_id_base=self.edge_id_base,
                           self_id_base=self.self_id_base + r0, self_rows=max(0, min(self.self_rows, r1) - r0))
            v.self_row0 = self.self_row0 + r0
            v.path_rows = self.path_rows or self.num_rows
            v.split_threshold, v.split_chunk = self.split_threshold, self.split_chunk
            cache[(r0, r1)] = v
        return v.with_dropedge(self.dropedge)

    def __repr__(self) -> str:
        return (f"TypedGraph(rows={self.num_rows}, cols={self.num_cols}, types={self.num_types}, "
                f"nnz={self.nnz}, has_self={self.has_self}, vals={'yes' if self.vals is not None else 'ones'}, "
                f"dropedge={self.dropedge})")

    # ----------------------------------------------------------- split plans
    def _split(self, which: str, F: int):
        """Cached heavy-row plan over rowptr ("csr") or colptr ("csc"), with
        its partials scratch grown to F floats per chunk; None if no row is
        heavier than the threshold."""
        key = f"split_{which}"
        if key not in self._shared:
            self._shared[key] = self._build_split(which)
        sp = self._shared[key]
        if sp is None:
            return None
        need = sp["plan"].num_chunks * F
        if sp["partials"] is None or sp["partials"].numel() < need:
            sp["partials"] = torch.empty(max(need, 1), dtype=torch.float32, device=self.device)
            sp["plan"].partials = sp["partials"].data_ptr()
            sp["plan"].partials_capacity = sp["partials"].numel()
        return sp["plan"]

    def _build_split(self, which: str):
        if self.nnz <= self.split_threshold:  # no row can be heavy: no device work, no sync
            return None
        if which == "csr":
            ptr, rows, nseg = self.rowptr, self.num_rows, self.num_types
        else:
            ptr, rows, nseg = self.csc()["colptr"], self.num_cols, 1
        dev = self.device
        stream = current_stream_handle(dev)
        ws_bytes = _lib.lib().grl_split_plan_workspace_size(rows)
        if ws_bytes == 0:
            raise _lib.GrlError("grl_split_plan_workspace_size failed")
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        counts = torch.zeros(2, dtype=torch.int64, device=dev)
        call("grl_split_plan_count", ptr.data_ptr(), rows, nseg, self.split_threshold, self.split_chunk,
             counts.data_ptr(), ws.data_ptr(), ws_bytes, stream)
        num_heavy, num_chunks = (int(x) for x in counts.tolist())
        if num_heavy == 0:
            return None
        t = {name: torch.empty(max(n, 1), dtype=torch.int32, device=dev)
             for name, n in (("heavy_seg", num_heavy), ("heavy_cptr", num_heavy + 1), ("chunk_begin", num_chunks),
                             ("chunk_end", num_chunks))}
        plan = GrlSplitPlan()
        plan.threshold, plan.chunk_edges = self.split_threshold, self.split_chunk
        plan.num_heavy, plan.num_chunks = num_heavy, num_chunks
        for name, tensor in t.items():
            setattr(plan, name, tensor.data_ptr())
        call("grl_split_plan_build", ptr.data_ptr(), rows, nseg, ctypes.byref(plan), ws.data_ptr(), ws_bytes, stream)
        return {"plan": plan, "tensors": t, "partials": None}

    def split_stats(self) -> dict:
        out = {}
        for which in ("csr", "csc"):
            self._split(which, 1)
            sp = self._shared.get(f"split_{which}")
            out[which] = {"heavy_segments": 0, "chunks": 0} if sp is None else {
                "heavy_segments": sp["plan"].num_heavy, "chunks": sp["plan"].num_chunks}
        return out

    # ------------------------------------------------------------ C structs
    def csr_c(self, F: Optional[int] = None) -> GrlTypedCsr:
        g = GrlTypedCsr()
        g.num_rows = self.num_rows
        g.num_types = self.num_types
        g.has_self = int(self.has_self)
        g.rowptr = self.rowptr.data_ptr()
        g.colidx = self.colidx.data_ptr() if self.nnz else None
        g.vals = self.vals.data_ptr() if self.vals is not None and self.nnz else None
        g.nnz = self.nnz
        g.edge_id_base = self.edge_id_base
        g.self_id_base = self.self_id_base
        g.self_row0 = self.self_row0
        g.path_rows = self.path_rows
        plan = self._split("csr", F) if F is not None else None
        g.split = ctypes.pointer(plan) if plan is not None else None
        return g

    def csc(self) -> dict:
        """CSC (colptr, zrow, eid, cvals), built once on the device and cached."""
        c = self._shared.get("csc")
        if c is not None:
            return c
        dev = self.device
        ws_bytes = _lib.lib().grl_csr_to_csc_workspace_size(self.nnz, self.num_cols)
        if ws_bytes == 0:
            raise _lib.GrlError("grl_csr_to_csc_workspace_size failed")
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        colptr = torch.empty(self.num_cols + 1, dtype=torch.int32, device=dev)
        n = max(self.nnz, 1)
        zrow = torch.empty(n, dtype=torch.int32, device=dev)
        eid = torch.empty(n, dtype=torch.int32, device=dev)
        cvals = torch.empty(n, dtype=torch.float32, device=dev) if self.vals is not None else None
        csr = self.csr_c()
        call("grl_csr_to_csc", ctypes.byref(csr), self.num_cols, colptr.data_ptr(), zrow.data_ptr(),
             eid.data_ptr(), cvals.data_ptr() if cvals is not None else None, ws.data_ptr(), ws_bytes,
             current_stream_handle(dev))
        c = {"colptr": colptr, "zrow": zrow, "eid": eid, "cvals": cvals}
        self._shared["csc"] = c
        return c

    @property
    def transpose_ok(self) -> bool:
        """False for a graph whose arrays are static buffers refilled in place
        (a captured training step's bucket, step_graph.py): a cached typed
        transpose would go stale, so the one-kernel data gradient is not
        used on it.  Nor for a row-range view (rows_view): no transpose of its
        own."""
        return not self._shared.get("static_buffers", False) and self.self_row0 == 0

    def typed_transpose(self):
        """(gt, eid): the typed transpose, built once and cached -- gt's row m
        (one per column of this graph: a shard's own and halo rows), segment
        t lists the forward rows n with a type-t edge n <- m, in forward-CSR
        order; eid[e] = entry e's forward CSR position (its DropEdge id minus
        edge_id_base); values follow.  It is the CSC builder (grl_csr_to_csc:
        a stable radix sort by column) run with the column of edge (n, t, m)
        keyed as m * L + t.  The one-kernel data gradient
        (grl_graphconv_bwd_data) runs the GraphConv forward kernel over it;
        rows m < num_rows carry the self term there."""
        tt = self._shared.get("typed_transpose")
        if tt is not None:
            return tt
        if not self.transpose_ok:
            raise _lib.GrlError("typed_transpose: this graph's arrays are refilled in place (static buffers); "
                                "a cached transpose would go stale")
        if self.self_rows != self.num_rows or self.num_cols < self.num_rows:
            raise _lib.GrlError("typed_transpose needs every row to own its self loop (self_rows == num_rows) and "
                                "the rows among the columns")
        L, S = self.num_types, self.segments
        if self.num_cols * L >= 2 ** 31:
            raise _lib.GrlError("typed_transpose: num_cols * num_types exceeds int32")
        seg = torch.arange(self.num_rows * L, dtype=torch.int32, device=self.device) % L
        t = torch.repeat_interleave(seg, self.rowptr.diff(), output_size=self.nnz)
        keyed = TypedGraph(self.rowptr, self.colidx * L + t, L, vals=self.vals, has_self=self.has_self,
                           num_cols=self.num_cols * L, edge_id_base=self.edge_id_base,
                           self_id_base=self.self_id_base, self_rows=self.self_rows)
        del seg, t
        c = keyed.csc()
        n = max(self.nnz, 1)
        gt = TypedGraph(c["colptr"], (c["zrow"][:n] // S).contiguous(), L, vals=c["cvals"], has_self=self.has_self,
                        num_cols=self.num_rows, edge_id_base=self.edge_id_base, self_id_base=self.self_id_base,
                        self_rows=self.num_rows) if self.nnz else None  # rows: self.num_cols
        if gt is None:  # no edges: every segment empty
            gt = TypedGraph(torch.zeros(self.num_cols * L + 1, dtype=torch.int32, device=self.device),
                            torch.zeros(0, dtype=torch.int32, device=self.device), L, has_self=self.has_self,
                            num_cols=self.num_rows, edge_id_base=self.edge_id_base, self_id_base=self.self_id_base,
                            self_rows=self.num_rows)
        gt.split_threshold, gt.split_chunk = self.split_threshold, self.split_chunk
        tt = (gt, c["eid"])
        self._shared["typed_transpose"] = tt
        return tt

    def csc_c(self, F: Optional[int] = None) -> GrlTypedCsc:
        c = self.csc()
        s = GrlTypedCsc()
        s.num_rows = self.num_cols
        s.self_rows = min(self.self_rows, self.num_cols)
        s.num_types = self.num_types
        s.has_self = int(self.has_self)
        s.colptr = c["colptr"].data_ptr()
        s.zrow = c["zrow"].data_ptr()
        s.eid = c["eid"].data_ptr()
        s.vals = c["cvals"].data_ptr() if c["cvals"] is not None else None
        s.nnz = self.nnz
        s.edge_id_base = self.edge_id_base
        s.self_id_base = self.self_id_base
        plan = self._split("csc", F) if F is not None else None
        s.split = ctypes.pointer(plan) if plan is not None else None
        return s

    # ----------------------------------------------------------- builders
    @classmethod
    def from_dense(cls, A: torch.Tensor, layout: str = "bnln", has_self: bool = True,
                   keep_values: Optional[bool] = None) -> "TypedGraph":
        """Dense adjacency -> TypedGraph on A's device.

        layout "bnln": the collate layout (B, N, L, N) the dataset emits
            (gnn/data_generator/data_process/graph_utils.py:782-834);
        layout "bnnl": the permuted (B, N, N, L) view GraphConv.forward takes
            (drop_robust_gcn.py:63, robust_gcn.py:32-37);
        layout "pre":  an already preprocessed A_pre (B, (L+1)N, N)
            (robust_gcn.py:71); its identity block becomes an ordinary typed
            segment (has_self=False, L+1 types) so arbitrary values, e.g. a
            dropout-scaled A_pre, are honoured exactly.
        keep_values None: store vals only if some nonzero differs from 1.
        """
        _require_device(A, "adjacency")
        if A.dtype != torch.float32:
            A = A.float()
        if layout == "bnln":
            B, N, L, N2 = A.shape
            sb, sn, st, sm = A.stride()
        elif layout == "bnnl":
            B, N, N2, L = A.shape
            sb, sn, sm, st = A.stride()
        elif layout == "pre":
            B, R, N = A.shape
            if R % N:
                raise _lib.GrlError(f"A_pre rows {R} not a multiple of N={N}")
            L = R // N
            N2 = N
            A = A.reshape(B, N, L, N)
            sb, sn, st, sm = A.stride()
            has_self = False
        else:
            raise _lib.GrlError(f"unknown adjacency layout {layout!r}")
        if N != N2:
            raise _lib.GrlError(f"adjacency is not square over nodes: {tuple(A.shape)}")
        dev = A.device
        stream = current_stream_handle(dev)
        strides = (ctypes.c_int64 * 4)(sb, sn, st, sm)
        rows = B * N * L
        ws_bytes = _lib.lib().grl_dense_to_csr_workspace_size(rows)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        rowptr = torch.empty(rows + 1, dtype=torch.int32, device=dev)
        call("grl_dense_to_csr_rowptr", A.data_ptr(), B, N, L, strides, rowptr.data_ptr(), ws.data_ptr(),
             ws_bytes, stream)
        nnz = int(rowptr[-1].item())
        colidx = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
        vals = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        call("grl_dense_to_csr_fill", A.data_ptr(), B, N, L, strides, rowptr.data_ptr(), colidx.data_ptr(),
             vals.data_ptr(), stream)
        colidx, vals = colidx[:nnz], vals[:nnz]
        if keep_values is None:
            keep_values = bool(nnz) and not bool((vals == 1.0).all().item())
        return cls(rowptr, colidx, L, vals=vals if keep_values else None, has_self=has_self,
                   num_cols=B * N, batch_shape=(B, N))

    @classmethod
    def from_csr_host(cls, rowptr, colidx, num_types: int, device, **kw) -> "TypedGraph":
        """From host (numpy / CPU tensor) CSR arrays."""
        rp = torch.as_tensor(rowptr, dtype=torch.int32).to(device)
        ci = torch.as_tensor(colidx, dtype=torch.int32).to(device)
        vals = kw.pop("vals", None)
        if vals is not None:
            vals = torch.as_tensor(vals, dtype=torch.float32).to(device)
        return cls(rp, ci, num_types, vals=vals, **kw)

    @staticmethod
    def _synth_spec(num_nodes, avg_deg, num_types, kind, seed, rb, re) -> GrlSynthSpec:
        spec = GrlSynthSpec()
        spec.kind = {"er": 0, "rmat": 1}[kind]
        spec.num_types = num_types
        spec.num_nodes = num_nodes
        spec.num_candidates = int(round(num_nodes * avg_deg))
        spec.seed = seed
        spec.row_begin, spec.row_end = rb, re
        return spec

    @staticmethod
    def synthetic_degrees(num_nodes: int, avg_deg: float, num_types: int = 6, *, kind: str = "er", seed: int = 0,
                          device="cuda") -> torch.Tensor:
        """Candidate out-degree of every node (before dedupe), int32 on device."""
        dev = torch.device(device)
        spec = TypedGraph._synth_spec(num_nodes, avg_deg, num_types, kind, seed, 0, num_nodes)
        deg = torch.zeros(num_nodes, dtype=torch.int32, device=dev)
        call("grl_synth_degrees", ctypes.byref(spec), deg.data_ptr(), current_stream_handle(dev))
        return deg

    @classmethod
    def synthetic(cls, num_nodes: int, avg_deg: float, num_types: int = 6, *, kind: str = "er", seed: int = 0,
                  row_range: Optional[Tuple[int, int]] = None, device="cuda") -> "TypedGraph":
        """Seeded synthetic typed graph: num_nodes*avg_deg
        candidate edges (src, type, dst), deduped.  kind "er" (uniform) or
        "rmat" (a,b,c,d = .57,.19,.19,.05, num_nodes = 2^scale).  row_range
        selects the node-range shard [begin, end) this rank owns; colidx stay
        global node ids."""
        dev = torch.device(device)
        rb, re = (0, num_nodes) if row_range is None else row_range
        spec = cls._synth_spec(num_nodes, avg_deg, num_types, kind, seed, rb, re)
        stream = current_stream_handle(dev)
        cnt_t = torch.zeros(1, dtype=torch.int64, device=dev)
        call("grl_synth_count", ctypes.byref(spec), cnt_t.data_ptr(), stream)
        count = int(cnt_t.item())
        ws_bytes = _lib.lib().grl_synth_workspace_size(ctypes.byref(spec), count)
        if ws_bytes == 0:
            raise _lib.GrlError("grl_synth_workspace_size failed")
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        rowptr = torch.empty((re - rb) * num_types + 1, dtype=torch.int32, device=dev)
        colidx = torch.empty(max(count, 1), dtype=torch.int32, device=dev)
        nnz_t = torch.zeros(1, dtype=torch.int64, device=dev)
        call("grl_synth_build", ctypes.byref(spec), count, rowptr.data_ptr(), colidx.data_ptr(), nnz_t.data_ptr(),
             ws.data_ptr(), ws_bytes, stream)
        nnz = int(nnz_t.item())
        colidx = colidx[:nnz].clone()
        del ws
        return cls(rowptr, colidx, num_types, has_self=True, num_cols=num_nodes)

    # -------------------------------------------------------------- helpers
    def to_host(self) -> dict:
        """numpy copies of the CSR arrays (tests / CPU baseline)."""
        return {"rowptr": self.rowptr.cpu().numpy(), "colidx": self.colidx.cpu().numpy(),
                "vals": None if self.vals is None else self.vals.cpu().numpy()}

    def dropedge_mask(self, de: DropEdge, id_base: int, count: int) -> torch.Tensor:
        keep = torch.empty(max(count, 1), dtype=torch.uint8, device=self.device)
        c = de.to_c()
        call("grl_dropedge_mask", ctypes.byref(c), id_base, count, keep.data_ptr(),
             current_stream_handle(self.device))
        return keep[:count]


# Edges per block of an EdgeBlockedGraph: the kernels index edges with 32-bit
# positions (4-byte rowptr, cheap address arithmetic on the hot path).
MAX_BLOCK_EDGES = 2**31 - 1


class EdgeBlockedGraph:
    """A typed graph with 2^31 or more edges (SURVEY.md §8(b) Dtypes row:
    "int64 rowptr when E >= 2^31"), held as consecutive row blocks of fewer
    than MAX_BLOCK_EDGES edges each.  Every block is a TypedGraph over rows
    [row0, row1) with an int32 rowptr relative to its first edge, global column
    ids, and edge_id_base = the block's first global CSR position, so DropEdge
    ids are the 64-bit global positions of one big CSR.  The forward runs one
    aggregation per block (grl_typed_spmm_fwd_slice, self rows at row0, Z
    rows at row0); the backward runs the blocks' CSCs in block order, the
    first with grl_typed_spmm_bwd, the rest with grl_typed_spmm_bwd_accum --
    the same fmaf chain per element as a single int64 CSR (heavy-row chunks
    are cut per block)."""

    def __init__(self, blocks, row_bounds, num_cols: int):
        self.blocks = list(blocks)
        self.row_bounds = list(row_bounds)  # [0, r1, r2, ..., num_rows]
        b0 = self.blocks[0]
        self.num_types, self.has_self = b0.num_types, b0.has_self
        self.num_rows = self.row_bounds[-1]
        self.num_cols = int(num_cols)
        self.nnz = sum(b.nnz for b in self.blocks)
        self.dropedge: Optional[DropEdge] = None

    @property
    def device(self) -> torch.device:
        return self.blocks[0].device

    @property
    def segments(self) -> int:
        return self.num_types + (1 if self.has_self else 0)

    def with_dropedge(self, de: Optional[DropEdge]) -> "EdgeBlockedGraph":
        g = EdgeBlockedGraph.__new__(EdgeBlockedGraph)
        g.__dict__.update(self.__dict__)
        g.blocks = [b.with_dropedge(de) for b in self.blocks]
        g.dropedge = de
        return g

    def __repr__(self) -> str:
        return (f"EdgeBlockedGraph(rows={self.num_rows}, cols={self.num_cols}, types={self.num_types}, "
                f"nnz={self.nnz}, blocks={len(self.blocks)}, dropedge={self.dropedge})")

    @classmethod
    def from_csr64(cls, rowptr: torch.Tensor, colidx: torch.Tensor, num_types: int, *, num_cols: Optional[int] = None,
                   has_self: bool = True, max_block_edges: int = MAX_BLOCK_EDGES) -> "EdgeBlockedGraph":
        """One typed CSR with an int64 rowptr [num_rows*num_types + 1] and
        int32 colidx, cut into row blocks of <= max_block_edges edges (a row
        with more edges than that is refused)."""
        _require_device(rowptr, "rowptr")
        if rowptr.dtype != torch.int64 or colidx.dtype != torch.int32:
            raise _lib.GrlError("from_csr64: rowptr must be int64 and colidx int32")
        L = int(num_types)
        num_rows = (rowptr.numel() - 1) // L
        node_ptr = rowptr[::L].contiguous()  # [num_rows + 1]
        nnz = int(node_ptr[-1])
        E_total = nnz
        bounds = [0]
        while bounds[-1] < num_rows:
            r0 = bounds[-1]
            limit = torch.tensor([int(node_ptr[r0]) + max_block_edges], dtype=torch.int64, device=rowptr.device)
            r1 = int(torch.searchsorted(node_ptr, limit, right=True)) - 1
            r1 = min(max(r1, r0), num_rows)
            if r1 == r0:
                raise _lib.GrlError(f"row {r0} alone holds more than {max_block_edges} edges")
            bounds.append(r1)
        blocks = []
        ncols = num_rows if num_cols is None else int(num_cols)
        for r0, r1 in zip(bounds[:-1], bounds[1:]):
            e0, e1 = int(node_ptr[r0]), int(node_ptr[r1])
            rp = (rowptr[r0 * L: r1 * L + 1] - e0).to(torch.int32)
            blocks.append(TypedGraph(rp, colidx[e0:e1], L, has_self=has_self, num_cols=ncols, edge_id_base=e0,
                                     self_id_base=E_total + r0, self_rows=r1 - r0))
        return cls(blocks, bounds, ncols)

    @classmethod
    def synthetic(cls, num_nodes: int, avg_deg: float, num_types: int = 6, *, kind: str = "er", seed: int = 0,
                  device="cuda", max_block_edges: int = MAX_BLOCK_EDGES) -> "EdgeBlockedGraph":
        """TypedGraph.synthetic's graph (same edges, same global order) built
        as row blocks, for edge counts beyond one int32 CSR: the blocks are
        row ranges holding <= max_block_edges candidate edges each."""
        deg = TypedGraph.synthetic_degrees(num_nodes, avg_deg, num_types, kind=kind, seed=seed, device=device)
        cum = torch.cumsum(deg.to(torch.int64), 0)
        bounds = [0]
        while bounds[-1] < num_nodes:
            r0 = bounds[-1]
            base = int(cum[r0 - 1]) if r0 else 0
            limit = torch.tensor([base + max_block_edges], dtype=torch.int64, device=cum.device)
            r1 = min(num_nodes, int(torch.searchsorted(cum, limit, right=True)))
            if r1 == r0:
                raise _lib.GrlError(f"node {r0} alone has more than {max_block_edges} candidate edges")
            bounds.append(r1)
        parts = [TypedGraph.synthetic(num_nodes, avg_deg, num_types, kind=kind, seed=seed, row_range=(a, b),
                                      device=device) for a, b in zip(bounds[:-1], bounds[1:])]
        E_total = sum(p.nnz for p in parts)
        blocks, e0 = [], 0
        for (a, b), p in zip(zip(bounds[:-1], bounds[1:]), parts):
            blocks.append(TypedGraph(p.rowptr, p.colidx, num_types, num_cols=num_nodes, edge_id_base=e0,
                                     self_id_base=E_total + a, self_rows=b - a))
            e0 += p.nnz
        return cls(blocks, bounds, num_nodes)


def degree_order(graph: TypedGraph) -> Tuple[TypedGraph, torch.Tensor]:
    """Relabel the nodes of a square typed graph by descending in-degree (how
    often a node is gathered as a source), keeping every row's edges in their
    order: returns (G', perm) with node i of G' = node perm[i] of G.

    For power-law graphs (R-MAT) the rows most often gathered then sit in one
    contiguous head of X (C5: the 43.5k sources behind half of all edges span
    85 MiB instead of pages all over a 17 GB table), which the Infinity Cache
    and the address-translation caches cover.  A one-time preprocessing step
    of the graph, like the CSC and the split plan: features go in permuted
    once (X' = X[perm]) and outputs come back once (Z[perm] = Z'); every layer
    in between runs on G'.  Z' rows are the same fmaf chains as G's rows
    (bitwise equal without DropEdge); DropEdge ids are G' CSR positions."""
    if graph.num_cols != graph.num_rows or graph.self_rows != graph.num_rows:
        raise _lib.GrlError("degree_order needs a square graph (one node set for rows and sources)")
    dev, L, N = graph.device, graph.num_types, graph.num_rows
    col = graph.colidx.long()
    indeg = torch.bincount(col, minlength=N)
    perm = torch.sort(indeg, descending=True, stable=True).indices
    rank = torch.empty_like(perm)
    rank[perm] = torch.arange(N, device=dev)
    rp = graph.rowptr.long()
    seglen = (rp[1:] - rp[:-1]).view(N, L)[perm]                      # new row i = old row perm[i]
    new_rp = torch.zeros(N * L + 1, dtype=torch.int64, device=dev)
    torch.cumsum(seglen.reshape(-1), 0, out=new_rp[1:])
    row_len = seglen.sum(1)
    old_start = rp[perm * L]
    new_start = new_rp[:-1:L]
    pos = torch.arange(graph.nnz, dtype=torch.int64, device=dev)
    pos += torch.repeat_interleave(old_start - new_start, row_len, output_size=graph.nnz)
    colidx = rank[col[pos]].to(torch.int32)
    vals = None if graph.vals is None else graph.vals[pos]
    del pos
    g2 = TypedGraph(new_rp.to(torch.int32), colidx, L, vals=vals, has_self=graph.has_self, num_cols=N)
    g2.split_threshold, g2.split_chunk = graph.split_threshold, graph.split_chunk
    return g2, perm
