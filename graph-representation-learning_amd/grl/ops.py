"""Autograd ops over the libgrl kernels.

  typed_aggregate(X, graph)   Z = A_drop X           robust_gcn.py:45-47
                              (+ edge_dropout, drop_robust_gcn.py:76,80,85)
  graph_linear(Z, W, b, relu) out = Z W + b [ReLU]    robust_gcn.py:50
                              (+ F.relu, drop_robust_gcn.py:76,80,85)

Both run on the current torch HIP stream; backward regenerates the DropEdge
mask from the graph's (p, seed, call) record, exactly like forward.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call
from .graph import EdgeBlockedGraph, TypedGraph, _require_device, current_stream_handle


def _rows_view(X: torch.Tensor) -> torch.Tensor:
    """2-D row view with unit column stride (no copy when possible)."""
    X2 = X.reshape(-1, X.shape[-1])
    if X2.stride(-1) != 1:
        X2 = X2.contiguous()
    return X2


def spmm_forward(X: torch.Tensor, graph: TypedGraph, out: torch.Tensor = None) -> torch.Tensor:
    """Z = A_drop X without autograd bookkeeping, optionally into `out`
    (contiguous [num_rows, segments*F] fp32): the inference / benchmark form."""
    if isinstance(graph, EdgeBlockedGraph):
        return _blocked_forward(X, graph, out)
    _require_device(X, "node features")
    if X.dtype != torch.float32:
        raise _lib.GrlError(f"node features must be float32 (got {X.dtype})")
    X2 = _rows_view(X)
    if X2.shape[0] != graph.num_cols:
        raise _lib.GrlError(f"features have {X2.shape[0]} rows, graph gathers from {graph.num_cols}")
    F = X2.shape[1]
    shape = (graph.num_rows, graph.segments * F)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=X.device)
    elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous() \
            or out.device != X.device:
        raise _lib.GrlError(f"out must be a contiguous float32 {shape} tensor on {X.device}")
    csr = graph.csr_c(F)
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_typed_spmm_fwd", ctypes.byref(csr), X2.data_ptr(), X2.stride(0), F, out.data_ptr(),
         ctypes.byref(de) if de is not None else None, current_stream_handle(X.device))
    return out


def spmm_forward_slice(X: torch.Tensor, graph: TypedGraph, out: torch.Tensor, col0: int,
                       self_col0: int = 0) -> torch.Tensor:
    """Columns [col0, col0 + F) of Z = A_drop X into `out` (contiguous
    [num_rows, segments * F_total]), where X is that column slice's table
    ([graph.num_cols, F], any row stride) and row n's self term reads X row
    self_col0 + n (grl_typed_spmm_fwd_slice).  Bitwise equal, per element,
    to the whole-width spmm_forward: the pipelined halo exchange of grl.dist
    aggregates one slice while the next is in flight."""
    _require_device(X, "node features")
    if X.dtype != torch.float32 or X.dim() != 2 or X.stride(1) != 1:
        raise _lib.GrlError("slice table must be a 2-D float32 tensor with unit column stride")
    if X.shape[0] != graph.num_cols:
        raise _lib.GrlError(f"slice table has {X.shape[0]} rows, graph gathers from {graph.num_cols}")
    F = X.shape[1]
    S = graph.segments
    if out.dtype != torch.float32 or not out.is_contiguous() or out.shape[0] != graph.num_rows \
            or out.shape[1] % S or out.device != X.device:
        raise _lib.GrlError(f"out must be a contiguous float32 [{graph.num_rows}, {S} x F_total] tensor")
    zseg = out.shape[1] // S
    if col0 < 0 or col0 + F > zseg:
        raise _lib.GrlError(f"columns [{col0}, {col0 + F}) outside the {zseg}-column segments")
    csr = graph.csr_c(F)
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_typed_spmm_fwd_slice", ctypes.byref(csr), X.data_ptr(), X.stride(0), F, int(self_col0),
         out.data_ptr() + 4 * col0, out.stride(0), zseg, ctypes.byref(de) if de is not None else None,
         current_stream_handle(X.device))
    return out


def _blocked_forward(X: torch.Tensor, graph: EdgeBlockedGraph, out: torch.Tensor = None) -> torch.Tensor:
    """Z of a graph with >= 2^31 edges: one aggregation per row block (self
    rows at the block's first row, Z rows likewise)."""
    X2 = _rows_view(X)
    if X2.shape[0] != graph.num_cols:
        raise _lib.GrlError(f"features have {X2.shape[0]} rows, graph gathers from {graph.num_cols}")
    F = X2.shape[1]
    shape = (graph.num_rows, graph.segments * F)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=X.device)
    elif tuple(out.shape) != shape or not out.is_contiguous() or out.dtype != torch.float32:
        raise _lib.GrlError(f"out must be a contiguous float32 {shape} tensor")
    for blk, r0, r1 in zip(graph.blocks, graph.row_bounds[:-1], graph.row_bounds[1:]):
        spmm_forward_slice(X2, blk, out[r0:r1], 0, self_col0=r0)
    return out


def _blocked_backward(dZ: torch.Tensor, graph: EdgeBlockedGraph, F: int) -> torch.Tensor:
    """dX of a graph with >= 2^31 edges: the blocks' CSCs in block order --
    the first with the self term over every row, the rest continuing each
    column's sum (grl_typed_spmm_bwd_accum)."""
    dZ = dZ.contiguous().float()
    dX = torch.empty(graph.num_cols, F, dtype=torch.float32, device=dZ.device)
    stream = current_stream_handle(dZ.device)
    ldz = graph.segments * F
    for i, (blk, r0) in enumerate(zip(graph.blocks, graph.row_bounds[:-1])):
        csc = blk.csc_c(F)
        if i == 0:
            csc.self_rows = min(graph.num_rows, graph.num_cols)  # every node's self loop, dZ rows from 0
        de = blk.dropedge.to_c() if blk.dropedge is not None else None
        call("grl_typed_spmm_bwd" if i == 0 else "grl_typed_spmm_bwd_accum", ctypes.byref(csc),
             dZ.data_ptr() + 4 * r0 * ldz, F, dX.data_ptr(), F, ctypes.byref(de) if de is not None else None, stream)
    return dX


def spmm_backward(dZ: torch.Tensor, graph: TypedGraph, F: int) -> torch.Tensor:
    """dX = A_drop^T dZ (grl_typed_spmm_bwd over the cached CSC, same mask)."""
    if isinstance(graph, EdgeBlockedGraph):
        return _blocked_backward(dZ, graph, F)
    dZ = dZ.contiguous().float()
    dX = torch.empty(graph.num_cols, F, dtype=torch.float32, device=dZ.device)
    csc = graph.csc_c(F)
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_typed_spmm_bwd", ctypes.byref(csc), dZ.data_ptr(), F, dX.data_ptr(), F,
         ctypes.byref(de) if de is not None else None, current_stream_handle(dZ.device))
    return dX


def spmm_backward_slice(dZ: torch.Tensor, graph: TypedGraph, col0: int, out: torch.Tensor) -> torch.Tensor:
    """Columns [col0, col0 + F) of dX = A_drop^T dZ into `out` ([graph.num_cols,
    F] float32, unit column stride, any row stride), dZ contiguous
    [num_rows, segments * F_total] (grl_typed_spmm_bwd_slice).  Bitwise equal,
    per element, to spmm_backward: the pipelined backward of grl.dist sends
    one slice's halo-row gradients home while the next slice gathers."""
    if isinstance(graph, EdgeBlockedGraph):
        raise _lib.GrlError("column-slice backward takes a TypedGraph (edge-blocked graphs: spmm_backward)")
    _require_device(dZ, "dZ")
    if dZ.dtype != torch.float32 or not dZ.is_contiguous() or dZ.dim() != 2 or dZ.shape[0] != graph.num_rows \
            or dZ.shape[1] % graph.segments:
        raise _lib.GrlError(f"dZ must be a contiguous float32 [{graph.num_rows}, {graph.segments} x F_total] tensor")
    F_total = dZ.shape[1] // graph.segments
    if out.dtype != torch.float32 or out.dim() != 2 or out.stride(1) != 1 or out.shape[0] != graph.num_cols \
            or out.device != dZ.device:
        raise _lib.GrlError(f"out must be a float32 [{graph.num_cols}, F] tensor with unit column stride")
    F = out.shape[1]
    csc = graph.csc_c(F)
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_typed_spmm_bwd_slice", ctypes.byref(csc), dZ.data_ptr(), F_total, int(col0), F, out.data_ptr(),
         out.stride(0), ctypes.byref(de) if de is not None else None, current_stream_handle(dZ.device))
    return out


class _TypedAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X: torch.Tensor, graph: TypedGraph) -> torch.Tensor:
        Z = spmm_forward(X, graph)
        ctx.graph = graph
        ctx.xshape = X.shape
        return Z

    @staticmethod
    def backward(ctx, dZ: torch.Tensor):
        return spmm_backward(dZ, ctx.graph, ctx.xshape[-1]).view(ctx.xshape), None


def typed_aggregate(X: torch.Tensor, graph: TypedGraph) -> torch.Tensor:
    """Z[n, s*F:(s+1)*F]: segment 0 = own row (identity block), segment 1+t =
    sum over type-t neighbours; rows of X = graph.num_cols."""
    return _TypedAggregate.apply(X, graph)


# Row count from which the backward applies the ReLU mask to g once
# (torch.where, one elementwise pass) instead of inside the GEMM loads, so the
# two backward GEMMs qualify for libgrl's large-tile LDS-DMA path (which
# streams operands straight into LDS and cannot mask on the way).
PREMASK_ROWS = 65536


def relu_grad(g: torch.Tensor, out, want_db: bool = False):
    """(g_eff, mask_for_the_gemm, db): g through ReLU's derivative [out > 0].
    From PREMASK_ROWS rows the mask is applied here, in one pass
    (grl_relu_grad) that also sums db when asked -- bitwise the db
    linear_bwd_weight would give on g_eff; otherwise db is None and the GEMM
    (which then masks on its loads) gives it."""
    if out is None:
        return g, None, None
    if g.shape[0] < PREMASK_ROWS:
        return g, out, None
    _require_device(g, "relu_grad g")
    M, C = g.shape
    if out.shape != g.shape or not out.is_contiguous() or not g.is_contiguous():
        raise _lib.GrlError(f"relu_grad: g {tuple(g.shape)} and the ReLU output {tuple(out.shape)} "
                            "must be contiguous and of one shape")
    g_eff = torch.empty_like(g)
    db = torch.empty(C, dtype=torch.float32, device=g.device) if want_db else None
    ws_bytes = _lib.lib().grl_relu_grad_workspace_size(M, C) if want_db else 0
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device) if ws_bytes else None
    call("grl_relu_grad", g.data_ptr(), out.data_ptr(), g_eff.data_ptr(), db.data_ptr() if db is not None else None,
         M, C, ws.data_ptr() if ws is not None else None, ws_bytes, current_stream_handle(g.device))
    return g_eff, None, db


def linear_fwd(Z2: torch.Tensor, W: torch.Tensor, b, relu: bool) -> torch.Tensor:
    M, K = Z2.shape
    C = W.shape[1]
    out = torch.empty(M, C, dtype=torch.float32, device=Z2.device)
    ws_bytes = _lib.lib().grl_linear_fwd_workspace_size(M, K, C)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=Z2.device) if ws_bytes else None
    call("grl_linear_fwd", Z2.data_ptr(), Z2.stride(0), W.data_ptr(), b.data_ptr() if b is not None else None,
         out.data_ptr(), M, K, C, int(relu), ws.data_ptr() if ws is not None else None, ws_bytes,
         current_stream_handle(Z2.device))
    return out


def linear_bwd_data(g: torch.Tensor, relu_out, W: torch.Tensor) -> torch.Tensor:
    M, C = g.shape
    K = W.shape[0]
    dZ = torch.empty(M, K, dtype=torch.float32, device=g.device)
    ws_bytes = _lib.lib().grl_linear_bwd_data_workspace_size(M, K, C)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device) if ws_bytes else None
    call("grl_linear_bwd_data", g.data_ptr(), relu_out.data_ptr() if relu_out is not None else None, W.data_ptr(),
         dZ.data_ptr(), K, M, K, C, ws.data_ptr() if ws is not None else None, ws_bytes,
         current_stream_handle(g.device))
    return dZ


def linear_bwd_weight(Z2: torch.Tensor, g: torch.Tensor, relu_out, want_db: bool):
    M, K = Z2.shape
    C = g.shape[1]
    dW = torch.empty(K, C, dtype=torch.float32, device=g.device)
    db = torch.empty(C, dtype=torch.float32, device=g.device) if want_db else None
    ws_bytes = _lib.lib().grl_linear_bwd_weight_workspace_size(M, K, C)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device)
    call("grl_linear_bwd_weight", Z2.data_ptr(), Z2.stride(0), g.data_ptr(),
         relu_out.data_ptr() if relu_out is not None else None, dW.data_ptr(),
         db.data_ptr() if db is not None else None, M, K, C, ws.data_ptr(), ws_bytes,
         current_stream_handle(g.device))
    return dW, db


class _GraphLinear(torch.autograd.Function):
    """out = Z W + b [ReLU]; backward on the same MFMA GEMM kernel with the
    ReLU mask fused into the operand loads (no g*mask temporary)."""

    @staticmethod
    def forward(ctx, Z: torch.Tensor, W: torch.Tensor, b, relu: bool, path_rows: int = 0):
        Z2 = _rows_view(Z)
        Wc = W.contiguous()
        bc = b.contiguous() if b is not None else None
        # path_rows > 0: the GEMM path chosen for that many rows (a node-range
        # shard's whole graph), so the shard's rows are the one-GPU layer's bits
        out = linear_fwd_ex(Z2, Wc, 0, bc, relu, path_rows) if path_rows > 0 else linear_fwd(Z2, Wc, bc, relu)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.save_for_backward(Z2, Wc, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        Z2, W, out = ctx.saved_tensors
        want_b = ctx.has_b and ctx.needs_input_grad[2]
        g, mask, db_pre = relu_grad(g.contiguous().float(), out if ctx.relu else None, want_b)
        dZ = dW = db = None
        if ctx.needs_input_grad[0]:
            dZ = linear_bwd_data(g, mask, W)
        if ctx.needs_input_grad[1] or (want_b and db_pre is None):
            dW, db = linear_bwd_weight(Z2, g, mask, want_b and db_pre is None)
            if not ctx.needs_input_grad[1]:
                dW = None
        return dZ, dW, db_pre if db_pre is not None else db, None, None


# Widths of the one-kernel GraphConv (graphconv.hip): the gathered width (the
# forward's F, or the data gradient's C) and the largest output width of one
# call (the forward's C, or the data gradient's F; wider dX runs in column
# blocks).
FUSED_WIDTHS = (64, 128, 256, 512, 1024)
FUSED_MAX_OUT = 512


def x6_rows_ok(M: int, N: int, K: int, path_rows: int = 0) -> bool:
    """Whether an [M, K] x [K, N] product, chosen for max(M, path_rows) rows,
    takes the split-bf16 GEMM (and so a GraphConv the one-kernel forms): the
    size rule of x6_path_ok (csrc/linear.hip).  Both GEMM paths' per-element
    arithmetic is independent of M (the fp32 one sums K in fixed chunks), so
    row blocks of one layer match the whole call bitwise when both take the
    same path -- which path_rows (the whole call's rows) guarantees."""
    rows = max(M, path_rows)
    return (_lib.get_option("gemm_x6") != 0 and K > 0 and K % 16 == 0 and M >= 1 and rows >= 4
            and N >= 4 and 2.0 * rows * N * K >= 1.6e10)


def _bwd_data_enabled() -> bool:
    return _lib.get_option("graphconv_fused_bwd") != 0


def graph_conv_bwd_data(g: torch.Tensor, graph: TypedGraph, W: torch.Tensor, F: int, relu_out=None,
                        want_aggregate: bool = False):
    """dX of one GraphConv layer in one kernel (grl_graphconv_bwd_data):
    dX = sum_s (A_drop,s^T g) W_s^T over the graph's typed transpose, for g
    the output gradient ([num_rows, C]; through the ReLU's [relu_out > 0]
    when relu_out is given).  F > 512 (gcn3's 2C-wide input at C = 512) runs
    one call per <= 512-column block of dX (the gather repeats per block; dZ
    still never exists).  None when the shape is outside the one-kernel path (the caller
    then runs dZ = g W^T and the CSC gather).  The graphconv_fused_bwd path
    option 0 disables it.  want_aggregate: return (dX, G_agg, g_eff) with G_agg =
    [A_drop,s^T g_eff]_s ([num_cols, segments * C], written by the same
    kernel) and g_eff the gradient through the ReLU, for dW_s = X^T G_agg_s."""
    if not _bwd_data_enabled() or isinstance(graph, EdgeBlockedGraph) or not graph.transpose_ok:
        return None
    M, C = g.shape
    L, S = graph.num_types, graph.segments
    nblk = -(-F // FUSED_MAX_OUT)
    wblk = (-(-F // nblk) + 3) // 4 * 4 if nblk > 1 else F  # block width, a multiple of 4
    bounds = [(f0, min(F, f0 + wblk)) for f0 in range(0, F, wblk)]
    # cheap pre-checks before the (cached, once per graph) transpose build; the library decides
    if (C not in FUSED_WIDTHS or F % 4 or F > 2 * FUSED_MAX_OUT or L > 7 or graph.num_cols < graph.num_rows
            or graph.self_rows != graph.num_rows or M != graph.num_rows
            or 2.0 * graph.num_cols * S * C * min(b - a for a, b in bounds) < 1.6e10
            or g.dtype != torch.float32 or not g.is_contiguous() or W.dtype != torch.float32
            or tuple(W.shape) != (S * F, C)):
        return None
    gt, eid = graph.typed_transpose()
    gt = gt.with_dropedge(graph.dropedge)
    csr = gt.csr_c(C)
    ws_bytes = _lib.lib().grl_graphconv_bwd_data_workspace_query(ctypes.byref(csr), g.data_ptr(), g.stride(0), C,
                                                                 W.data_ptr(), bounds[0][1])
    if ws_bytes == 0:
        return None
    if relu_out is not None:
        g = torch.where(relu_out > 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device)
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    stream = current_stream_handle(g.device)
    rows = graph.num_cols  # dX rows: every column of the graph (a shard's halo rows get partials)
    dX = torch.empty(rows, F, dtype=torch.float32, device=g.device)
    G_agg = torch.empty(rows, S * C, dtype=torch.float32, device=g.device) if want_aggregate else None
    for i, (f0, f1) in enumerate(bounds):
        w = f1 - f0
        Wb = W.contiguous() if len(bounds) == 1 else W.reshape(S, F, C)[:, f0:f1, :].reshape(S * w, C).contiguous()
        out = dX if len(bounds) == 1 else torch.empty(rows, w, dtype=torch.float32, device=g.device)
        call("grl_graphconv_bwd_data", ctypes.byref(csr), eid.data_ptr(), g.data_ptr(), g.stride(0), M, C,
             Wb.data_ptr(), w, out.data_ptr(), G_agg.data_ptr() if G_agg is not None and i == 0 else None,
             ctypes.byref(de) if de is not None else None, ws.data_ptr(), ws_bytes, stream)
        if len(bounds) > 1:
            dX[:, f0:f1] = out
    return (dX, G_agg, g) if want_aggregate else dX


def _transpose_rows_view(gt: TypedGraph, r0: int, r1: int, dropedge) -> TypedGraph:
    """Rows [r0, r1) of the typed transpose as a TypedGraph (rowptr a slice,
    colidx / vals / eid shared), cached on the transpose so its split plan is
    built once per graph, not once per backward."""
    cache = gt._shared.setdefault("row_views", {})
    v = cache.get((r0, r1))
    if v is None:
        L = gt.num_types
        v = TypedGraph(gt.rowptr[r0 * L: r1 * L + 1], gt.colidx, L, vals=gt.vals, has_self=gt.has_self,
                       num_cols=gt.num_cols, edge_id_base=gt.edge_id_base, self_id_base=gt.self_id_base,
                       self_rows=r1 - r0)
        v.split_threshold, v.split_chunk = gt.split_threshold, gt.split_chunk
        cache[(r0, r1)] = v
    return v.with_dropedge(dropedge)


def graph_conv_bwd_data_rows_views(g: torch.Tensor, graph: TypedGraph, W: torch.Tensor, F: int, blocks):
    """The per-block launch data of graph_conv_bwd_data_rows -- [(view, csr,
    workspace bytes) or None for an empty block] -- or None when some block
    is outside the one-kernel path.  No device work beyond the cached
    transpose and split plans: a caller that must decide collectively
    (grl.dist rows_backward) asks this first, agrees, then launches."""
    if not _bwd_data_enabled() or isinstance(graph, EdgeBlockedGraph) or not graph.transpose_ok:
        return None
    M, C = g.shape
    L, S = graph.num_types, graph.segments
    if (C not in FUSED_WIDTHS or F % 4 or F > FUSED_MAX_OUT or L > 7 or graph.num_cols < graph.num_rows
            or graph.self_rows != graph.num_rows or M != graph.num_rows or g.dtype != torch.float32
            or not g.is_contiguous() or W.dtype != torch.float32 or tuple(W.shape) != (S * F, C)):
        return None
    for r0, r1 in blocks:
        if not (r0 == 0 or r0 >= graph.num_rows) or r1 < r0 or r1 > graph.num_cols:
            raise _lib.GrlError(f"row block [{r0}, {r1}) must start at 0 or at/after row {graph.num_rows}")
    gt, eid = graph.typed_transpose()
    Wc = W.contiguous()
    views = []
    for r0, r1 in blocks:
        if r1 == r0:
            views.append(None)
            continue
        v = _transpose_rows_view(gt, r0, r1, graph.dropedge)
        csr = v.csr_c(C)
        ws_bytes = _lib.lib().grl_graphconv_bwd_data_workspace_query(ctypes.byref(csr), g.data_ptr(), g.stride(0),
                                                                     C, Wc.data_ptr(), F)
        if ws_bytes == 0:
            return None
        views.append((v, csr, ws_bytes))
    return views


def graph_conv_bwd_data_rows(g: torch.Tensor, graph: TypedGraph, W: torch.Tensor, F: int, blocks, dX: torch.Tensor,
                             on_block=None, views=None) -> bool:
    """The one-kernel data gradient (graph_conv_bwd_data) computed in row
    blocks of dX, one grl_graphconv_bwd_data call per block [r0, r1) over a
    row-range view of the cached typed transpose, so a caller can act on a
    block (e.g. send a node-range shard's halo rows home) while the next one
    computes.  Every row is the same arithmetic as in the whole-range call
    (rows do not mix in the kernel), so dX is bitwise that call's.  A block
    starting at row 0 carries the self term of rows < graph.num_rows; other
    blocks must lie at or beyond num_rows (a shard's halo rows: no self term).
    g: the output gradient already through the ReLU.  dX: [graph.num_cols, F]
    (written).  on_block(r0, r1) runs after each block's launch.  views:
    graph_conv_bwd_data_rows_views' result for these arguments (else it is
    computed here).  False (and nothing written) when some block is outside
    the one-kernel path; the caller then takes the whole-range path."""
    if views is None:
        views = graph_conv_bwd_data_rows_views(g, graph, W, F, blocks)
    if views is None or tuple(dX.shape) != (graph.num_cols, F) or not dX.is_contiguous():
        return False
    gt, eid = graph.typed_transpose()
    Wc = W.contiguous()
    M, C = g.shape
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    stream = current_stream_handle(g.device)
    ws = None
    for (r0, r1), view in zip(blocks, views):
        if view is not None:
            v, csr, ws_bytes = view
            if ws is None or ws.numel() < ws_bytes:
                ws = torch.empty(ws_bytes, dtype=torch.uint8, device=g.device)
            g_rows = M if r0 == 0 else 0  # the self term: forward rows only
            call("grl_graphconv_bwd_data", ctypes.byref(csr), eid.data_ptr(), g.data_ptr(), g.stride(0),
                 min(g_rows, r1 - r0), C, Wc.data_ptr(), F, dX[r0:r1].data_ptr(), None,
                 ctypes.byref(de) if de is not None else None, ws.data_ptr(), ws_bytes, stream)
        if on_block is not None:
            on_block(r0, r1)
    return True


class _GraphConv(torch.autograd.Function):
    """One GraphConv layer, X -> Z = A_drop X -> out = Z W + b [ReLU]
    (robust_gcn.py:45-51), as one autograd node: the same kernels and
    results as typed_aggregate + graph_linear.  (Running dW on a second HIP
    stream beside dZ / the transposed gather was measured and bought nothing:
    39-41 ms per C3 layer either way, each kernel already fills the chip.)"""

    @staticmethod
    def forward(ctx, X: torch.Tensor, graph: TypedGraph, W: torch.Tensor, b, relu: bool, recompute: bool):
        Wc = W.contiguous()
        bc = b.contiguous() if b is not None else None
        if isinstance(graph, EdgeBlockedGraph):
            Z = spmm_forward(X, graph)
            out = linear_fwd(Z, Wc, bc, relu)
        elif recompute:  # Z is not kept: the one-kernel inference form (Z stays on chip)
            Z = None
            out = graph_conv_infer(X, graph, Wc, bc, relu)
        else:  # one kernel that also writes Z where it applies (grl_graphconv_fwd_train)
            out, Z = graph_conv_fwd_train(X, graph, Wc, bc, relu)
        ctx.graph, ctx.relu, ctx.has_b, ctx.xshape = graph, relu, b is not None, X.shape
        ctx.recompute = recompute
        # recompute: keep X (F wide) instead of Z ((L+1)F wide); the backward
        # regenerates Z with the same DropEdge record, so it is the same bits
        ctx.save_for_backward(X if recompute else Z, Wc, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        Z, W, out = ctx.saved_tensors
        want_w = ctx.needs_input_grad[2]
        want_b = ctx.has_b and ctx.needs_input_grad[3]
        g, mask, db_pre = relu_grad(g.contiguous().float(), out if ctx.relu else None, want_b)
        if ctx.recompute and ctx.needs_input_grad[0] and want_w:
            # X was kept, not Z: the one-kernel data gradient also writes G_s = A_drop,s^T g and
            # dW_s = Z_s^T g = X^T G_s -- no re-aggregation of Z (same products, another order)
            res = graph_conv_bwd_data(g, ctx.graph, W, ctx.xshape[-1], mask, want_aggregate=True)
            if res is not None:
                dX, G_agg, g_eff = res
                X2 = _rows_view(Z)
                S, F, C = ctx.graph.segments, X2.shape[1], g.shape[1]
                dWt, _ = linear_bwd_weight(X2, G_agg, None, False)  # [F, S*C]
                del G_agg
                dW = dWt.view(F, S, C).transpose(0, 1).reshape(S * F, C)
                db = (db_pre if db_pre is not None else g_eff.sum(0)) if want_b else None
                return dX.view(ctx.xshape), None, dW, db, None, None
        if ctx.recompute and (want_w or (want_b and db_pre is None)):
            Z = spmm_forward(Z, ctx.graph)
        dW = db = dX = None
        if ctx.needs_input_grad[0]:
            F = ctx.xshape[-1]
            dX = graph_conv_bwd_data(g, ctx.graph, W, F, mask)  # one kernel, no dZ (large graphs)
            if dX is None:
                dZ = linear_bwd_data(g, mask, W)
                dX = spmm_backward(dZ, ctx.graph, F)
                del dZ
            dX = dX.view(ctx.xshape)
        if want_w or (want_b and db_pre is None):
            dW, db = linear_bwd_weight(Z, g, mask, want_b and db_pre is None)
        if db_pre is not None:
            db = db_pre
        return dX, None, dW if want_w else None, db, None, None


def graph_conv_fwd_train(X: torch.Tensor, graph: TypedGraph, W: torch.Tensor, b=None, relu: bool = False,
                         out: torch.Tensor = None, Z: torch.Tensor = None):
    """(out, Z) of one GraphConv layer through grl_graphconv_fwd_train: the
    one-kernel path writes Z as a by-product (for the backward's dW); the
    result is bitwise spmm_forward then linear_fwd.  out / Z: contiguous
    [num_rows, C] / [num_rows, segments * F] fp32 tensors to write (e.g. the
    row block of a streamed layer)."""
    _require_device(X, "node features")
    if X.dtype != torch.float32 or W.dtype != torch.float32:
        raise _lib.GrlError("graph_conv_fwd_train: features and weights must be float32")
    X2 = _rows_view(X)
    if X2.shape[0] != graph.num_cols:
        raise _lib.GrlError(f"features have {X2.shape[0]} rows, graph gathers from {graph.num_cols}")
    F = X2.shape[1]
    Wc = W.contiguous()
    C = Wc.shape[1]
    K = graph.segments * F
    if Wc.shape[0] != K:
        raise _lib.GrlError(f"weights have {Wc.shape[0]} rows, expected {graph.segments} x {F}")
    bc = b.contiguous() if b is not None else None
    for t, shape, what in ((out, (graph.num_rows, C), "out"), (Z, (graph.num_rows, K), "Z")):
        if t is not None and (tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous()):
            raise _lib.GrlError(f"graph_conv_fwd_train: {what} must be a contiguous float32 {shape} tensor")
    if out is None:
        out = torch.empty(graph.num_rows, C, dtype=torch.float32, device=X.device)
    if Z is None:
        Z = torch.empty(graph.num_rows, K, dtype=torch.float32, device=X.device)
    csr = graph.csr_c(F)
    ws_bytes = _lib.lib().grl_linear_fwd_ex_workspace_size(graph.num_rows, K, C, graph.path_rows)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=X.device) if ws_bytes else None
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_graphconv_fwd_train", ctypes.byref(csr), X2.data_ptr(), X2.stride(0), F, Wc.data_ptr(),
         bc.data_ptr() if bc is not None else None, C, int(relu), out.data_ptr(), Z.data_ptr(),
         ctypes.byref(de) if de is not None else None, ws.data_ptr() if ws is not None else None, ws_bytes,
         current_stream_handle(X.device))
    return out, Z


def graph_conv_infer(X: torch.Tensor, graph: TypedGraph, W: torch.Tensor, b=None, relu: bool = False,
                     max_workspace_bytes: int = None, out: torch.Tensor = None) -> torch.Tensor:
    """GraphConv forward for inference through one grl_graphconv_fwd call
    (aggregation + linear [+ReLU]).  On large graphs this is one fused kernel
    and Z never reaches HBM; otherwise Z lives only in the call's workspace
    and max_workspace_bytes bounds it (the call then works in row chunks,
    bitwise equal to the whole-graph result).  out: a contiguous
    [num_rows, C] float32 tensor to write (e.g. a row block of a halo table)."""
    _require_device(X, "node features")
    if X.dtype != torch.float32 or W.dtype != torch.float32:
        raise _lib.GrlError("graph_conv_infer: features and weights must be float32")
    X2 = _rows_view(X)
    if X2.shape[0] != graph.num_cols:
        raise _lib.GrlError(f"features have {X2.shape[0]} rows, graph gathers from {graph.num_cols}")
    F = X2.shape[1]
    Wc = W.contiguous()
    C = Wc.shape[1]
    if Wc.shape[0] != graph.segments * F:
        raise _lib.GrlError(f"weights have {Wc.shape[0]} rows, expected {graph.segments} x {F}")
    bc = b.contiguous() if b is not None else None
    if out is None:
        out = torch.empty(graph.num_rows, C, dtype=torch.float32, device=X.device)
    elif (tuple(out.shape) != (graph.num_rows, C) or out.dtype != torch.float32 or not out.is_contiguous()
          or out.device != X.device):
        raise _lib.GrlError(f"out must be a contiguous float32 ({graph.num_rows}, {C}) tensor on {X.device}")
    csr = graph.csr_c(F)
    # the fused one-kernel path needs only W's planes; else Z whole
    full = _lib.lib().grl_graphconv_fwd_workspace_query(ctypes.byref(csr), X2.data_ptr(), X2.stride(0), F,
                                                         Wc.data_ptr(), C)
    ws_bytes = full if max_workspace_bytes is None else min(full, int(max_workspace_bytes))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=X.device) if ws_bytes else None
    de = graph.dropedge.to_c() if graph.dropedge is not None else None
    call("grl_graphconv_fwd", ctypes.byref(csr), X2.data_ptr(), X2.stride(0), F, Wc.data_ptr(),
         bc.data_ptr() if bc is not None else None, C, int(relu), out.data_ptr(),
         ctypes.byref(de) if de is not None else None, ws.data_ptr() if ws is not None else None, ws_bytes,
         current_stream_handle(X.device))
    return out


# Z bytes above which a training GraphConv keeps X and recomputes Z in the
# backward instead of holding Z between the passes (recompute=None): at C5
# scale (2^23 nodes, d=512) Z is 120 GB per layer, X 17 GB.  (The one-kernel
# backward's transient G_agg is Z-sized when C == F: recompute bounds the
# memory held between the passes, not the backward's peak -- graph_conv.)
RECOMPUTE_Z_BYTES = 8 << 30


def graph_conv(X: torch.Tensor, graph: TypedGraph, W: torch.Tensor, b=None, relu: bool = False,
               recompute: bool = None) -> torch.Tensor:
    """GraphConv forward (aggregation + linear [+ReLU]) as one autograd node;
    X: [num_cols, F] (or [B, N, F] for a batch graph).  When no gradient is
    wanted (eval, torch.no_grad) it is one grl_graphconv_fwd call instead:
    the same kernels, so the same bits.
    recompute: True keeps X instead of Z between the passes ((L+1)x less
    saved memory); None decides by Z's size (RECOMPUTE_Z_BYTES).  Where the
    one-kernel data gradient applies (grl_graphconv_bwd_data), the backward
    takes dW_s = X^T G_s from the aggregate G_s = A_drop,s^T g it writes:
    out and dX are bitwise the saved-Z path's, dW / db the same products
    summed in another order (fp32 rounding level).  Elsewhere Z is
    re-aggregated (one more SpMM pass) and every gradient is bitwise the
    saved-Z path's.  Peak memory in the G_s form: the transient G_agg
    [num_cols, (L+1) C] of the backward is Z-sized when C == F, so recompute
    lowers the memory held BETWEEN the passes, not the backward's peak."""
    if not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in (X, W, b))):
        if isinstance(graph, EdgeBlockedGraph):  # one int32 CSR per call: aggregate by blocks, then the linear
            return linear_fwd(spmm_forward(X, graph), W.contiguous(), b.contiguous() if b is not None else None,
                              relu)
        return graph_conv_infer(X, graph, W, b, relu)
    if recompute is None:
        recompute = graph.num_rows * graph.segments * X.shape[-1] * 4 > RECOMPUTE_Z_BYTES
    return _GraphConv.apply(X, graph, W, b, relu, bool(recompute))


def graph_linear(Z: torch.Tensor, W: torch.Tensor, b=None, relu: bool = False, path_rows: int = 0) -> torch.Tensor:
    """out = Z W + b (optionally ReLU) on MFMA; Z rows x (L+1)F.  path_rows:
    the row count the GEMM path is chosen for (0: Z's own rows; a node-range
    shard passes the whole graph's, as graph_conv does through
    GrlTypedCsr.path_rows)."""
    _require_device(Z, "aggregated features")
    return _GraphLinear.apply(Z, W, b, relu, int(path_rows))


# -------------------------------------------------------- feature dropout
def feature_dropout_apply(x2: torch.Tensor, de, row0: int, out: torch.Tensor = None) -> torch.Tensor:
    """out = x2 * keep * 1/(1-p) for the element ids (row0 + r) * cols + c
    (grl_feature_dropout); x2 a 2-D fp32 row view."""
    _require_device(x2, "dropout input")
    if x2.dtype != torch.float32 or x2.dim() != 2 or x2.stride(1) != 1:
        raise _lib.GrlError("feature_dropout: a 2-D float32 tensor with unit column stride")
    if out is None:
        out = torch.empty(x2.shape, dtype=torch.float32, device=x2.device)
    dc = de.to_c()
    call("grl_feature_dropout", x2.data_ptr(), x2.stride(0), out.data_ptr(), out.stride(0), x2.shape[0], x2.shape[1],
         int(row0), ctypes.byref(dc), current_stream_handle(x2.device))
    return out


class _FeatureDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, de, row0: int):
        ctx.de, ctx.row0 = de, row0
        return feature_dropout_apply(x2, de, row0)

    @staticmethod
    def backward(ctx, g):
        return feature_dropout_apply(_rows_view(g.contiguous()), ctx.de, ctx.row0), None, None


def feature_dropout(x: torch.Tensor, de, row0: int = 0) -> torch.Tensor:
    """nn.Dropout(p) over node-feature rows with the mask of element (global
    row, column) a counter hash under the DropEdge record `de` (its p, seed
    / seed tensor and call id): drop_robust_gcn.py:64,77,81,86,100.  row0:
    the global row of x's first row (a node-range shard's row_begin), so a
    shard's rows get the one-GPU model's mask."""
    lead = x.shape[:-1]
    x2 = _rows_view(x)
    return _FeatureDropout.apply(x2, de, int(row0)).view(*lead, x.shape[-1])


# ------------------------------------------------------- row-local linears
def linear_fwd_ex(X2: torch.Tensor, W: torch.Tensor, w_layout: int, b, relu: bool, path_rows: int = 0,
                  out: torch.Tensor = None) -> torch.Tensor:
    """out = X2 W (+ b) [ReLU] through grl_linear_fwd_ex; W [K, C]
    (w_layout 0) or [C, K] (1, nn.Linear.weight); the path chosen for
    max(M, path_rows) rows."""
    M, K = X2.shape
    C = W.shape[1] if w_layout == 0 else W.shape[0]
    if out is None:
        out = torch.empty(M, C, dtype=torch.float32, device=X2.device)
    ws_bytes = _lib.lib().grl_linear_fwd_ex_workspace_size(M, K, C, int(path_rows))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=X2.device) if ws_bytes else None
    call("grl_linear_fwd_ex", X2.data_ptr(), X2.stride(0), W.data_ptr(), int(w_layout),
         b.data_ptr() if b is not None else None, out.data_ptr(), M, K, C, int(relu), int(path_rows),
         ws.data_ptr() if ws is not None else None, ws_bytes, current_stream_handle(X2.device))
    return out


class _RowLinear(torch.autograd.Function):
    """nn.Linear (+ ReLU) on the libgrl GEMM: out = X W^T + b.  Every output
    row is the same fp32 operations whatever the row count (both GEMM paths
    are M-invariant and path_rows pins the choice), so a node-range shard's
    rows are bitwise the one-GPU model's."""

    @staticmethod
    def forward(ctx, X2, W, b, relu: bool, path_rows: int):
        C = W.shape[0]
        pad = -C % 4  # an output width off the float4 grid (the classifier's 53) runs padded with zero rows of W
        Wc = W.contiguous() if not pad else torch.nn.functional.pad(W, (0, 0, 0, pad))
        bc = None if b is None else (b.contiguous() if not pad else torch.nn.functional.pad(b, (0, pad)))
        out = linear_fwd_ex(X2, Wc, 1, bc, relu, path_rows)
        ctx.relu, ctx.path_rows, ctx.C = relu, path_rows, C
        ctx.save_for_backward(X2, Wc, out if relu else None)
        return out if not pad else out[:, :C].contiguous()

    @staticmethod
    def backward(ctx, g):
        X2, W, out = ctx.saved_tensors
        g = g.contiguous().float()
        C, Cp = ctx.C, W.shape[0]
        if Cp != C:
            g = torch.nn.functional.pad(g, (0, Cp - C))
        if ctx.relu:
            g = torch.where(out > 0, g, torch.zeros((), dtype=g.dtype, device=g.device))
        dX = dW = db = None
        if ctx.needs_input_grad[0]:
            dX = linear_fwd_ex(g, W, 0, None, False, ctx.path_rows)  # g [M, C] x W [C, K]
        want_b = ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            dWt, db = linear_bwd_weight(X2, g, None, want_b)  # X^T g [K, C]
            dW = dWt.t()[:C] if ctx.needs_input_grad[1] else None
            db = db[:C] if db is not None else None
        return dX, dW, db, None, None


def row_linear(X: torch.Tensor, W: torch.Tensor, b=None, relu: bool = False, path_rows: int = 0) -> torch.Tensor:
    """nn.Linear(K, C) [+ ReLU] over the rows of X [..., K] (W [C, K], b [C])
    on the libgrl GEMM (grl_linear_fwd_ex): the row-local linears of
    GraphCNNDropEdge (drop_robust_gcn.py:36-58, robust_gcn.py:81-83).
    path_rows: the row count the GEMM path is chosen for (a node-range
    shard passes the whole graph's)."""
    _require_device(X, "linear input")
    if X.dtype != torch.float32 or W.dtype != torch.float32:
        raise _lib.GrlError("row_linear: float32 input and weight required")
    lead = X.shape[:-1]
    X2 = _rows_view(X)
    # path_rows >= M: the M-invariant kernels only (never grl_linear_fwd's unpinned large-M tile)
    out = _RowLinear.apply(X2, W, b, relu, int(max(path_rows, X2.shape[0])))
    return out.view(*lead, W.shape[0])


# ---------------------------------------------------------------- attention
def _attn_check(Q, K, H, V, gamma):
    for t, what in ((Q, "queries"), (K, "keys"), (H, "values"), (V, "residual"), (gamma, "gamma")):
        _require_device(t, what)
        if t.dtype != torch.float32:
            raise _lib.GrlError(f"attention {what} must be float32 (got {t.dtype})")
    if Q.dim() != 3 or K.shape != Q.shape or H.dim() != 3 or H.shape[:2] != Q.shape[:2] or V.shape != H.shape \
            or gamma.shape != (H.shape[2],):
        raise _lib.GrlError(f"attention shapes: Q {tuple(Q.shape)}, K {tuple(K.shape)}, H {tuple(H.shape)}, "
                            f"V {tuple(V.shape)}, gamma {tuple(gamma.shape)}")


def _attn_workspace(B, N, dk, dv, device, backward: bool = False):
    """bf16 planes of the attention operands, split once per call, and the
    backward's partials (grl.h)."""
    lib = _lib.lib()
    n = (lib.grl_node_attention_bwd_workspace_size if backward else lib.grl_node_attention_workspace_size)(B, N, dk, dv)
    if not n:
        return None, 0
    try:
        return torch.empty(n, dtype=torch.uint8, device=device), n
    except torch.cuda.OutOfMemoryError:
        if not backward:
            raise
        # the backward's dQ slabs (N^2 / 4 bytes at dk <= 16) do not fit: the smaller
        # workspace runs the separate dQ kernel instead (grl.h)
        n = lib.grl_node_attention_workspace_size(B, N, dk, dv)
        return (torch.empty(n, dtype=torch.uint8, device=device), n) if n else (None, 0)


# Value columns per kernel call: the kernels hold one query's output row in
# registers (dv <= 256; 128 when dk > 32, where the fp32 kernels also carry
# 64-wide Q/K rows).  Wider values run as column blocks of one softmax: each
# block recomputes S = Q K^T (same bits, so the same P), and the backward's
# dS = P o (dP - D) is linear in the per-block dP_b and D_b, so dQ and dK are
# the block sums (robust_gcn.py:78-96 for any input_dim up to 512).
def _dv_blocks(dk: int, dv: int):
    width = 256 if dk <= 32 else 128
    n = -(-dv // width)
    step = -(-dv // n)
    step = -(-step // 32) * 32
    return [(c0, min(dv, c0 + step)) for c0 in range(0, dv, step)]


def node_attention_forward(Q, K, H, V, gamma, stats: bool = False, q_range=None):
    """out = gamma * softmax(Q K^T) H + V (robust_gcn.py:90-96), fused.
    stats=True also returns (o_norm, row_max, row_sum) for the backward.
    q_range=(q0, q1): only those query rows are computed (the other rows of
    the outputs are zeros) -- a node-range shard's queries against every key
    (grl_node_attention_fwd_rows)."""
    _attn_check(Q, K, H, V, gamma)
    Q, K, H, V, gamma = (t.contiguous() for t in (Q, K, H, V, gamma))
    B, N, dk = Q.shape
    dv = H.shape[2]
    q0, q1 = (0, N) if q_range is None else (int(q_range[0]), int(q_range[1]))
    blocks = _dv_blocks(dk, dv)
    if len(blocks) > 1:
        parts = [node_attention_forward(Q, K, H[..., a:b].contiguous(), V[..., a:b].contiguous(),
                                        gamma[a:b].contiguous(), stats=stats, q_range=q_range) for a, b in blocks]
        if not stats:
            return torch.cat(parts, -1)
        out = torch.cat([p[0] for p in parts], -1)
        onorm = torch.cat([p[1] for p in parts], -1)
        return out, onorm, parts[0][2], parts[0][3]
    alloc = torch.empty_like if q_range is None else torch.zeros_like  # ranged: rows outside stay defined
    out = alloc(V)
    onorm = alloc(V) if stats else None
    rmax = alloc(V[..., 0]) if stats else None
    rsum = (torch.ones_like(V[..., 0]) if q_range is not None else torch.empty_like(V[..., 0])) if stats else None
    ptr = (lambda t: t.data_ptr() if t is not None else None)  # noqa: E731
    ws, ws_bytes = _attn_workspace(B, N, dk, dv, V.device)
    call("grl_node_attention_fwd_rows", Q.data_ptr(), K.data_ptr(), H.data_ptr(), V.data_ptr(), gamma.data_ptr(),
         out.data_ptr(), ptr(onorm), ptr(rmax), ptr(rsum), B, N, dk, dv, q0, q1, ptr(ws), ws_bytes,
         current_stream_handle(V.device))
    return (out, onorm, rmax, rsum) if stats else out


def node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout, q_range=None):
    """(dQ, dK, dH) of out = gamma * softmax(Q K^T) H + V for the output
    gradient dout, from the forward's stats (grl_node_attention_bwd).
    q_range=(q0, q1): only those queries -- dQ of the range (other rows
    zero), dK / dH of every key from the range's queries alone (partials)."""
    dout = dout.contiguous().float()
    B, N, dk = Q.shape
    dv = H.shape[2]
    q0, q1 = (0, N) if q_range is None else (int(q_range[0]), int(q_range[1]))
    dO = dout * gamma
    dQ = dK = None
    dHs = []
    for a, b in _dv_blocks(dk, dv):  # one block unless dv exceeds a call's width
        dO_b = dO[..., a:b].contiguous()
        D = (dO_b * onorm[..., a:b]).sum(-1).contiguous()
        dQ_b = torch.empty_like(Q) if q_range is None else torch.zeros_like(Q)
        dK_b = torch.empty_like(K)
        dH_b = torch.empty(B, N, b - a, dtype=H.dtype, device=H.device)
        H_b = H[..., a:b].contiguous()
        ws, ws_bytes = _attn_workspace(B, N, dk, b - a, Q.device, backward=True)
        call("grl_node_attention_bwd_rows", Q.data_ptr(), K.data_ptr(), H_b.data_ptr(), dO_b.data_ptr(),
             rmax.data_ptr(), rsum.data_ptr(), D.data_ptr(), dQ_b.data_ptr(), dK_b.data_ptr(), dH_b.data_ptr(),
             B, N, dk, b - a, q0, q1, ws.data_ptr() if ws is not None else None, ws_bytes,
             current_stream_handle(Q.device))
        dQ = dQ_b if dQ is None else dQ + dQ_b
        dK = dK_b if dK is None else dK + dK_b
        dHs.append(dH_b)
    dH = dHs[0] if len(dHs) == 1 else torch.cat(dHs, -1)
    return dQ, dK, dH


class _NodeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Q, K, H, V, gamma):
        out, onorm, rmax, rsum = node_attention_forward(Q, K, H, V, gamma, stats=True)
        ctx.save_for_backward(Q.contiguous(), K.contiguous(), H.contiguous(), gamma, onorm, rmax, rsum)
        return out

    @staticmethod
    def backward(ctx, dout):
        Q, K, H, gamma, onorm, rmax, rsum = ctx.saved_tensors
        dout = dout.contiguous().float()
        dQ, dK, dH = node_attention_backward(Q, K, H, gamma, onorm, rmax, rsum, dout)
        dgamma = (dout * onorm).sum((0, 1))
        return dQ, dK, dH, dout, dgamma


def node_self_attention(Q: torch.Tensor, K: torch.Tensor, H: torch.Tensor, V: torch.Tensor,
                        gamma: torch.Tensor) -> torch.Tensor:
    """Autograd op: gamma * softmax_rows(Q K^T) H + V on the fused kernels
    (grl_node_attention_fwd / _bwd); never materialises the N x N scores."""
    return _NodeAttention.apply(Q, K, H, V, gamma)


# ------------------------------------------------------ bag-of-chars linear
def bag_linear_forward(V2: torch.Tensor, Wt: torch.Tensor, b, relu: bool) -> torch.Tensor:
    """relu?(V2 @ Wt + b) gathering only the nonzero rows of Wt per row of V2."""
    M, K = V2.shape
    C = Wt.shape[1]
    out = torch.empty(M, C, dtype=torch.float32, device=V2.device)
    call("grl_bag_linear_fwd", V2.data_ptr(), V2.stride(0), M, K, Wt.data_ptr(), C,
         b.data_ptr() if b is not None else None, int(relu), out.data_ptr(), current_stream_handle(V2.device))
    return out


# emb1's weight gradient on the sparse kernel from this many rows on (A/B at
# K = 4369, C = 256, ~7 + 4 nonzeros per row, profiles/r02_probe_bag_dw.json:
# M = 4096 dense GEMM 0.16 vs sparse 0.25 ms; 20k 0.59 vs 0.47; 100k 2.71 vs 1.51)
BAG_DW_SPARSE_ROWS = 16384


def bag_linear_bwd_weight(V2: torch.Tensor, g: torch.Tensor, relu_out, want_db: bool):
    """(dWt [K, C], db [C] or None) = V2^T g', 1^T g' with g' = g [out > 0],
    reading a row of g' only for V2's nonzeros (grl_bag_linear_bwd_weight)."""
    M, K = V2.shape
    C = g.shape[1]
    dWt = torch.empty(K, C, dtype=torch.float32, device=g.device)
    db = torch.empty(C, dtype=torch.float32, device=g.device) if want_db else None
    ws_bytes = _lib.lib().grl_bag_linear_bwd_weight_workspace_size(M, K, C)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=g.device)
    call("grl_bag_linear_bwd_weight", V2.data_ptr(), V2.stride(0), g.data_ptr(),
         relu_out.data_ptr() if relu_out is not None else None, dWt.data_ptr(),
         db.data_ptr() if db is not None else None, M, K, C, ws.data_ptr(), ws_bytes,
         current_stream_handle(g.device))
    return dWt, db


class _BagLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, V2, W, b, relu: bool):
        Wt = W.t().contiguous()
        out = bag_linear_forward(V2, Wt, b, relu)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.save_for_backward(V2, Wt, out)
        return out

    @staticmethod
    def backward(ctx, g):
        V2, Wt, out = ctx.saved_tensors
        g, relu_out, _ = relu_grad(g.contiguous().float(), out if ctx.relu else None)
        dV = linear_bwd_data(g, relu_out, Wt) if ctx.needs_input_grad[0] else None
        if V2.shape[0] >= BAG_DW_SPARSE_ROWS:  # large M: only V's nonzeros read a row of g
            dWt, db = bag_linear_bwd_weight(V2, g, relu_out, ctx.has_b)
        else:  # few rows: the split-K MFMA GEMM is faster (tools/probe_bag_dw.py)
            dWt, db = linear_bwd_weight(V2, g, relu_out, ctx.has_b)
        return dV, dWt.t(), db, None


def bag_linear(V: torch.Tensor, W: torch.Tensor, b, relu: bool = False) -> torch.Tensor:
    """nn.Linear(K, C) (+ReLU) for sparse inputs such as emb1's bag-of-chars
    rows: V [..., K], W [C, K] (nn.Linear.weight), b [C] or None."""
    _require_device(V, "bag-of-chars input")
    if V.dtype != torch.float32 or W.dtype != torch.float32:
        raise _lib.GrlError("bag_linear: float32 input and weight required")
    lead = V.shape[:-1]
    V2 = V.reshape(-1, V.shape[-1])
    if V2.stride(-1) != 1:
        V2 = V2.contiguous()
    return _BagLinear.apply(V2, W, b, relu).view(*lead, W.shape[0])
