/*
 * grl.h — C ABI of the MI355X (gfx950) message-passing engine behind
 * gnn.models.GraphCNNDropEdge / gnn.models.networks.robust_gcn.GraphConv.
 *
 * The reference (hoangthanh283/graph-representation-learning) is pure
 * Python/PyTorch and has no FFI; every entry point below replaces one aten
 * call (or one block of Python) on its GraphConv/DropEdge hot path.  The
 * citation on each function names the reference code it stands in for
 * (paths relative to the reference repository root).  A maintainer binds
 * these with ctypes; nothing here mentions torch.
 *
 * Conventions
 *  - Every pointer marked "device" is HBM memory owned by the caller (torch
 *    caching allocator).  The library never allocates or frees persistent
 *    memory; scratch comes from a caller workspace sized by *_workspace_size.
 *  - Every call is stream-ordered on `stream` (a hipStream_t passed as void*,
 *    NULL = default stream) and never synchronises the device, so calls can
 *    be captured into a hipGraph.  Failures found on the device are
 *    stream-ordered too: where grl_graphconv_fwd, grl_graphconv_fwd_train
 *    and grl_graphconv_bwd_data run their persistent one-kernel form, a
 *    follow-up kernel fills that call's outputs with NaN if a bounded wait
 *    ran out and records the entry point in a sticky per-device status word;
 *    grl_check() (the caller's existing sync point: a loss.item(), an event
 *    wait) reads and clears that word and returns GRL_E_TIMEOUT.
 *  - Return value 0 = success, negative GRL_E_* = failure; grl_last_error()
 *    returns a thread-local message for the last failure on this thread.
 *  - Empty operands: an operand with no rows (an empty torch tensor, whose
 *    data pointer is NULL) may be NULL whenever the call reads none of it --
 *    e.g. a node-range shard with no own rows: its typed-SpMM backward,
 *    ReLU/bias gradient (db = 0), weight gradient (dW = 0, db = 0) and
 *    one-kernel data gradient succeed and write zeros where they write.
 *  - fp32 features, int32 indices.  Sums over a row's edges run in CSR order
 *    with one fmaf per edge, so results are bitwise reproducible run to run
 *    (no float atomics anywhere).
 */
#ifndef GRL_H_
#define GRL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* grl_stream_t; /* hipStream_t */

enum {
  GRL_OK = 0,
  GRL_E_INVALID = -1,     /* bad shape / null pointer / inconsistent sizes   */
  GRL_E_UNSUPPORTED = -2, /* well-formed request this build does not handle  */
  GRL_E_HIP = -3,         /* a HIP runtime call failed                       */
  GRL_E_WORKSPACE = -4,   /* workspace smaller than *_workspace_size()       */
  GRL_E_OVERFLOW = -5,    /* a count does not fit the int32 index type       */
  GRL_E_TIMEOUT = -6      /* a persistent kernel's bounded wait ran out; its  */
                          /* outputs are invalid (see grl_graphconv_fwd)      */
};

/*
 * Heavy-row split plan (load balance for power-law graphs, e.g. R-MAT hubs).
 * A row whose edge count exceeds `threshold` is not gathered by one
 * wavefront: each of its segments is cut into chunks of at most
 * `chunk_edges` edges, every chunk is summed by its own wavefront into
 * `partials` (num_chunks x F floats), and a fixup pass adds a segment's
 * chunk partials in chunk order (deterministic, no atomics).  Built once per
 * graph by grl_split_plan_count / grl_split_plan_build; attach it to the
 * GrlTypedCsr / GrlTypedCsc `split` field (NULL = no splitting).
 */
typedef struct GrlSplitPlan {
  int32_t threshold;          /* rows with more edges than this are split   */
  int32_t chunk_edges;        /* max edges per chunk                         */
  int64_t num_heavy;          /* heavy segments (all segments of heavy rows) */
  int64_t num_chunks;
  const int32_t* heavy_seg;   /* device [num_heavy]: segment id row*nseg+t   */
  const int32_t* heavy_cptr;  /* device [num_heavy+1]: chunk range per seg   */
  const int32_t* chunk_begin; /* device [num_chunks]: first edge position    */
  const int32_t* chunk_end;   /* device [num_chunks]: one past last edge     */
  float* partials;            /* device scratch, >= num_chunks * F floats    */
  int64_t partials_capacity;  /* floats available in `partials`              */
} GrlSplitPlan;

/*
 * Typed CSR: the sparse form of the reference's preprocessed adjacency
 * A_pre[b, n*(L+1)+l, m] (gnn/models/networks/robust_gcn.py:53-72).
 * Row segment (n, t) for t in [0, num_types) lists the source rows m whose
 * features node n aggregates through edge type t, i.e. the nonzeros of
 * A_in[b, n, t, m] in the collate layout (B, N, L, N).  With has_self = 1 the
 * identity block l = 0 of A_pre is implicit (robust_gcn.py:58-65) and output
 * segment 0 of row n is the node's own feature row.
 *
 * Z row n has (has_self + num_types) segments of F floats:
 *   Z[n, has_self + t, :] = sum_{e in seg(n,t)} w_e * X[colidx[e], :]
 *   Z[n, 0, :]            = w_self(n) * X[n, :]             (if has_self)
 * which is exactly new_V of robust_gcn.py:45-47 for one graph of the batch.
 */
typedef struct GrlTypedCsr {
  int64_t num_rows;      /* destination nodes (rows of Z)                     */
  int32_t num_types;     /* typed segments per node (L, num_edges)            */
  int32_t has_self;      /* 1: implicit identity segment 0                    */
  const int32_t* rowptr; /* device [num_rows*num_types + 1], rowptr[0] == 0   */
  const int32_t* colidx; /* device [nnz]: source row of X                     */
  const float* vals;     /* device [nnz] edge values, or NULL for all-ones    */
  int64_t nnz;
  uint64_t edge_id_base; /* global DropEdge id of colidx[0] (node-range shard)*/
  uint64_t self_id_base; /* global DropEdge id of row 0's self loop           */
  const GrlSplitPlan* split; /* heavy-row plan over rowptr, or NULL           */
  int64_t self_row0;     /* X row of row 0's self term (0; a row-range view of
                            a graph -- rowptr a slice, the identity rows from
                            this row on -- sets its first row).  Forward entry
                            points only: grl_csr_to_csc and
                            grl_graphconv_bwd_data require 0.               */
  int64_t path_rows;     /* rows the GEMM path (split-bf16 x6 or fp32) is
                            chosen for; 0 = num_rows.  A node-range shard (or
                            a row-range view) passes the whole graph's row
                            count, so its rows take the one-GPU layer's path:
                            with it, every output row is bitwise the whole
                            graph's (both paths' per-row arithmetic is
                            independent of the row count).                   */
} GrlTypedCsr;

/*
 * Transposed typed CSR (CSC over source rows), used by the backward pass
 * dX = A_drop^T dZ (the BmmBackward0 of robust_gcn.py:45).
 *   dX[m, :] = w_self(m) * dZ[m, 0, :]  (m < self_rows, if has_self)
 *            + sum_{i in col(m)} w_{eid[i]} * dZ_rows[zrow[i], :]
 * where dZ_rows is dZ viewed as contiguous rows of F floats, so
 * zrow = n*(has_self+num_types) + has_self + t for edge (n, t, m).
 */
typedef struct GrlTypedCsc {
  int64_t num_rows;      /* rows of dX (local + halo rows in a shard)         */
  int64_t self_rows;     /* rows that own a self loop (local rows)            */
  int32_t num_types;
  int32_t has_self;
  const int32_t* colptr; /* device [num_rows + 1]                              */
  const int32_t* zrow;   /* device [nnz]                                       */
  const int32_t* eid;    /* device [nnz]: CSR position of the edge (local)     */
  const float* vals;     /* device [nnz] values in CSC order, or NULL          */
  int64_t nnz;
  uint64_t edge_id_base; /* as in the matching GrlTypedCsr                     */
  uint64_t self_id_base;
  const GrlSplitPlan* split; /* heavy-column plan over colptr, or NULL        */
} GrlTypedCsc;

/*
 * DropEdge: the reference's nn.Dropout(p) applied to A_pre
 * (gnn/models/networks/drop_robust_gcn.py:38,76,80,85) as a fused,
 * regenerable mask.  An entry with global id `id` is kept iff
 *   grl_dropedge_bits(key, id) >= threshold,   weight = value * scale,
 * with scale = float(1/(1-p)) as torch's native dropout computes it.
 * Edge ids are CSR positions (+ edge_id_base); the self loop of global node g
 * has id E_total + g.  No mask tensor ever exists.
 */
typedef struct GrlDropEdge {
  uint64_t key;       /* grl_dropedge_key(seed, call_id)                       */
  uint32_t threshold; /* floor(p * 2^32); 0 keeps everything                   */
  float scale;        /* 1/(1-p) (0 when p >= 1); 1 when p == 0                */
  int32_t active;     /* 0: identity (eval mode / p == 0)                      */
  int32_t drop_self;  /* 1: the identity block is masked too (efficient_mode)  */
  /* Device-resident stream (HIP-graph replays): when seed_dev != NULL every
   * kernel derives key = grl_dropedge_key(*seed_dev, call_id) at launch
   * instead of using `key`, so a captured training step draws a fresh mask
   * on each replay from a seed written on the device (e.g. by the RNG kernel
   * captured with it).  NULL for grl_dropedge_init.                        */
  const uint64_t* seed_dev;
  uint64_t call_id;
} GrlDropEdge;

/* Library identity / errors. */
const char* grl_version(void);
const char* grl_last_error(void);

/* Sticky device status of the current device: waits for `stream`, reads the
 * word the persistent kernels' follow-up kernels set (see Conventions) and
 * clears it.  GRL_OK, or GRL_E_TIMEOUT naming every entry point whose
 * outputs were invalidated (NaN) since the last check.  The one call that
 * synchronises; meant for points where the caller syncs anyway (the
 * reference's loss.item(), kv_procedure.py:140; an event wait).  Not
 * capturable.                                                              */
int grl_check(grl_stream_t stream);

/* Path options: the test / A-B hooks that pick among the kernel forms of one
 * entry point (e.g. "gemm_x6" 0 = the fp32-MFMA GEMMs, "graphconv_fused" 0 =
 * SpMM + GEMM instead of the one-kernel layer, "attn_x6" 0 = the fp32-MFMA
 * attention kernels, "ws_spin" = the persistent kernels' wait bound).  The
 * defaults are the production paths; every form computes the same result
 * within its documented tolerance.  Process-wide, read at each call (a
 * workspace query and the call it sizes must see the same settings).  The
 * names and ranges are listed in csrc/common.hip; an unknown name or an
 * out-of-range value is GRL_E_INVALID.  Nothing in the library reads the
 * environment.                                                             */
int grl_set_option(const char* name, int64_t value);
int grl_get_option(const char* name, int64_t* value);

/* roctx ranges (rocprofv3 --marker-trace): the hot entry points push their
 * own; these let a host layer bracket its steps, e.g. the halo exchange of a
 * node-range shard (grl/dist.py).  Pop closes the innermost open range.   */
void grl_trace_push(const char* name);
void grl_trace_pop(void);

/* Fills *de for drop probability p, RNG stream (seed, call_id).
 * drop_self = 1 reproduces efficient_mode=True (drop_robust_gcn.py:69,76):
 * the mask covers the identity block; 0 reproduces efficient_mode=False,
 * where dropout hits raw A before preprocess_adj adds the identity.
 * Host-only, no device work.  Replaces nn.Dropout.__init__/bernoulli_ setup. */
int grl_dropedge_init(GrlDropEdge* de, float p, uint64_t seed, uint64_t call_id,
                      int32_t drop_self);

/* As grl_dropedge_init, with the seed read on the device at each launch
 * from *seed_dev (device memory, 8 bytes; must stay valid while `de` is used,
 * including by graph replays).  Host-only, no device work.                 */
int grl_dropedge_init_device(GrlDropEdge* de, float p, const uint64_t* seed_dev,
                             uint64_t call_id, int32_t drop_self);

/* Feature dropout on node rows (nn.Dropout(p) at drop_robust_gcn.py:64,77,81,
 * 86,100): out[r][c] = x[r][c] * scale if element id (row0 + r) * cols + c
 * survives `de` (the DropEdge hash and keep rule above; the caller gives the
 * feature draws their own call ids), else 0.  row0 = the global row of x's
 * first row (a node-range shard's row_begin), so every row's mask is the
 * one-GPU model's wherever the row is computed.  The backward is the same
 * call on the gradient.  x / out [rows][ld*] fp32 (out may alias x).      */
int grl_feature_dropout(const float* x, int64_t ldx, float* out, int64_t ldo,
                        int64_t rows, int32_t cols, int64_t row0,
                        const GrlDropEdge* de, grl_stream_t stream);

/* keep[i] = 1 if id_base + i survives DropEdge `de`, else 0 (i < count).
 * Exposes the fused mask for parity checks against the dense reference
 * (the mask nn.Dropout would draw over A_pre, drop_robust_gcn.py:76).    */
int grl_dropedge_mask(const GrlDropEdge* de, uint64_t id_base, int64_t count,
                      uint8_t* keep /* device */, grl_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Hot path                                                                */
/* ---------------------------------------------------------------------- */

/* Z = A_drop X in typed-CSR form.  Replaces
 *   new_V = torch.matmul(A, V.view(-1, N, F)).view(-1, N, (L+1)*F)
 * (gnn/models/networks/robust_gcn.py:45-47) together with the edge_dropout
 * applied to A right before it (drop_robust_gcn.py:76,80,85).
 * X: device, row stride ldx floats (>= F).  Z: device, contiguous
 * [num_rows, (has_self+num_types)*F].  de may be NULL (eval).            */
int grl_typed_spmm_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx,
                       int32_t F, float* Z, const GrlDropEdge* de,
                       grl_stream_t stream);

/* Column slice of Z = A_drop X, for the pipelined halo exchange of a
 * node-range shard (grl/dist.py): the aggregation of
 * robust_gcn.py:45-47 restricted to F feature columns, so columns whose halo
 * rows have arrived are aggregated while the next slice is still in flight.
 *   Z[n*ldz + s*zseg + j] = segment s of row n, column j < F
 *   (s < has_self+num_types; Z points at the slice's first column),
 * the self term of row n reads X row self_col0 + n (the shard's own rows
 * inside a gathered table).  X: the slice's table, row stride ldx >= F.
 * Per element the same edges in the same order as grl_typed_spmm_fwd, so a
 * sliced aggregation is bitwise equal to the whole one.                     */
int grl_typed_spmm_fwd_slice(const GrlTypedCsr* g, const float* X, int64_t ldx,
                             int32_t F, int64_t self_col0, float* Z,
                             int64_t ldz, int32_t zseg, const GrlDropEdge* de,
                             grl_stream_t stream);

/* dX = A_drop^T dZ.  Replaces autograd's BmmBackward0 for robust_gcn.py:45
 * (grad of V through the aggregation), with the same DropEdge mask as the
 * forward call that used `de`.  dZ: contiguous [*, (has_self+num_types)*F];
 * dX: device, row stride lddx, num_rows rows, fully overwritten.          */
int grl_typed_spmm_bwd(const GrlTypedCsc* g, const float* dZ, int32_t F,
                       float* dX, int64_t lddx, const GrlDropEdge* de,
                       grl_stream_t stream);

/* dX += A_drop^T dZ over this CSC's edges, continuing every column's sum
 * from the value dX already holds (no self term).  Graphs with >= 2^31 typed
 * edges run as row blocks of < 2^31 edges (int32 positions inside a block,
 * 64-bit global edge ids via edge_id_base): the first block's CSC goes
 * through grl_typed_spmm_bwd, the later ones through this call, in block
 * order -- their CSC positions all follow the earlier blocks', so each
 * column's fmaf chain is the one a single CSC over all edges would run.   */
int grl_typed_spmm_bwd_accum(const GrlTypedCsc* g, const float* dZ, int32_t F,
                             float* dX, int64_t lddx, const GrlDropEdge* de,
                             grl_stream_t stream);

/* Columns [col0, col0 + F) of dX = A_drop^T dZ into dX (row stride lddx,
 * num_rows rows of F floats, fully overwritten), dZ contiguous
 * [*, (has_self+num_types)*F_total].  Per element bitwise equal to
 * grl_typed_spmm_bwd (same edges, same order): the multi-GPU backward
 * (grl.dist.HaloPipeline.backward) gathers one column slice of the halo-row
 * gradients while the previous slice travels back to its owners -- the
 * reverse of the forward halo exchange that replaces the dense
 * BmmBackward0 of robust_gcn.py:45 on a node-range shard.               */
int grl_typed_spmm_bwd_slice(const GrlTypedCsc* g, const float* dZ,
                             int32_t F_total, int32_t col0, int32_t F,
                             float* dX, int64_t lddx, const GrlDropEdge* de,
                             grl_stream_t stream);

/* out = Z W + bias (optionally ReLU), fp32-accurate on the matrix cores.
 * Replaces torch.matmul(new_V, self.h_weights) + self.bias
 * (robust_gcn.py:50) and, with relu = 1, the F.relu around the layer
 * (drop_robust_gcn.py:76).  Z [M, K] row-major (ldz), W [K, C] row-major,
 * bias [C] or NULL, out [M, C] contiguous.
 * Large M (>= 16 GFLOP, K % 16 == 0, 16-B aligned): fp32 values split
 * exactly into three bf16 parts, six partial products on
 * v_mfma_f32_32x32x16_bf16 (error at the fp32-rounding level, DESIGN.md
 * §4.2); W's bf16 planes go to `workspace`.  The path option gemm_x6 = 0
 * (grl_set_option) selects v_mfma_f32_32x32x2_f32 instead.
 * Otherwise, calls of >= 256 output tiles walk all of K in one pass; calls
 * that cannot fill the chip (small graphs: a 74-node page is one 128-row
 * tile) split K into chunks over workgroups -- sized from K and the call's
 * tile count, at most 64 -- as fp32 slabs in `workspace`, added in chunk
 * order (deterministic) with bias/ReLU applied once (slabs over 256 MB in
 * row blocks).  Each form is M-invariant, and grl_linear_fwd_ex's path_rows
 * makes every choice for the whole call's rows.
 * grl_linear_fwd_workspace_size() is 0 when no workspace is needed (it may
 * then be NULL), else the bytes the call requires.                        */
size_t grl_linear_fwd_workspace_size(int64_t M, int32_t K, int32_t C);
int grl_linear_fwd(const float* Z, int64_t ldz, const float* W,
                   const float* bias, float* out, int64_t M, int32_t K,
                   int32_t C, int32_t relu, void* workspace,
                   size_t workspace_bytes, grl_stream_t stream);

/* grl_linear_fwd with the weight's layout and the path's row count explicit:
 * w_layout 0: W [K, C] row-major (GraphConv.h_weights); 1: W [C, K]
 * row-major (nn.Linear.weight: out = Z W^T + bias, the row-local linears of
 * GraphCNNDropEdge -- emb2, NodeSelfAtten's f / g / h, the RanPAC projection,
 * the classifier -- drop_robust_gcn.py:36-58, robust_gcn.py:81-83).
 * path_rows: the row count every arithmetic choice is made for (x6 vs fp32,
 * one pass vs chunk slabs and the chunk size; 0 = M); a node-range shard
 * passes the whole graph's, so its rows are bitwise the one-GPU call's.
 * Workspace: grl_linear_fwd_ex_workspace_size().                           */
size_t grl_linear_fwd_ex_workspace_size(int64_t M, int32_t K, int32_t C,
                                        int64_t path_rows);
int grl_linear_fwd_ex(const float* Z, int64_t ldz, const float* W,
                      int32_t w_layout, const float* bias, float* out,
                      int64_t M, int32_t K, int32_t C, int32_t relu,
                      int64_t path_rows, void* workspace,
                      size_t workspace_bytes, grl_stream_t stream);

/* One GraphConv layer forward in one call (inference):
 *   out = relu?( (A_drop X) W + bias )       robust_gcn.py:45-51 (+ the F.relu
 * of drop_robust_gcn.py:76), i.e. grl_typed_spmm_fwd then grl_linear_fwd with
 * Z = A_drop X held in `workspace` (W [(has_self+num_types)*F, C] row-major,
 * bias [C] or NULL, out [num_rows, C] contiguous).  With the workspace of
 * grl_graphconv_fwd_workspace_size() Z exists whole (7.2 GB at C3); a smaller
 * workspace makes the call aggregate and multiply rows in chunks that fit
 * (>= 256 rows of Z plus W's bf16 planes), bitwise equal to the whole-graph
 * result -- allowed when the linear takes the x6 path (large graphs) and the
 * graph has no heavy-row split plan, else GRL_E_WORKSPACE.  Replaces the
 * GraphConv.forward pair `torch.matmul(A, V)` / `matmul(new_V, h_weights)`
 * for eval; training keeps Z for dW (grl_linear_bwd_weight).              */
size_t grl_graphconv_fwd_workspace_size(int64_t num_rows, int32_t num_types,
                                        int32_t has_self, int32_t F, int32_t C);
int grl_graphconv_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx,
                      int32_t F, const float* W, const float* bias, int32_t C,
                      int32_t relu, float* out, const GrlDropEdge* de,
                      void* workspace, size_t workspace_bytes,
                      grl_stream_t stream);

/* Workspace grl_graphconv_fwd uses for THIS graph, X and W (0 on bad
 * arguments).  Large graphs without a heavy-row split plan, F in {64, 128,
 * 256}, C <= 256, float4-aligned X rows and W run as ONE kernel
 * (graphconv.hip): Z = A_drop X stays on chip (32-row tiles in LDS as x6
 * bf16 planes, MFMA against W's planes) and the workspace holds only W's
 * planes (2.75 MB at K = 1792, C = 256) -- bitwise the two-kernel result.
 * Otherwise this is grl_graphconv_fwd_workspace_size().
 * graphconv_fused = 0 forces the two-kernel path.                      */
size_t grl_graphconv_fwd_workspace_query(const GrlTypedCsr* g, const float* X,
                                         int64_t ldx, int32_t F,
                                         const float* W, int32_t C);

/* Training forward of one GraphConv layer: out as grl_graphconv_fwd AND
 * Z = A_drop X ([num_rows, (has_self+num_types)*F] contiguous, 16-B aligned),
 * which the backward needs for dW (grl_linear_bwd_weight).  Where the
 * one-kernel path applies, Z is written by the gather waves as they finish
 * rows (its 7.2 GB write at C3 overlaps the MFMAs; the 7.2 GB read-back of
 * the two-kernel path disappears); elsewhere grl_typed_spmm_fwd then
 * grl_linear_fwd.  Bitwise the same out and Z either way.  Workspace:
 * grl_linear_fwd_workspace_size(num_rows, K, C).                         */
int grl_graphconv_fwd_train(const GrlTypedCsr* g, const float* X, int64_t ldx,
                            int32_t F, const float* W, const float* bias,
                            int32_t C, int32_t relu, float* out, float* Z,
                            const GrlDropEdge* de, void* workspace,
                            size_t workspace_bytes, grl_stream_t stream);

/* Data gradient of one GraphConv layer in ONE kernel.  Replaces the
 * autograd chain MmBackward0 (dZ = G W^T, robust_gcn.py:50) then
 * BmmBackward0 (dX = A_drop^T dZ, robust_gcn.py:45) by its reassociation
 *   dX = sum_s (A_drop,s^T G) W_s^T     (W_s = rows [s F, (s+1) F) of W),
 * i.e. the one-kernel GraphConv forward run over the typed transpose gt
 * (rows = source nodes, segments (m, t) in forward-CSR order, colidx = the
 * forward row n, vals = the CSC values; entry e's DropEdge id is
 * gt->edge_id_base + eid[e], its forward CSR position, and row m's self id
 * gt->self_id_base + m, so the mask is the forward's).  dZ (7.2 GB at C3)
 * never exists.  G = the output gradient through the ReLU, [num_rows, C]
 * (ldg); W the forward h_weights [(has_self+num_types)*F, C]; dX
 * [num_rows, F] contiguous, overwritten.  Floating point: the same products
 * summed in another order than the two-kernel chain (fp32-level difference,
 * tests/test_gpu_graphconv.py).  G has g_rows rows (the forward rows); gt
 * rows m < g_rows carry the self term w_self(m) G[m] W_0^T, rows beyond
 * (a node-range shard's halo columns) none -- dX of those rows is the
 * partial gradient the halo exchange sends home.  G_agg (NULL, or
 * [gt->num_rows, (has_self+num_types)*C] contiguous) also receives the
 * gathered sums A_drop,s^T G per segment -- with them the weight gradient
 * is dW_s = X^T (A_drop,s^T G), so a layer that kept X instead of Z needs
 * no re-aggregation (grl.ops.graph_conv, recompute mode).  Eligible shapes: a nonzero
 * grl_graphconv_bwd_data_workspace_query(), which is also the workspace
 * size; otherwise GRL_E_UNSUPPORTED and the caller runs the chain.       */
size_t grl_graphconv_bwd_data_workspace_query(const GrlTypedCsr* gt,
                                              const float* G, int64_t ldg,
                                              int32_t C, const float* W,
                                              int32_t F);
int grl_graphconv_bwd_data(const GrlTypedCsr* gt, const int32_t* eid,
                           const float* G, int64_t ldg, int64_t g_rows,
                           int32_t C, const float* W, int32_t F, float* dX,
                           float* G_agg, const GrlDropEdge* de,
                           void* workspace, size_t workspace_bytes,
                           grl_stream_t stream);

/* Backward of grl_linear_fwd (autograd MmBackward0 of robust_gcn.py:50, with
 * the ReLU of drop_robust_gcn.py:76 folded in when relu_out != NULL):
 *   dZ = (g * [relu_out > 0]) W^T           grl_linear_bwd_data,  dZ [M, K] (ld lddz)
 *   dW = Z^T (g * [relu_out > 0])           grl_linear_bwd_weight, dW [K, C]
 *   db = sum over rows of (g * [relu_out > 0])                     db [C] (or NULL)
 * g, relu_out: [M, C] contiguous (relu_out = the forward's ReLU output).
 * dW's reduction over M is split over workgroups into fp32 slabs (workspace)
 * added in split order: deterministic, no atomics.  dZ splits its short
 * reduction (C) the same way when M is small (workspace rule as
 * grl_linear_fwd).                                                          */
size_t grl_linear_bwd_data_workspace_size(int64_t M, int32_t K, int32_t C);
int grl_linear_bwd_data(const float* g, const float* relu_out, const float* W,
                        float* dZ, int64_t lddz, int64_t M, int32_t K, int32_t C,
                        void* workspace, size_t workspace_bytes,
                        grl_stream_t stream);
size_t grl_linear_bwd_weight_workspace_size(int64_t M, int32_t K, int32_t C);
int grl_linear_bwd_weight(const float* Z, int64_t ldz, const float* g,
                          const float* relu_out, float* dW, float* db, int64_t M,
                          int32_t K, int32_t C, void* workspace,
                          size_t workspace_bytes, grl_stream_t stream);

/* ReLU's derivative applied once (autograd ThresholdBackward of the ReLU at
 * drop_robust_gcn.py:76, the bias gradient of robust_gcn.py:51 with it):
 *   g_eff = g * [relu_out > 0]  (masked entries +0.0; g_eff may alias g)
 *   db    = sum over rows of g_eff                     (db may be NULL)
 * in one pass.  db is summed in the row blocks and order grl_linear_bwd_weight
 * uses for its db, so the two are bitwise equal on the same g_eff.  Used
 * before the large-M backward GEMMs, whose LDS-DMA operand path cannot mask
 * on the way.  g, relu_out, g_eff: [M, C] contiguous.                       */
size_t grl_relu_grad_workspace_size(int64_t M, int32_t C);
int grl_relu_grad(const float* g, const float* relu_out, float* g_eff, float* db,
                  int64_t M, int32_t C, void* workspace, size_t workspace_bytes,
                  grl_stream_t stream);

/* emb1: Linear(K -> C) (+ReLU) over sparse bag-of-characters rows
 * (drop_robust_gcn.py:36,64; rows from TextlineEncoding,
 * textline_encoding.py:23-42):
 *   out[m, :] = relu?(bias + sum_{k: V[m,k] != 0, ascending} V[m,k] Wt[k, :])
 * V [M, K] row stride ldv (dense storage, mostly zeros), Wt [K, C]
 * contiguous (= nn.Linear.weight^T), bias [C] or NULL, out [M, C].  Only the
 * nonzeros cost gathers; C in [1, 512].  Backward: grl_bag_linear_bwd_weight
 * (dWt, db) and grl_linear_bwd_data (dV).                                 */
int grl_bag_linear_fwd(const float* V, int64_t ldv, int64_t M, int32_t K,
                       const float* Wt, int32_t C, const float* bias,
                       int32_t relu, float* out, grl_stream_t stream);

/* emb1's weight gradient (autograd MmBackward0 / AddmmBackward0 of
 * drop_robust_gcn.py:64 through nn.Linear) on the same sparse rows:
 *   dWt[k, :] = sum_{m: V[m,k] != 0, ascending m} V[m,k] g'[m, :],
 *   db = sum_m g'[m, :],   g' = g * [relu_out > 0] (relu_out NULL: g' = g).
 * V [M, K] stride ldv, g / relu_out [M, C] contiguous, dWt [K, C], db [C] or
 * NULL; C in [1, 512].  Only V's nonzeros read a row of g'.  Row ranges are
 * summed in range order (deterministic).  Workspace from the query.       */
size_t grl_bag_linear_bwd_weight_workspace_size(int64_t M, int32_t K, int32_t C);
int grl_bag_linear_bwd_weight(const float* V, int64_t ldv, const float* g,
                              const float* relu_out, float* dWt, float* db,
                              int64_t M, int32_t K, int32_t C, void* workspace,
                              size_t workspace_bytes, grl_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Node self-attention                                                     */
/* ---------------------------------------------------------------------- */
/* NodeSelfAtten (robust_gcn.py:78-99) fused, flash-style (no B x N x N
 * score matrix):  out = gamma * softmax_rows(Q K^T) H + V   per batch,
 * Q = f(V), K = g(V) [B, N, dk], H = h(V), V [B, N, dv], gamma [dv], all
 * contiguous fp32; no 1/sqrt(dk) scale and no mask (every node of the padded
 * batch attends to every node, as the reference does).  dk in [0, 32]
 * (input_dim // 8; 0 = uniform attention, Q/K may then be NULL), dv in
 * [1, 256].  For training pass o_norm [B, N, dv]
 * (= softmax(QK^T) H) and row_max/row_sum [B, N] (the softmax statistics);
 * NULL otherwise.
 * fp32-accurate on the bf16 matrix cores (each fp32 value split exactly into
 * three bf16 parts, six partial products; attn_x6 = 0 selects the
 * fp32-MFMA kernels).  `workspace` (grl_node_attention_workspace_size bytes,
 * or NULL) holds the once-per-call bf16 splits of K and H (backward: also Q
 * and dO); NULL or too small makes every workgroup split its own blocks.   */
size_t grl_node_attention_workspace_size(int64_t B, int64_t N, int32_t dk,
                                         int32_t dv);
int grl_node_attention_fwd(const float* Q, const float* K, const float* H,
                           const float* V, const float* gamma, float* out,
                           float* o_norm, float* row_max, float* row_sum,
                           int64_t B, int64_t N, int32_t dk, int32_t dv,
                           void* workspace, size_t workspace_bytes,
                           grl_stream_t stream);

/* Backward of the attention core.  dO = gamma * d_out [B, N, dv] and
 * D = rowsum(dO * o_norm) [B, N] come from the caller (elementwise); the
 * kernels recompute P from row_max/row_sum and write dQ, dK [B, N, dk] and
 * dH [B, N, dv] (fully overwritten).  Deterministic, no atomics: dK / dH are
 * key-stationary; dQ is query-stationary, or -- with a workspace of
 * grl_node_attention_bwd_workspace_size bytes, dk <= 16 -- folded into the
 * dK kernel as one partial slab per 256-key workgroup (B ceil(N/256) N 64
 * bytes; beyond 24 GiB the fused pass runs in key chunks, each chunk's slabs
 * added onto dQ in order: the same additions) added in workgroup order.  d gamma = sum(d_out * o_norm) and the residual's d_out are the
 * caller's.                                                                  */
size_t grl_node_attention_bwd_workspace_size(int64_t B, int64_t N, int32_t dk,
                                             int32_t dv);
int grl_node_attention_bwd(const float* Q, const float* K, const float* H,
                           const float* dO, const float* row_max,
                           const float* row_sum, const float* D, float* dQ,
                           float* dK, float* dH, int64_t B, int64_t N,
                           int32_t dk, int32_t dv, void* workspace,
                           size_t workspace_bytes, grl_stream_t stream);

/* The same two calls over the query rows [q_begin, q_end) only -- a node-
 * range shard's own queries against EVERY key (NodeSelfAtten on a sharded
 * graph, robust_gcn.py:90-96; grl/dist.py sharded_node_attention).  All
 * arrays keep their [B, N, ...] shapes; rows outside the range of Q / V /
 * dO are read as padding only, and those of out / o_norm / row_max /
 * row_sum / dQ are not written.  fwd: out, o_norm and the stats of the
 * range.  bwd: dQ of the range (complete), and dK, dH of EVERY key as the
 * range's queries' contribution (partials: a shard adds the other shards'
 * in rank order); row_max / row_sum / D must hold the range's rows (the
 * whole softmax's statistics).  The whole range (0, N) is exactly
 * grl_node_attention_fwd / _bwd.  No key split, no folded dQ when ranged. */
int grl_node_attention_fwd_rows(const float* Q, const float* K, const float* H,
                                const float* V, const float* gamma, float* out,
                                float* o_norm, float* row_max, float* row_sum,
                                int64_t B, int64_t N, int32_t dk, int32_t dv,
                                int64_t q_begin, int64_t q_end, void* workspace,
                                size_t workspace_bytes, grl_stream_t stream);
int grl_node_attention_bwd_rows(const float* Q, const float* K, const float* H,
                                const float* dO, const float* row_max,
                                const float* row_sum, const float* D, float* dQ,
                                float* dK, float* dH, int64_t B, int64_t N,
                                int32_t dk, int32_t dv, int64_t q_begin,
                                int64_t q_end, void* workspace,
                                size_t workspace_bytes, grl_stream_t stream);

/* ---------------------------------------------------------------------- */
/* Graph formats                                                           */
/* ---------------------------------------------------------------------- */

/* Dense adjacency -> typed CSR, block-diagonal over the batch.
 * Replaces GraphConv.preprocess_adj (robust_gcn.py:53-72): instead of the
 * dense (B, (L+1)N, N) A_pre, emit the nonzeros of A[b, n, t, m] addressed by
 * element strides {sb, sn, st, sm} (the collate layout (B,N,L,N) has
 * sm = 1; the permuted view GraphConv.forward receives, (B,N,N,L), is the
 * same storage).  Global node id = b*N + n; global row = (b*N + n)*L + t.
 * Two phases because nnz is data-dependent:
 *   1) grl_dense_to_csr_rowptr writes rowptr[B*N*L + 1] (the caller reads
 *      rowptr[B*N*L] to size colidx/vals);
 *   2) grl_dense_to_csr_fill writes colidx (global source node b*N + m) and
 *      vals (the A value; NULL to skip) in ascending m within each row.   */
size_t grl_dense_to_csr_workspace_size(int64_t num_segments);
int grl_dense_to_csr_rowptr(const float* A, int64_t B, int64_t N, int32_t L,
                            const int64_t strides[4], int32_t* rowptr,
                            void* workspace, size_t workspace_bytes,
                            grl_stream_t stream);
int grl_dense_to_csr_fill(const float* A, int64_t B, int64_t N, int32_t L,
                          const int64_t strides[4], const int32_t* rowptr,
                          int32_t* colidx, float* vals, grl_stream_t stream);

/* Heavy-row plan over a segment pointer array ptr[rows*nseg + 1] (rowptr
 * with nseg = L for the forward CSR, colptr with nseg = 1 for the CSC).
 *   grl_split_plan_count -> counts[0] = heavy segments, counts[1] = chunks
 *                           (device int64[2]; the caller reads them to size
 *                           the plan arrays)
 *   grl_split_plan_build -> fills plan->heavy_seg/heavy_cptr/chunk_begin/
 *                           chunk_end (caller-allocated, sizes from count)
 * Deterministic: segments and chunks are emitted in row, segment, edge order. */
size_t grl_split_plan_workspace_size(int64_t rows);
int grl_split_plan_count(const int32_t* ptr, int64_t rows, int32_t nseg, int32_t threshold,
                         int32_t chunk_edges, int64_t* counts, void* workspace,
                         size_t workspace_bytes, grl_stream_t stream);
int grl_split_plan_build(const int32_t* ptr, int64_t rows, int32_t nseg, GrlSplitPlan* plan,
                         void* workspace, size_t workspace_bytes, grl_stream_t stream);

/* Typed CSR -> CSC over source rows [0, num_cols) for the backward pass.
 * Stable: within a column, entries keep CSR (edge id) order, so dX sums are
 * deterministic.  colptr [num_cols+1], zrow/eid [nnz], vals_out [nnz] (only
 * written when g->vals != NULL).                                          */
size_t grl_csr_to_csc_workspace_size(int64_t nnz, int64_t num_cols);
int grl_csr_to_csc(const GrlTypedCsr* g, int64_t num_cols, int32_t* colptr,
                   int32_t* zrow, int32_t* eid, float* vals_out,
                   void* workspace, size_t workspace_bytes,
                   grl_stream_t stream);

/* Heuristic spatial graph of one document (host-only, no device work).
 * Replaces Graph(...) and Graph._get_adj_matrix
 * (gnn/data_generator/data_process/utils/graph_utils.py:425-834) as called by
 * HeuristicGraphBuilder.process (heuristic_graph_builder.py:56-83).
 * Items are the sample's text lines in label-index order with their axis-
 * aligned boxes (min/max of the polygon); kind 0 = text line, 1 = "cell",
 * 2 = "table" (dropped, as in the reference).  Edge types are
 * lr, rl, tb, bt, child, parent (graph_utils.py:434).
 *   grl_layout_graph_size  -> *out_n = min(#items, #graph nodes), the side of
 *                             the adjacency the reference keeps
 *   grl_layout_graph_dense -> (out_n, 6, out_n) adjacency as IEEE fp16 bits
 *                             (the reference's float16 array); edge_type
 *                             0 = normal_binary, 1 = fc_similarity, 2 = fc_binary
 *   grl_layout_graph_edges -> the normal_binary edges as sorted unique
 *                             (src, type, dst) int32 triples: typed CSR input
 *                             without the dense O(N^2) matrix.  *count is the
 *                             number of edges; nothing is written if it
 *                             exceeds `capacity` (call again with room).   */
typedef struct GrlLayoutItem {
  double x1, y1, x2, y2; /* box: min/max of the polygon's x and y            */
  int32_t kind;          /* 0 text line, 1 cell, 2 table                      */
  int32_t has_text;      /* str(text) != ""                                  */
} GrlLayoutItem;
int grl_layout_graph_size(const GrlLayoutItem* items, int32_t n, int32_t* out_n);
int grl_layout_graph_dense(const GrlLayoutItem* items, int32_t n, int32_t edge_type,
                           int32_t out_n, uint16_t* adj_half);
int grl_layout_graph_edges(const GrlLayoutItem* items, int32_t n, int32_t out_n,
                           int32_t* edges, int64_t capacity, int64_t* count);

/* Synthetic graphs for the benchmark configs.
 * Candidate edge k in [0, num_candidates) is (src, type, dst) drawn from a
 * counter-based hash of (seed, k): Erdos-Renyi (kind 0: src, dst uniform in
 * [0, N)) or R-MAT (kind 1: a,b,c,d = 0.57,0.19,0.19,0.05, N = 2^scale);
 * type uniform in [0, L).  Node-range shard [row_begin, row_end) keeps the
 * candidates whose src falls in it, dedupes (src, type, dst) and emits typed
 * CSR rows for those nodes (global colidx).  Three phases:
 *   grl_synth_count   -> *count (device int64) = candidates in the shard
 *   grl_synth_build   -> rowptr [(row_end-row_begin)*L + 1], colidx, and
 *                        *nnz (device int64) after dedupe
 * Workspace from grl_synth_workspace_size(count).                         */
typedef struct GrlSynthSpec {
  int32_t kind;           /* 0 = Erdos-Renyi, 1 = R-MAT                     */
  int32_t num_types;      /* L                                              */
  int64_t num_nodes;      /* N                                              */
  int64_t num_candidates; /* N * avg_deg before dedupe                      */
  uint64_t seed;
  int64_t row_begin, row_end;
} GrlSynthSpec;
int grl_synth_count(const GrlSynthSpec* spec, int64_t* count /* device */,
                    grl_stream_t stream);
size_t grl_synth_workspace_size(const GrlSynthSpec* spec, int64_t count);
/* deg[v - row_begin] += candidates with src v, for v in [row_begin, row_end)
 * (before dedupe; deg must be zeroed by the caller).  Used to choose
 * edge-balanced node-range shard boundaries for power-law graphs. */
int grl_synth_degrees(const GrlSynthSpec* spec, int32_t* deg, grl_stream_t stream);
int grl_synth_build(const GrlSynthSpec* spec, int64_t count, int32_t* rowptr,
                    int32_t* colidx, int64_t* nnz /* device */,
                    void* workspace, size_t workspace_bytes,
                    grl_stream_t stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* GRL_H_ */
