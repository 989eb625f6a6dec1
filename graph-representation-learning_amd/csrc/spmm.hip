// Typed-CSR SpMM with fused DropEdge for gfx950 (MI355X).
//
// Replaces the dense aggregation of the reference GraphConv,
//   new_V = torch.matmul(A_pre, V)       gnn/models/networks/robust_gcn.py:45-47
// with the edge_dropout applied to A_pre right before each call
//   (gnn/models/networks/drop_robust_gcn.py:38,76,80,85),
// and its autograd backward dV = A_drop^T dZ (BmmBackward0).
//
// Design (HBM-bound gather):
//  * one wavefront owns one work item at a time (grid-stride): a destination
//    row, or -- for rows heavier than the split threshold (power-law hubs) --
//    one chunk of <= chunk_edges edges of one segment, summed into a partial
//    row that a fixup pass adds in chunk order (deterministic, no atomics).
//    Chunk items come first in the item space so hub work overlaps the rest;
//  * each lane owns VEC*NV contiguous feature columns, so every gathered
//    neighbour row is one coalesced 16 B/lane sweep (1 KiB per
//    wave-instruction at F = 256);
//  * 64 edge indices are loaded per wave-instruction, the DropEdge weights of
//    all 64 are computed in parallel from the counter hash, and a ballot keeps
//    only surviving edges: dropped edges cost no gather bytes;
//  * surviving edges are issued U at a time (U independent row loads in flight
//    per wave) and accumulated with one fmaf per edge in CSR order, so results
//    are deterministic and equal the oracle's fmaf chain;
//  * type-segment boundaries are wave-uniform scalar compares, so a row's
//    edges of all types stream through one loop (no per-type round trip).
#include <climits>

#include <hipcub/hipcub.hpp>

#include "grl_internal.h"

#include <cstdlib>

namespace grl {
namespace {

template <int VEC>
struct VecT;
template <>
struct VecT<4> {
  using type = float4;
};
template <>
struct VecT<1> {
  using type = float;
};

__device__ __forceinline__ void vzero(float4& a) { a = make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void vzero(float& a) { a = 0.f; }
__device__ __forceinline__ void vfma(float4& acc, float w, const float4& x) {
  acc.x = __builtin_fmaf(w, x.x, acc.x);
  acc.y = __builtin_fmaf(w, x.y, acc.y);
  acc.z = __builtin_fmaf(w, x.z, acc.z);
  acc.w = __builtin_fmaf(w, x.w, acc.w);
}
__device__ __forceinline__ void vfma(float& acc, float w, const float& x) { acc = __builtin_fmaf(w, x, acc); }
__device__ __forceinline__ float4 vmul(float w, const float4& x) {
  return make_float4(w * x.x, w * x.y, w * x.z, w * x.w);
}
__device__ __forceinline__ float vmul(float w, const float& x) { return w * x; }
__device__ __forceinline__ void vadd(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}
__device__ __forceinline__ void vadd(float& a, const float& b) { a += b; }

// Output stores are non-temporal: the 7 GB Z stream (C3) is written once and
// should not evict gathered X rows from L2 / the MALL.  Measured A/B on the
// same MI355X: C3 forward 7.46 -> 7.07 ms.  GRL_NT_STORE=0 restores plain stores.
#ifndef GRL_NT_STORE
#define GRL_NT_STORE 1
#endif
using f4v = __attribute__((ext_vector_type(4))) float;
__device__ __forceinline__ void vstore(float* p, const float4& v) {
#if GRL_NT_STORE
  f4v t = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(p));
#else
  *reinterpret_cast<float4*>(p) = v;
#endif
}
__device__ __forceinline__ void vstore(float* p, const float& v) {
#if GRL_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}


// Whole-row (F <= 256) gathers in flight per wave (A/B builds: -DGRL_SPMM_U=n).
#ifndef GRL_SPMM_U
#define GRL_SPMM_U 8
#endif

// Persistent-grid size: 24 four-wave blocks per CU.  Measured
// (tools/ab_spmm_blocks*.sh, interleaved, two boxes): against 16, C3 forward
// 6.24 vs 6.41-6.67 ms, p=0.3 forward and CSC backward 2-3 % faster, C4
// 28.3-28.9 vs 29.1-29.6 ms, C5 125.9 vs 130.3 ms; 20 and 26 are slower
// than either (6.45-6.55 ms at C3), 22 and 28 close to 24.  The
// spmm_blocks_per_cu path option overrides it (tuning aid, e.g. to leave
// room for a concurrent GEMM on another stream).
int spmm_blocks_per_cu() { return (int)opt(OPT_SPMM_BLOCKS_PER_CU); }

// Device view of a split plan (all null / zero when the graph is not split).
struct SplitDev {
  int threshold;  // INT_MAX: nothing is heavy
  int64_t num_chunks;
  const int32_t* chunk_begin;
  const int32_t* chunk_end;
  float* partials;
};

// BWD = false: forward, rows are destination nodes with S typed segments,
//               sources are X rows (index = colidx), ids = edge_base + e.
// BWD = true : backward, rows are source nodes with one segment (CSC column),
//               sources are dZ rows (index = zrow), ids = edge_base + eid[e].
// ACCUM (backward only): continue each column's sum from the value already in
// dX instead of starting from the self term -- the later edge blocks of a
// graph with >= 2^31 edges (grl_typed_spmm_bwd_accum), whose CSC positions all
// follow the earlier blocks', so the fmaf chain equals the one-CSC chain.
template <int VEC, int NV, int U, bool VALS, bool BWD, bool ACCUM = false>
__global__ __launch_bounds__(256) void spmm_kernel(
    int64_t num_rows, int64_t self_rows, int S, int hs,
    const int32_t* __restrict__ ptr,   // fwd: rowptr [rows*S+1]; bwd: colptr [rows+1]
    const int32_t* __restrict__ idx,   // fwd: colidx; bwd: zrow
    const int32_t* __restrict__ eidv,  // bwd: eid (CSR positions); fwd: unused
    const float* __restrict__ vals, uint64_t edge_base, uint64_t self_base,
    int64_t self_row0,  // fwd: X row of item row 0's self term (row-range launches)
    const float* __restrict__ src, int64_t lds,  // gathered matrix + row stride
    int F, float* __restrict__ out, int64_t ldo,
    int zseg,  // fwd: floats between output segments (F, or the full width for a column slice);
               // bwd: dZ segment width (F, or the full width for a column slice)
    DropDev de, SplitDev sp) {
  using vec_t = typename VecT<VEC>::type;
  de = resolve_key(de);
  const int lane = threadIdx.x & 63;
  const int cbase = blockIdx.y * (64 * VEC * NV);
  int coff[NV];
  bool cval[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    coff[k] = cbase + (k * 64 + lane) * VEC;
    cval[k] = coff[k] < F;
  }
  const int nseg_row = BWD ? 1 : S;
  const int64_t zstride = (int64_t)(S + hs) * (BWD ? zseg : F);  // bwd self term: dZ row stride

  const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + uniform_i(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t num_items = sp.num_chunks + num_rows;

  for (int64_t item = wave0; item < num_items; item += nwaves) {
    vec_t acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) vzero(acc[k]);
    int pv, nseg;
    float* obase;
    if (item < sp.num_chunks) {
      // ---- chunk of a heavy segment -> partial row --------------------------
      const int64_t c = item;
      pv = lane == 0 ? sp.chunk_begin[c] : (lane == 1 ? sp.chunk_end[c] : 0);
      nseg = 1;
      obase = sp.partials + c * F;
    } else {
      const int64_t n = item - sp.num_chunks;
      float* orow = out + n * ldo;
      pv = lane <= nseg_row ? ptr[n * nseg_row + lane] : 0;
      nseg = nseg_row;
      const bool heavy = readlane_i(pv, nseg) - readlane_i(pv, 0) > sp.threshold;
      if (ACCUM && !heavy) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
          if (cval[k]) acc[k] = *reinterpret_cast<const vec_t*>(orow + coff[k]);
      }
      // ---- self term (identity block of A_pre, robust_gcn.py:58-65) ------
      if (!ACCUM && hs && (!BWD || (n < self_rows && !heavy))) {
        float w = 1.0f;
        if (de.active && de.drop_self) w = dropedge_weight(de, 1.0f, self_base + (uint64_t)n);
        const float* srow = BWD ? (src + n * zstride) : (src + (n + self_row0) * lds);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          if (cval[k]) {
            vec_t x;
            if (w != 0.0f)
              x = vmul(w, *reinterpret_cast<const vec_t*>(srow + coff[k]));
            else
              vzero(x);
            if (BWD)
              acc[k] = x;
            else
              vstore(orow + coff[k], x);
          }
        }
      }
      if (heavy) continue;  // typed segments come from the chunk partials (fixup)
      obase = BWD ? orow : orow + hs * zseg;
    }

    // ---- gather-accumulate over the item's edges ------------------------
    const int e_begin = readlane_i(pv, 0);
    const int e_end = readlane_i(pv, nseg);
    int t = 0;
    int seg_end = readlane_i(pv, 1);
    for (int c0 = e_begin; c0 < e_end; c0 += 64) {
      const int cnt = min(64, e_end - c0);
      int sidx = 0;
      float w = 0.0f;
      if (lane < cnt) {
        sidx = idx[c0 + lane];
        const float v = VALS ? vals[c0 + lane] : 1.0f;
        w = v;
        if (de.active) {  // the CSC edge-id list is only read when DropEdge draws
          const uint64_t id = BWD ? edge_base + (uint64_t)(uint32_t)eidv[c0 + lane]
                                  : edge_base + (uint64_t)(c0 + lane);
          w = dropedge_weight(de, v, id);
        }
      }
      uint64_t kept = __ballot(w != 0.0f);
      while (kept) {
        int jj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (kept) {
            jj[u] = __builtin_ctzll(kept);
            kept &= kept - 1;
          } else {
            jj[u] = -1;
          }
        }
        vec_t xv[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (jj[u] >= 0) {
            const int r = readlane_i(sidx, jj[u]);
            const float* srow = src + (int64_t)r * lds;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
              if (cval[k])
                xv[u][k] = *reinterpret_cast<const vec_t*>(srow + coff[k]);
              else
                vzero(xv[u][k]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (jj[u] >= 0) {
            if (!BWD) {
              const int e = c0 + jj[u];
              while (e >= seg_end) {  // flush finished segments (wave-uniform)
#pragma unroll
                for (int k = 0; k < NV; ++k) {
                  if (cval[k]) vstore(obase + t * zseg + coff[k], acc[k]);
                  vzero(acc[k]);
                }
                ++t;
                seg_end = readlane_i(pv, t + 1);
              }
            }
            const float wj = readlane_f(w, jj[u]);
#pragma unroll
            for (int k = 0; k < NV; ++k) vfma(acc[k], wj, xv[u][k]);
          }
        }
      }
    }
    // ---- flush the remaining (possibly empty) segments -----------------
    for (; t < nseg; ++t) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (cval[k]) vstore(obase + t * zseg + coff[k], acc[k]);
        vzero(acc[k]);
      }
    }
  }
}

// Narrow rows (forward, F <= 128 in float4 columns: the column slices of a
// pipelined halo exchange).  A whole-row wave would leave half its lanes idle
// and move 512 B per gather instruction; here every gather instruction
// fetches two edges' rows -- lanes 0-31 edge j, lanes 32-63 edge j+1 -- and
// v_permlane32_swap hands edge j+1's row to lanes 0-31, which accumulate the
// two in CSR order (fmaf chain identical to spmm_kernel: bitwise equal).
// Lanes 32-63 only fetch; stores and the self term are lanes 0-31's.
// BWD: the same over CSC columns (one segment, self term = dZ's own row
// first, edge ids from eid): the column slices of the pipelined backward.
__device__ __forceinline__ float swap_halves(float x) {
  return __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false)[1]);
}

template <int U, bool VALS, bool BWD = false>
__global__ __launch_bounds__(256) void spmm_pair_kernel(
    int64_t num_rows, int S, int hs, const int32_t* __restrict__ ptr, const int32_t* __restrict__ idx,
    const float* __restrict__ vals, uint64_t edge_base, uint64_t self_base, int64_t self_row0,
    const float* __restrict__ src, int64_t lds, int F, float* __restrict__ out, int64_t ldo, int zseg, DropDev de,
    SplitDev sp, const int32_t* __restrict__ eidv, int64_t self_rows) {
  de = resolve_key(de);
  const int nseg_row = BWD ? 1 : S;
  const int lane = threadIdx.x & 63;
  const int half = lane >> 5;
  const int coff = (lane & 31) * 4;
  const bool ld_ok = coff < F;
  const bool own = half == 0 && ld_ok;
  const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + uniform_i(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int64_t num_items = sp.num_chunks + num_rows;

  for (int64_t item = wave0; item < num_items; item += nwaves) {
    float4 acc;
    vzero(acc);
    int pv, nseg;
    float* obase;
    if (item < sp.num_chunks) {
      const int64_t c = item;
      pv = lane == 0 ? sp.chunk_begin[c] : (lane == 1 ? sp.chunk_end[c] : 0);
      nseg = 1;
      obase = sp.partials + c * F;
    } else {
      const int64_t n = item - sp.num_chunks;
      float* orow = out + n * ldo;
      pv = lane <= nseg_row ? ptr[n * nseg_row + lane] : 0;
      nseg = nseg_row;
      const bool heavy = readlane_i(pv, nseg) - readlane_i(pv, 0) > sp.threshold;
      if (hs && (!BWD || (n < self_rows && !heavy))) {
        float w = 1.0f;
        if (de.active && de.drop_self) w = dropedge_weight(de, 1.0f, self_base + (uint64_t)n);
        if (own) {
          float4 x;
          const float* srow = BWD ? src + n * ((int64_t)(S + hs) * zseg) : src + (n + self_row0) * lds;
          if (w != 0.0f)
            x = vmul(w, *reinterpret_cast<const float4*>(srow + coff));
          else
            vzero(x);
          if (BWD)
            acc = x;
          else
            vstore(orow + coff, x);
        }
      }
      if (heavy) continue;
      obase = BWD ? orow : orow + hs * zseg;
    }

    const int e_begin = readlane_i(pv, 0);
    const int e_end = readlane_i(pv, nseg);
    int t = 0;
    int seg_end = readlane_i(pv, 1);
    for (int c0 = e_begin; c0 < e_end; c0 += 64) {
      const int cnt = min(64, e_end - c0);
      int sidx = 0;
      float w = 0.0f;
      if (lane < cnt) {
        sidx = idx[c0 + lane];
        const float v = VALS ? vals[c0 + lane] : 1.0f;
        w = v;
        if (de.active) {
          const uint64_t id = BWD ? edge_base + (uint64_t)(uint32_t)eidv[c0 + lane] : edge_base + (uint64_t)(c0 + lane);
          w = dropedge_weight(de, v, id);
        }
      }
      uint64_t kept = __ballot(w != 0.0f);
      while (kept) {
        int jj[2 * U];
#pragma unroll
        for (int u = 0; u < 2 * U; ++u) {
          if (kept) {
            jj[u] = __builtin_ctzll(kept);
            kept &= kept - 1;
          } else {
            jj[u] = -1;
          }
        }
        float4 xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ja = jj[2 * u], jb = jj[2 * u + 1];
          if (ja >= 0) {
            const int ra = readlane_i(sidx, ja);
            const int rb = jb >= 0 ? readlane_i(sidx, jb) : ra;
            const int r = half ? rb : ra;
            if (ld_ok && (half == 0 || jb >= 0))
              xv[u] = *reinterpret_cast<const float4*>(src + (int64_t)r * lds + coff);
            else
              vzero(xv[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = jj[2 * u + h];
            if (j < 0) continue;
            const int e = c0 + j;
            while (!BWD && e >= seg_end) {  // flush finished segments (wave-uniform)
              if (own) vstore(obase + t * zseg + coff, acc);
              vzero(acc);
              ++t;
              seg_end = readlane_i(pv, t + 1);
            }
            const float wj = readlane_f(w, j);
            if (h == 0) {
              vfma(acc, wj, xv[u]);
            } else {
              const float4 y = make_float4(swap_halves(xv[u].x), swap_halves(xv[u].y), swap_halves(xv[u].z),
                                           swap_halves(xv[u].w));
              vfma(acc, wj, y);
            }
          }
        }
      }
    }
    for (; t < nseg; ++t) {
      if (own) vstore(obase + t * zseg + coff, acc);
      vzero(acc);
    }
  }
}

// Heavy segment h: out = [self term (bwd)] + sum of its chunk partials in
// chunk order.  One wavefront per heavy segment.
template <int VEC, int NV, bool BWD, bool ACCUM = false>
__global__ __launch_bounds__(256) void spmm_fixup_kernel(
    int64_t num_heavy, const int32_t* __restrict__ heavy_seg, const int32_t* __restrict__ heavy_cptr,
    const float* __restrict__ partials, int nseg, int S, int hs, int64_t self_rows, uint64_t self_base,
    const float* __restrict__ dZ, int F, float* __restrict__ out, int64_t ldo, int zseg, DropDev de) {
  using vec_t = typename VecT<VEC>::type;
  de = resolve_key(de);
  const int lane = threadIdx.x & 63;
  const int cbase = blockIdx.y * (64 * VEC * NV);
  const int64_t zstride = (int64_t)(S + hs) * zseg;  // bwd: dZ row stride
  const int64_t wave0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + uniform_i(threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t h = wave0; h < num_heavy; h += nwaves) {
    const int64_t s = heavy_seg[h];
    const int64_t n = s / nseg, t = s % nseg;
    const int c_begin = heavy_cptr[h], c_end = heavy_cptr[h + 1];
    float w_self = 0.0f;
    if (!ACCUM && BWD && hs && n < self_rows) {
      w_self = 1.0f;
      if (de.active && de.drop_self) w_self = dropedge_weight(de, 1.0f, self_base + (uint64_t)n);
    }
    float* orow = BWD ? out + n * ldo : out + n * ldo + (hs + t) * zseg;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int col = cbase + (k * 64 + lane) * VEC;
      if (col >= F) continue;
      vec_t acc;
      vzero(acc);
      if (ACCUM) acc = *reinterpret_cast<const vec_t*>(orow + col);
      if (BWD && w_self != 0.0f) acc = vmul(w_self, *reinterpret_cast<const vec_t*>(dZ + n * zstride + col));
      for (int c = c_begin; c < c_end; ++c) vadd(acc, *reinterpret_cast<const vec_t*>(partials + (int64_t)c * F + col));
      *reinterpret_cast<vec_t*>(orow + col) = acc;
    }
  }
}

__global__ void mask_kernel(DropDev de, uint64_t id_base, int64_t count, uint8_t* __restrict__ keep) {
  de = resolve_key(de);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    keep[i] = dropedge_weight(de, 1.0f, id_base + (uint64_t)i) != 0.0f ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
// split plan construction
// ---------------------------------------------------------------------------
// per row: number of heavy segments (nseg or 0) and chunks
__global__ void split_count_kernel(const int32_t* __restrict__ ptr, int64_t rows, int nseg, int threshold,
                                   int chunk_edges, int64_t* __restrict__ hcnt, int64_t* __restrict__ ccnt) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* p = ptr + r * nseg;
    const bool heavy = p[nseg] - p[0] > threshold;
    int64_t ch = 0;
    if (heavy)
      for (int t = 0; t < nseg; ++t) ch += (p[t + 1] - p[t] + chunk_edges - 1) / chunk_edges;
    hcnt[r] = heavy ? nseg : 0;
    ccnt[r] = ch;
  }
}

__global__ void split_build_kernel(const int32_t* __restrict__ ptr, int64_t rows, int nseg, int threshold,
                                   int chunk_edges, const int64_t* __restrict__ hoff, const int64_t* __restrict__ coff,
                                   int32_t* __restrict__ heavy_seg, int32_t* __restrict__ heavy_cptr,
                                   int32_t* __restrict__ chunk_begin, int32_t* __restrict__ chunk_end,
                                   int64_t num_heavy, int64_t num_chunks) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t* p = ptr + r * nseg;
    if (p[nseg] - p[0] <= threshold) continue;
    int64_t h = hoff[r], c = coff[r];
    for (int t = 0; t < nseg; ++t, ++h) {
      heavy_seg[h] = (int32_t)(r * nseg + t);
      heavy_cptr[h] = (int32_t)c;
      for (int32_t e = p[t]; e < p[t + 1]; e += chunk_edges, ++c) {
        chunk_begin[c] = e;
        chunk_end[c] = min(e + chunk_edges, p[t + 1]);
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) heavy_cptr[num_heavy] = (int32_t)num_chunks;
}

__global__ void split_totals_kernel(const int64_t* __restrict__ hoff, const int64_t* __restrict__ coff, int64_t rows,
                                    int64_t* __restrict__ counts) {
  counts[0] = hoff[rows];
  counts[1] = coff[rows];
}

__global__ void set_zero_i64(int64_t* p) { *p = 0; }

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// workspace: hcnt[rows+1], ccnt[rows+1], hoff[rows+1], coff[rows+1], cub temp
int split_offsets(const int32_t* ptr, int64_t rows, int nseg, int threshold, int chunk_edges, void* ws,
                  size_t ws_bytes, hipStream_t st, int64_t** hoff_out, int64_t** coff_out) {
  const size_t a = align_up((size_t)(rows + 1) * 8);
  char* w = static_cast<char*>(ws);
  int64_t* hcnt = reinterpret_cast<int64_t*>(w);
  int64_t* ccnt = reinterpret_cast<int64_t*>(w + a);
  int64_t* hoff = reinterpret_cast<int64_t*>(w + 2 * a);
  int64_t* coff = reinterpret_cast<int64_t*>(w + 3 * a);
  void* temp = w + 4 * a;
  size_t temp_bytes = ws_bytes - 4 * a;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, 256), 65536));
  if (rows > 0) {
    hipLaunchKernelGGL(split_count_kernel, dim3(grid), dim3(256), 0, st, ptr, rows, nseg, threshold, chunk_edges,
                       hcnt, ccnt);
    GRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(set_zero_i64, dim3(1), dim3(1), 0, st, hcnt + rows);
  hipLaunchKernelGGL(set_zero_i64, dim3(1), dim3(1), 0, st, ccnt + rows);
  GRL_LAUNCH_CHECK();
  GRL_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, hcnt, hoff, (int)(rows + 1), st));
  GRL_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, ccnt, coff, (int)(rows + 1), st));
  *hoff_out = hoff;
  *coff_out = coff;
  return GRL_OK;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
struct LaunchShape {
  int vec, nv, ycols;
};

// Gathered tables above 12 GB keep a whole row (up to 512 columns) in one
// wave.  The spmm_wide path option 1 / 0 forces whole-row / 256-column waves
// (A/B aid and tests).
int64_t wide_table_bytes() {
  const int64_t w = opt(OPT_SPMM_WIDE);
  if (w == 1) return 0;
  if (w == 0) return INT64_MAX;
  return (int64_t)12 << 30;
}

LaunchShape pick_shape(const float* a, const float* b, int64_t lda, int64_t ldb, int F, int64_t table_bytes,
                       int zseg) {
  const bool al = (reinterpret_cast<uintptr_t>(a) % 16 == 0) && (reinterpret_cast<uintptr_t>(b) % 16 == 0) &&
                  (lda % 4 == 0) && (ldb % 4 == 0) && (F % 4 == 0) && (zseg % 4 == 0);
  if (al) {
    // One float4 per lane, 256 columns per wave: wider rows go to more waves
    // along grid.y (each re-reads the row's indices) instead of more
    // registers per wave.  Half / whole rows (tools/ab_spmm_wide.sh): ER
    // d=512 X 2 GB 12.6 / 13.7 ms, X 8 GB 57.6 / 61.2; R-MAT d=512 X 2 GB
    // 25.6 / 28.3.  Far beyond that each half-row visit pays its own address
    // translation and a wave gathers the whole 2 KB row: C5 (R-MAT, X 17 GB)
    // 293 / 233 ms.  Threshold between the measured 8 and 17 GB.
    if (F > 256 && F <= 512 && table_bytes > wide_table_bytes()) return {4, 2, 64 * 4 * 2};
    return {4, 1, 64 * 4};
  }
  const int nv = F <= 64 ? 1 : (F <= 128 ? 2 : 4);
  return {1, nv, 64 * nv};
}

int to_split_dev(const GrlSplitPlan* plan, int F, SplitDev& sp) {
  sp = SplitDev{INT_MAX, 0, nullptr, nullptr, nullptr};
  if (!plan) return GRL_OK;
  GRL_CHECK_ARG(plan->threshold >= 0 && plan->chunk_edges > 0 && plan->num_heavy >= 0 && plan->num_chunks >= 0,
                "split plan: bad threshold/chunk_edges/counts");
  if (plan->num_chunks > 0) {
    GRL_CHECK_ARG(plan->chunk_begin && plan->chunk_end && plan->partials, "split plan: NULL chunk arrays");
    if (plan->partials_capacity < plan->num_chunks * (int64_t)F)
      GRL_FAIL(GRL_E_WORKSPACE, "split plan: partials hold %lld floats, need %lld", (long long)plan->partials_capacity,
               (long long)(plan->num_chunks * (int64_t)F));
  }
  GRL_CHECK_ARG(plan->num_heavy == 0 || (plan->heavy_seg && plan->heavy_cptr), "split plan: NULL heavy arrays");
  sp.threshold = plan->threshold;
  sp.num_chunks = plan->num_chunks;
  sp.chunk_begin = plan->chunk_begin;
  sp.chunk_end = plan->chunk_end;
  sp.partials = plan->partials;
  return GRL_OK;
}

template <bool BWD>
int launch_spmm(int64_t num_rows, int64_t self_rows, int S, int hs, const int32_t* ptr, const int32_t* idx,
                const int32_t* eid, const float* vals, uint64_t edge_base, uint64_t self_base, const float* src,
                int64_t lds, int F, float* out, int64_t ldo, const DropDev& de, const GrlSplitPlan* plan,
                hipStream_t stream, const float* align_probe, int64_t self_row0 = 0, int64_t table_rows = -1,
                int zseg = 0, bool accum = false) {
  if (zseg <= 0) zseg = F;
  if (num_rows == 0) return GRL_OK;
  SplitDev sp;
  int rc = to_split_dev(plan, F, sp);
  if (rc) return rc;
  // gathered table: X (~num_rows rows of lds floats) forward, dZ rows (S per node) backward
  if (table_rows < 0) table_rows = num_rows;
  const int64_t table_bytes = BWD ? table_rows * (int64_t)S * F * 4 : table_rows * lds * 4;
  const LaunchShape sh = pick_shape(src, align_probe, lds, ldo, F, table_bytes, zseg);
  const int64_t items = num_rows + sp.num_chunks;
  const int64_t cap = (int64_t)device_cu_count() * spmm_blocks_per_cu();  // 4-wave blocks per CU in flight
  const int64_t gx = std::min<int64_t>(ceil_div(items, 4), cap);
  const dim3 grid((unsigned)gx, (unsigned)ceil_div(F, sh.ycols));
  const dim3 block(256);
  const bool v = vals != nullptr;
#define GRL_SPMM_LAUNCH(VEC, NV, U, VALS)                                                                  \
  do {                                                                                                     \
    if (BWD && accum)                                                                                      \
      hipLaunchKernelGGL((spmm_kernel<VEC, NV, U, VALS, BWD, true>), grid, block, 0, stream, num_rows,      \
                         self_rows, S, hs, ptr, idx, eid, vals, edge_base, self_base, self_row0, src, lds, F, \
                         out, ldo, zseg, de, sp);                                                          \
    else                                                                                                   \
      hipLaunchKernelGGL((spmm_kernel<VEC, NV, U, VALS, BWD>), grid, block, 0, stream, num_rows, self_rows, \
                         S, hs, ptr, idx, eid, vals, edge_base, self_base, self_row0, src, lds, F, out, ldo, \
                         zseg, de, sp);                                                                    \
  } while (0)
  if (sh.vec == 4) {
    if (sh.nv == 1 && F <= 128 && !(BWD && accum)) {
      // narrow rows (column slices of a pipelined halo): two edges per gather instruction
      if (v)
        hipLaunchKernelGGL((spmm_pair_kernel<8, true, BWD>), grid, block, 0, stream, num_rows, S, hs, ptr, idx, vals,
                           edge_base, self_base, self_row0, src, lds, F, out, ldo, zseg, de, sp, eid, self_rows);
      else
        hipLaunchKernelGGL((spmm_pair_kernel<8, false, BWD>), grid, block, 0, stream, num_rows, S, hs, ptr, idx,
                           vals, edge_base, self_base, self_row0, src, lds, F, out, ldo, zseg, de, sp, eid,
                           self_rows);
    } else if (sh.nv == 1) {
      if (v) GRL_SPMM_LAUNCH(4, 1, GRL_SPMM_U, true); else GRL_SPMM_LAUNCH(4, 1, GRL_SPMM_U, false);
    } else {  // whole 2 KB rows (F in (256, 512]) 4 at a time (8 in flight measured no faster, round 4)
      if (v) GRL_SPMM_LAUNCH(4, 2, 4, true); else GRL_SPMM_LAUNCH(4, 2, 4, false);
    }
  } else {
    if (sh.nv == 1) {
      if (v) GRL_SPMM_LAUNCH(1, 1, 8, true); else GRL_SPMM_LAUNCH(1, 1, 8, false);
    } else if (sh.nv == 2) {
      if (v) GRL_SPMM_LAUNCH(1, 2, 8, true); else GRL_SPMM_LAUNCH(1, 2, 8, false);
    } else {
      if (v) GRL_SPMM_LAUNCH(1, 4, 8, true); else GRL_SPMM_LAUNCH(1, 4, 8, false);
    }
  }
#undef GRL_SPMM_LAUNCH
  GRL_LAUNCH_CHECK();
  if (plan && plan->num_heavy > 0) {
    const dim3 fgrid((unsigned)std::min<int64_t>(ceil_div(plan->num_heavy, 4), cap), grid.y);
    const int nseg = BWD ? 1 : S;
#define GRL_FIXUP_LAUNCH(VEC, NV)                                                                            \
  do {                                                                                                       \
    if (BWD && accum)                                                                                        \
      hipLaunchKernelGGL((spmm_fixup_kernel<VEC, NV, BWD, true>), fgrid, block, 0, stream, plan->num_heavy,  \
                         plan->heavy_seg, plan->heavy_cptr, plan->partials, nseg, S, hs, self_rows, self_base, \
                         src, F, out, ldo, zseg, de);                                                        \
    else                                                                                                     \
      hipLaunchKernelGGL((spmm_fixup_kernel<VEC, NV, BWD>), fgrid, block, 0, stream, plan->num_heavy,        \
                         plan->heavy_seg, plan->heavy_cptr, plan->partials, nseg, S, hs, self_rows, self_base, \
                         src, F, out, ldo, zseg, de);                                                        \
  } while (0)
    if (sh.vec == 4) {
      if (sh.nv == 1) GRL_FIXUP_LAUNCH(4, 1); else GRL_FIXUP_LAUNCH(4, 2);
    } else {
      if (sh.nv == 1) GRL_FIXUP_LAUNCH(1, 1); else if (sh.nv == 2) GRL_FIXUP_LAUNCH(1, 2); else GRL_FIXUP_LAUNCH(1, 4);
    }
#undef GRL_FIXUP_LAUNCH
    GRL_LAUNCH_CHECK();
  }
  return GRL_OK;
}

}  // namespace

// Z rows [0, rows) = rows [r0, r0 + rows) of A_drop X (grl_graphconv_fwd's
// row chunks): rowptr offset by r0 rows (edge positions, hence edge ids, stay
// absolute), self term X row and self id shifted by r0.  Per row identical to
// the whole-graph launch; no split plan (the caller checks).
int spmm_fwd_rows(const GrlTypedCsr* g, int64_t r0, int64_t rows, const float* X, int64_t ldx, int F, float* Z,
                  const GrlDropEdge* de, hipStream_t st) {
  const int hs = g->has_self ? 1 : 0;
  const int64_t ldz = (int64_t)(g->num_types + hs) * F;
  return launch_spmm<false>(rows, rows, g->num_types, hs, g->rowptr + r0 * g->num_types, g->colidx, nullptr, g->vals,
                            g->edge_id_base, g->self_id_base + (uint64_t)r0, X, ldx, F, Z, ldz, to_dev(de), nullptr,
                            st, Z, g->self_row0 + r0, g->num_rows);
}

}  // namespace grl

using namespace grl;

extern "C" void grl_trace_push(const char* name) { roctxRangePushA(name ? name : "grl"); }
extern "C" void grl_trace_pop(void) { roctxRangePop(); }

extern "C" int grl_dropedge_init(GrlDropEdge* de, float p, uint64_t seed, uint64_t call_id, int32_t drop_self) {
  GRL_CHECK_ARG(de != nullptr, "grl_dropedge_init: de is NULL");
  GRL_CHECK_ARG(p >= 0.0f && p == p, "grl_dropedge_init: p must be >= 0 (got %f)", (double)p);
  de->key = dropedge_key(seed, call_id);
  de->drop_self = drop_self ? 1 : 0;
  de->seed_dev = nullptr;
  de->call_id = call_id;
  if (p <= 0.0f) {
    de->active = 0;
    de->threshold = 0;
    de->scale = 1.0f;
    return GRL_OK;
  }
  de->active = 1;
  if (p >= 1.0f) {  // torch: dropout(p=1) zeroes everything
    de->threshold = 0xFFFFFFFFu;
    de->scale = 0.0f;
    return GRL_OK;
  }
  const double thr = std::floor((double)p * 4294967296.0);
  de->threshold = thr >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)thr;
  // torch native_dropout: scale = 1/(1-p) computed in double, applied as float.
  de->scale = (float)(1.0 / (1.0 - (double)p));
  return GRL_OK;
}

extern "C" int grl_dropedge_init_device(GrlDropEdge* de, float p, const uint64_t* seed_dev, uint64_t call_id,
                                        int32_t drop_self) {
  GRL_CHECK_ARG(seed_dev != nullptr, "grl_dropedge_init_device: seed_dev is NULL");
  const int rc = grl_dropedge_init(de, p, 0, call_id, drop_self);
  if (rc) return rc;
  de->seed_dev = seed_dev;
  return GRL_OK;
}

extern "C" int grl_dropedge_mask(const GrlDropEdge* de, uint64_t id_base, int64_t count, uint8_t* keep,
                                 grl_stream_t stream) {
  GRL_CHECK_ARG(count >= 0, "grl_dropedge_mask: negative count");
  if (count == 0) return GRL_OK;
  GRL_CHECK_ARG(keep != nullptr, "grl_dropedge_mask: keep is NULL");
  const DropDev d = to_dev(de);
  const int64_t blocks = std::min<int64_t>(ceil_div(count, 256), 65536);
  hipLaunchKernelGGL(mask_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), d, id_base, count, keep);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

extern "C" int grl_typed_spmm_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx, int32_t F, float* Z,
                                  const GrlDropEdge* de, grl_stream_t stream) {
  TraceRange trace_("grl_typed_spmm_fwd");
  GRL_CHECK_ARG(g != nullptr, "grl_typed_spmm_fwd: graph is NULL");
  GRL_CHECK_ARG(g->num_rows >= 0 && g->num_types >= 1 && g->num_types <= 63,
                "grl_typed_spmm_fwd: num_types must be in [1, 63] (got %d)", g->num_types);
  GRL_CHECK_ARG(F > 0 && ldx >= F, "grl_typed_spmm_fwd: need F > 0 and ldx >= F (F=%d ldx=%lld)", F,
                (long long)ldx);
  if (g->num_rows == 0) return GRL_OK;
  GRL_CHECK_ARG(X && Z && g->rowptr && (g->nnz == 0 || g->colidx), "grl_typed_spmm_fwd: NULL pointer");
  GRL_CHECK_ARG(g->nnz < 2147483647LL, "grl_typed_spmm_fwd: nnz %lld exceeds int32", (long long)g->nnz);
  GRL_CHECK_ARG(g->self_row0 >= 0, "grl_typed_spmm_fwd: negative self_row0");
  const int hs = g->has_self ? 1 : 0;
  const int64_t ldz = (int64_t)(g->num_types + hs) * F;
  return launch_spmm<false>(g->num_rows, g->num_rows, g->num_types, hs, g->rowptr, g->colidx, nullptr, g->vals,
                            g->edge_id_base, g->self_id_base, X, ldx, F, Z, ldz, to_dev(de), g->split,
                            as_stream(stream), Z, g->self_row0);
}

extern "C" int grl_typed_spmm_fwd_slice(const GrlTypedCsr* g, const float* X, int64_t ldx, int32_t F,
                                        int64_t self_col0, float* Z, int64_t ldz, int32_t zseg,
                                        const GrlDropEdge* de, grl_stream_t stream) {
  TraceRange trace_("grl_typed_spmm_fwd_slice");
  GRL_CHECK_ARG(g != nullptr, "grl_typed_spmm_fwd_slice: graph is NULL");
  GRL_CHECK_ARG(g->num_rows >= 0 && g->num_types >= 1 && g->num_types <= 63,
                "grl_typed_spmm_fwd_slice: num_types must be in [1, 63] (got %d)", g->num_types);
  GRL_CHECK_ARG(F > 0 && ldx >= F && zseg >= F && self_col0 >= 0,
                "grl_typed_spmm_fwd_slice: need F > 0, ldx >= F, zseg >= F, self_col0 >= 0 (F=%d ldx=%lld zseg=%d)",
                F, (long long)ldx, zseg, (long long)self_col0);
  const int hs = g->has_self ? 1 : 0;
  GRL_CHECK_ARG(ldz >= (int64_t)(g->num_types + hs - 1) * zseg + F,
                "grl_typed_spmm_fwd_slice: ldz %lld too small for %d segments of stride %d", (long long)ldz,
                g->num_types + hs, zseg);
  if (g->num_rows == 0) return GRL_OK;
  GRL_CHECK_ARG(X && Z && g->rowptr && (g->nnz == 0 || g->colidx), "grl_typed_spmm_fwd_slice: NULL pointer");
  GRL_CHECK_ARG(g->nnz < 2147483647LL, "grl_typed_spmm_fwd_slice: nnz %lld exceeds int32", (long long)g->nnz);
  GRL_CHECK_ARG(g->self_row0 >= 0, "grl_typed_spmm_fwd_slice: negative self_row0");
  return launch_spmm<false>(g->num_rows, g->num_rows, g->num_types, hs, g->rowptr, g->colidx, nullptr, g->vals,
                            g->edge_id_base, g->self_id_base, X, ldx, F, Z, ldz, to_dev(de), g->split,
                            as_stream(stream), Z, self_col0 + g->self_row0, -1, zseg);
}

// dX columns [0, F) = columns [col0, col0 + F) of A_drop^T dZ, dZ segments
// F_total wide (F_total = F, col0 = 0: the whole gradient).
static int spmm_bwd_entry(const char* who, const GrlTypedCsc* g, const float* dZ, int32_t F_total, int32_t col0,
                          int32_t F, float* dX, int64_t lddx, const GrlDropEdge* de, grl_stream_t stream, bool accum) {
  GRL_CHECK_ARG(g != nullptr, "%s: graph is NULL", who);
  GRL_CHECK_ARG(g->num_rows >= 0 && g->self_rows >= 0 && g->self_rows <= g->num_rows, "%s: bad num_rows/self_rows",
                who);
  GRL_CHECK_ARG(g->num_types >= 1 && g->num_types <= 63, "%s: num_types must be in [1, 63]", who);
  GRL_CHECK_ARG(F > 0 && lddx >= F, "%s: need F > 0 and lddx >= F", who);
  GRL_CHECK_ARG(col0 >= 0 && (int64_t)col0 + F <= F_total, "%s: columns [%d, %d) outside the %d-column segments",
                who, col0, col0 + F, F_total);
  if (g->num_rows == 0) return GRL_OK;
  // dZ is never read when no entry and no self term points into it (a node-range shard without own
  // rows or edges: its halo rows' dX is zero, and its empty dZ has no storage)
  GRL_CHECK_ARG((dZ || (g->nnz == 0 && g->self_rows == 0)) && dX && g->colptr && (g->nnz == 0 || (g->zrow && g->eid)),
                "%s: NULL pointer", who);
  const int hs = g->has_self ? 1 : 0;
  return launch_spmm<true>(g->num_rows, g->self_rows, g->num_types, hs, g->colptr, g->zrow, g->eid, g->vals,
                           g->edge_id_base, g->self_id_base, dZ + col0, (int64_t)F_total, F, dX, lddx, to_dev(de),
                           g->split, as_stream(stream), dX, 0, -1, F_total, accum);
}

extern "C" int grl_typed_spmm_bwd_accum(const GrlTypedCsc* g, const float* dZ, int32_t F, float* dX, int64_t lddx,
                                        const GrlDropEdge* de, grl_stream_t stream) {
  TraceRange trace_("grl_typed_spmm_bwd_accum");
  return spmm_bwd_entry("grl_typed_spmm_bwd_accum", g, dZ, F, 0, F, dX, lddx, de, stream, true);
}

extern "C" int grl_typed_spmm_bwd(const GrlTypedCsc* g, const float* dZ, int32_t F, float* dX, int64_t lddx,
                                  const GrlDropEdge* de, grl_stream_t stream) {
  TraceRange trace_("grl_typed_spmm_bwd");
  return spmm_bwd_entry("grl_typed_spmm_bwd", g, dZ, F, 0, F, dX, lddx, de, stream, false);
}

extern "C" int grl_typed_spmm_bwd_slice(const GrlTypedCsc* g, const float* dZ, int32_t F_total, int32_t col0,
                                        int32_t F, float* dX, int64_t lddx, const GrlDropEdge* de,
                                        grl_stream_t stream) {
  TraceRange trace_("grl_typed_spmm_bwd_slice");
  return spmm_bwd_entry("grl_typed_spmm_bwd_slice", g, dZ, F_total, col0, F, dX, lddx, de, stream, false);
}

extern "C" size_t grl_split_plan_workspace_size(int64_t rows) {
  size_t temp = 0;
  int64_t* d = nullptr;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, temp, d, d, (int)std::max<int64_t>(rows + 1, 1)) != hipSuccess)
    return 0;
  return 4 * align_up((size_t)(rows + 1) * 8) + align_up(temp);
}

extern "C" int grl_split_plan_count(const int32_t* ptr, int64_t rows, int32_t nseg, int32_t threshold,
                                    int32_t chunk_edges, int64_t* counts, void* workspace, size_t workspace_bytes,
                                    grl_stream_t stream) {
  GRL_CHECK_ARG(ptr && counts && rows >= 0 && nseg >= 1 && threshold >= 0 && chunk_edges > 0,
                "grl_split_plan_count: bad arguments");
  GRL_CHECK_ARG(rows < 2147483647LL, "grl_split_plan_count: too many rows");
  const size_t need = grl_split_plan_workspace_size(rows);
  if (!workspace || workspace_bytes < need)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_split_plan_count: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  int64_t *hoff, *coff;
  int rc = split_offsets(ptr, rows, nseg, threshold, chunk_edges, workspace, workspace_bytes, st, &hoff, &coff);
  if (rc) return rc;
  hipLaunchKernelGGL(split_totals_kernel, dim3(1), dim3(1), 0, st, hoff, coff, rows, counts);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

extern "C" int grl_split_plan_build(const int32_t* ptr, int64_t rows, int32_t nseg, GrlSplitPlan* plan,
                                    void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  GRL_CHECK_ARG(ptr && plan && rows >= 0 && nseg >= 1, "grl_split_plan_build: bad arguments");
  GRL_CHECK_ARG(plan->threshold >= 0 && plan->chunk_edges > 0, "grl_split_plan_build: bad threshold/chunk_edges");
  GRL_CHECK_ARG(plan->heavy_cptr != nullptr, "grl_split_plan_build: heavy_cptr is NULL");
  GRL_CHECK_ARG(plan->num_heavy == 0 || plan->heavy_seg, "grl_split_plan_build: heavy_seg is NULL");
  GRL_CHECK_ARG(plan->num_chunks == 0 || (plan->chunk_begin && plan->chunk_end),
                "grl_split_plan_build: chunk arrays are NULL");
  GRL_CHECK_ARG(plan->num_chunks < 2147483647LL, "grl_split_plan_build: too many chunks");
  const size_t need = grl_split_plan_workspace_size(rows);
  if (!workspace || workspace_bytes < need)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_split_plan_build: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  int64_t *hoff, *coff;
  int rc = split_offsets(ptr, rows, nseg, plan->threshold, plan->chunk_edges, workspace, workspace_bytes, st, &hoff,
                         &coff);
  if (rc) return rc;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows, 256), 65536));
  hipLaunchKernelGGL(split_build_kernel, dim3(grid), dim3(256), 0, st, ptr, rows, nseg, plan->threshold,
                     plan->chunk_edges, hoff, coff, const_cast<int32_t*>(plan->heavy_seg),
                     const_cast<int32_t*>(plan->heavy_cptr), const_cast<int32_t*>(plan->chunk_begin),
                     const_cast<int32_t*>(plan->chunk_end), plan->num_heavy, plan->num_chunks);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
