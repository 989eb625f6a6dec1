// One GraphConv layer forward in ONE kernel for gfx950 (inference):
//
//   out = relu?( (A_drop X) W + bias )
//       gnn/models/networks/robust_gcn.py:45-51 (new_V = matmul(A_pre, V);
//       matmul(new_V, h_weights) + bias) and the F.relu of drop_robust_gcn.py:76.
//
// The two-kernel path (grl_typed_spmm_fwd, then the x6 GEMM) writes Z =
// A_drop X to HBM and reads it back: 7.2 GB each way at C3 (N = 1M, L = 6,
// F = 256).  Here Z never leaves the CU.  Two kernels share the pieces:
//  * graphconv_ws_kernel (default): persistent, one workgroup per CU, gather
//    waves and MFMA waves specialised and coupled by an LDS ring of Z tiles
//    (64 rows x 128 columns); see its comment below;
//  * graphconv_fused_kernel (fg_ws = 0): 32-row tiles, every wave
//    alternates gather and multiply phases, three workgroups per CU.
// Shared pieces: the gather sums a wave's rows' segment-t neighbour rows
// (one float4 per lane, one 1 KB row per wave-instruction, the rows' edge
// lists streamed as one list with flushes at row boundaries); the multiply
// runs v_mfma_f32_32x32x16_bf16 six plane products per K16 step into fp32
// accumulators with W pre-split (fused_w_planes_kernel) in MFMA fragment
// order, fetched from L2 straight into registers (one coalesced 1 KB load
// per fragment); bias + ReLU in the epilogue; only out (N x C) is written.
// Arithmetic: each Z element is the same fmaf chain as spmm_kernel (CSR
// order, the same DropEdge weights), split and multiplied in the same K16
// order and product order as gemm_x6_kernel, so the result is bitwise that
// of the two-kernel path (tests/test_gpu_graphconv.py).
#include <cstring>

#include "grl_internal.h"

#include <cstdlib>
#include <mutex>
#include <vector>

// Diagnostic switches (GRL_WS_STAMP, GRL_WS_ONLY_ROLE, GRL_WS_DIAG_*,
// GRL_WS_WHATIF below) are honoured only in diagnostic builds, which
// tools/build_diag.sh and tools/ws_regs.sh make with -DGRL_DIAG; a product
// build ignores them.
#ifndef GRL_DIAG
#undef GRL_WS_STAMP
#undef GRL_WS_ONLY_ROLE
#undef GRL_WS_DIAG_LB
#undef GRL_WS_DIAG_ONE
#undef GRL_WS_WHATIF
#endif

namespace grl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int FG_R = 32;                  // destination rows per tile
constexpr int FG_WAVES = 4;               // waves per workgroup
constexpr int FG_RW = FG_R / FG_WAVES;    // rows per wave in the gather
constexpr int FG_LD = 256 + 8;            // bf16 per Z-tile plane row (F <= 256) + one 16-B pad chunk
constexpr int FG_PLANE = FG_R * FG_LD;    // bf16 per plane
#ifndef GRL_FG_U
#define GRL_FG_U 8
#endif
// GRL_FG_PIPE_IDX=1: segment t+1's edge list and first 64 source rows /
// weights are loaded before segment t is gathered (their latency hidden)
#ifndef GRL_FG_PIPE_IDX
#define GRL_FG_PIPE_IDX 1
#endif
// GRL_FG_BDEPTH: register stages of W fragments in the multiply (2 or 3)
#ifndef GRL_FG_BDEPTH
#define GRL_FG_BDEPTH 2
#endif
#ifndef GRL_FG_WPE
#define GRL_FG_WPE 3
#endif
constexpr int FG_U = GRL_FG_U;            // neighbour rows in flight per wave
constexpr int FG_CB = 8;                  // 32-column blocks of out (C <= 256, zero padded)
constexpr int FG_FRAG = 64 * 8;           // bf16 per MFMA fragment (64 lanes x 8)

// the x6 split, as linear.hip (same instructions, so the same bits)
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  f32x2_t p = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2_t));
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

__device__ __forceinline__ void split3(float4 v, uint2& p0, uint2& p1, uint2& p2) {
  p0.x = pack_bf16(v.x, v.y);
  p0.y = pack_bf16(v.z, v.w);
  float4 r = make_float4(v.x - lo_f(p0.x), v.y - hi_f(p0.x), v.z - lo_f(p0.y), v.w - hi_f(p0.y));
  p1.x = pack_bf16(r.x, r.y);
  p1.y = pack_bf16(r.z, r.w);
  r = make_float4(r.x - lo_f(p1.x), r.y - hi_f(p1.x), r.z - lo_f(p1.y), r.w - hi_f(p1.y));
  p2.x = pack_bf16(r.x, r.y);
  p2.y = pack_bf16(r.z, r.w);
}

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void fma4(float4& acc, float w, const float4& x) {
  acc.x = __builtin_fmaf(w, x.x, acc.x);
  acc.y = __builtin_fmaf(w, x.y, acc.y);
  acc.z = __builtin_fmaf(w, x.z, acc.z);
  acc.w = __builtin_fmaf(w, x.w, acc.w);
}

// W [K][C] row-major -> three bf16 planes in MFMA B-fragment order:
// Wf[ks][cb][q][lane][e] = plane q of W(k = 16 ks + 8 (lane >> 5) + e,
// n = 32 cb + (lane & 31)) for cb < cbn (8: C <= 256, 16: C <= 512), zero for
// n >= C.  Scalar split as
// split_planes_kernel (linear.hip).
// t_cin > 0 (the data-gradient form, grl_graphconv_bwd_data): W(k, n) is the
// block-transposed forward weight, W(s t_cin + c, n) = Wfwd[s C + n][c] for
// the forward's [(L+1) C][t_cin] h_weights (block s of the result = W_s^T).
__global__ void fused_w_planes_kernel(const float* __restrict__ W, int64_t K, int C, uint16_t* __restrict__ Wf,
                                      int64_t t_cin, int cbn) {
  const int64_t total = K * cbn * 32;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const int64_t rest = i >> 9;
    const int cb = (int)(rest % cbn);
    const int64_t ks = rest / cbn;
    const int64_t k = ks * 16 + 8 * (lane >> 5) + e;
    const int n = cb * 32 + (lane & 31);
    const float v = n >= C ? 0.0f : (t_cin > 0 ? W[((k / t_cin) * C + n) * t_cin + k % t_cin] : W[k * C + n]);
    const uint32_t h0 = pack_bf16(v, 0.0f) & 0xFFFFu;
    const float r1 = v - lo_f(h0);
    const uint32_t h1 = pack_bf16(r1, 0.0f) & 0xFFFFu;
    const float r2 = r1 - lo_f(h1);
    const uint32_t h2 = pack_bf16(r2, 0.0f) & 0xFFFFu;
    const int64_t o = (rest * 3) * FG_FRAG + lane * 8 + e;
    Wf[o] = (uint16_t)h0;
    Wf[o + FG_FRAG] = (uint16_t)h1;
    Wf[o + 2 * FG_FRAG] = (uint16_t)h2;
  }
}

// Z-tile plane rows are 528 B apart (33 chunks of 16 B): row r's chunk c
// sits in bank slot (r + c) mod 16, so the fragment reads (ds_read_b128: lane
// groups of 16 rows at one chunk) and the row stores (ds_write_b64, 16 lanes
// on 128 contiguous bytes) are conflict-free, and a fragment's address is a
// per-lane base plus a compile-time offset per K16 step.
__device__ __forceinline__ int zoff(int r, int chunk) { return r * FG_LD + (chunk << 3); }

template <int KS, bool VALS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GRL_FG_WPE, GRL_FG_WPE))) void graphconv_fused_kernel(
    int64_t M, int L, int hs, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const float* __restrict__ vals, uint64_t edge_base, uint64_t self_base, const float* __restrict__ X,
    int64_t ldx, const uint16_t* __restrict__ Wf, const float* __restrict__ bias, int relu,
    float* __restrict__ out, int C, DropDev de) {
  constexpr int F = KS * 16;
  __shared__ __attribute__((aligned(16))) uint16_t zs[3 * FG_PLANE];
  de = resolve_key(de);
  const int lane = threadIdx.x & 63;
  const int wave = uniform_i(threadIdx.x >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * FG_R;
  const int64_t rw0 = m0 + wave * FG_RW;
  const int col = lane * 4;
  const bool col_ok = col < F;

  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;

  // one finished Z row (this wave's row `slot`, this lane's 4 columns) -> planes
  auto flush = [&](int slot, const float4& v) {
    if (col_ok) {
      uint2 q0, q1, q2;
      split3(v, q0, q1, q2);
      const int rr = wave * FG_RW + slot;
      const int off = zoff(rr, lane >> 1) + (lane & 1) * 4;
      *reinterpret_cast<uint2*>(zs + off) = q0;
      *reinterpret_cast<uint2*>(zs + FG_PLANE + off) = q1;
      *reinterpret_cast<uint2*>(zs + 2 * FG_PLANE + off) = q2;
    }
  };

  // ---------------- multiply: acc += Zs(32 x F) W_s(F x 64 cols of this wave) ----------------
  auto multiply = [&](int s) {
    const uint16_t* wk = Wf + ((int64_t)s * KS * FG_CB + wave * 2) * 3 * FG_FRAG + lane * 8;
    constexpr int WSTEP = FG_CB * 3 * FG_FRAG;  // bf16 between K16 steps
    auto load_b = [&](bf16x8_t (&bb)[2][3], int ks) {
      const uint16_t* w = wk + ks * WSTEP;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) bb[j][q] = *reinterpret_cast<const bf16x8_t*>(w + (j * 3 + q) * FG_FRAG);
    };
    auto step = [&](const bf16x8_t (&bb)[2][3], int ks) {
      bf16x8_t a[3];
      const int ao = zoff(l32, 2 * ks + h);
#pragma unroll
      for (int q = 0; q < 3; ++q) a[q] = *reinterpret_cast<const bf16x8_t*>(zs + q * FG_PLANE + ao);
      // gemm_x6_kernel's product order: small terms first, the leading product last
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bb[j][0], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[j][1], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[j][2], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bb[j][0], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[j][1], acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bb[j][0], acc[j], 0, 0, 0);
      }
    };
#if GRL_FG_BDEPTH == 2
    // ping-pong: the next step's W fragments are in flight during this step's MFMAs
    bf16x8_t b0[2][3], b1[2][3];
    load_b(b0, 0);
#pragma unroll 1
    for (int ks = 0; ks < KS; ks += 2) {
      load_b(b1, ks + 1);  // KS is even
      step(b0, ks);
      if (ks + 2 < KS) load_b(b0, ks + 2);
      step(b1, ks + 1);
    }
#else
    // three register stages: step ks's fragments were issued two steps
    // earlier (an L2 hit under load takes longer than one step's 12 MFMAs)
    bf16x8_t bb[3][2][3];
    load_b(bb[0], 0);
    load_b(bb[1], 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 2 < KS) load_b(bb[(ks + 2) % 3], ks + 2);
      // keep the scheduler from sinking the loads into the MFMA stream (its
      // vmcnt waits would then stop on fragments issued a few MFMAs earlier)
      __builtin_amdgcn_sched_barrier(0);
      step(bb[ks % 3], ks);
      __builtin_amdgcn_sched_barrier(0);
    }
#endif
  };

  // ---------------- edge lists, one typed segment ahead ----------------
  // rowptr window of this wave's rows (lane l: rowptr[rw0 L + l], l <= FG_RW L;
  // rows past M read as empty), loaded once per tile
  const int nvalid = (int)max<int64_t>(0, min<int64_t>(FG_RW, M - rw0));
  const int rp = lane <= FG_RW * L ? rowptr[min<int64_t>(rw0 * L + min(lane, nvalid * L), M * L)] : 0;
  struct SegList {
    int b, exc, incl, total;
  };
  // the wave's rows' segment-t edge ranges as one list (lanes < FG_RW: row lane)
  auto seg_list = [&](int t) {
    const int r = min(lane, FG_RW - 1);
    SegList sg;
    sg.b = __shfl(rp, r * L + t);
    const int e1 = __shfl(rp, r * L + t + 1);  // all lanes: ds_bpermute reads only active lanes
    const int cnt = lane < FG_RW ? e1 - sg.b : 0;
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < FG_RW; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    sg.incl = incl;
    sg.exc = incl - cnt;
    sg.total = readlane_i(incl, FG_RW - 1);
    return sg;
  };
  // list entries [c0, c0 + 64): source row and DropEdge weight (0 = dropped / past the end)
  auto fetch = [&](const SegList& sg, int c0, int& sidx, float& w) {
    const int p = c0 + lane;
    int sl = 0;
#pragma unroll
    for (int i = 0; i < FG_RW - 1; ++i) sl += p >= readlane_i(sg.incl, i) ? 1 : 0;
    const int e = __shfl(sg.b, sl) + (p - __shfl(sg.exc, sl));  // CSR position of entry p
    sidx = 0;
    w = 0.0f;
    if (p < sg.total) {
      sidx = colidx[e];
      const float v = VALS ? vals[e] : 1.0f;
      w = de.active ? dropedge_weight(de, v, edge_base + (uint64_t)e) : v;
    }
  };
  SegList cur = seg_list(0);
  int sidx_c;
  float w_c;
  fetch(cur, 0, sidx_c, w_c);  // in flight during segment 0

  // ---------------- segment 0: the identity block of A_pre (robust_gcn.py:58-65) ----------------
  if (hs) {
    float4 xv[FG_RW];
#pragma unroll
    for (int i = 0; i < FG_RW; ++i)
      xv[i] = (rw0 + i < M && col_ok) ? *reinterpret_cast<const float4*>(X + (rw0 + i) * ldx + col) : zero4();
#pragma unroll
    for (int i = 0; i < FG_RW; ++i) {
      float w = 1.0f;
      if (de.active && de.drop_self) w = dropedge_weight(de, 1.0f, self_base + (uint64_t)(rw0 + i));
      const float4 x = w != 0.0f ? make_float4(w * xv[i].x, w * xv[i].y, w * xv[i].z, w * xv[i].w) : zero4();
      flush(i, x);
    }
    __syncthreads();
    multiply(0);
    __syncthreads();
  }

  // ---------------- typed segments: gather Z segment t of this wave's rows, then multiply ----------------
  for (int t = 0; t < L; ++t) {
    // the next segment's list and first 64 entries load while this one gathers and multiplies
    SegList nxt = cur;
    int sidx_n = 0;
    float w_n = 0.0f;
#if GRL_FG_PIPE_IDX
    if (t + 1 < L) {
      nxt = seg_list(t + 1);
      fetch(nxt, 0, sidx_n, w_n);
    }
#else
    if (t > 0) {
      cur = seg_list(t);
      fetch(cur, 0, sidx_c, w_c);
    }
#endif
    const int total = cur.total;
    int slot = 0;
    int bound = readlane_i(cur.incl, 0);  // end position of row `slot` in the combined list
    float4 a4 = zero4();
    for (int c0 = 0; c0 < total; c0 += 64) {
      int sidx = sidx_c;
      float w = w_c;
      if (c0 > 0) fetch(cur, c0, sidx, w);  // rows with more than 64 segment edges together
      uint64_t kept = __ballot(w != 0.0f);
      while (kept) {
        int jj[FG_U];
#pragma unroll
        for (int u = 0; u < FG_U; ++u) {
          if (kept) {
            jj[u] = __builtin_ctzll(kept);
            kept &= kept - 1;
          } else {
            jj[u] = -1;
          }
        }
        float4 xv[FG_U];
#pragma unroll
        for (int u = 0; u < FG_U; ++u) {
          if (jj[u] >= 0) {
            const int r = readlane_i(sidx, jj[u]);
            xv[u] = col_ok ? *reinterpret_cast<const float4*>(X + (int64_t)r * ldx + col) : zero4();
          }
        }
#pragma unroll
        for (int u = 0; u < FG_U; ++u) {
          if (jj[u] >= 0) {
            const int pos = c0 + jj[u];
            while (pos >= bound) {  // rows finished before this entry (wave-uniform)
              flush(slot, a4);
              a4 = zero4();
              ++slot;
              bound = readlane_i(cur.incl, slot);
            }
            fma4(a4, readlane_f(w, jj[u]), xv[u]);
          }
        }
      }
    }
    for (; slot < FG_RW; ++slot) {
      flush(slot, a4);
      a4 = zero4();
    }
    __syncthreads();
    multiply(hs + t);
    __syncthreads();
    cur = nxt;
    sidx_c = sidx_n;
    w_c = w_n;
  }

  // ---------------- epilogue: bias + ReLU, as gemm_x6_kernel ----------------
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = (wave * 2 + j) * 32 + l32;
    if (n >= C) continue;
    const bool epi = bias != nullptr || relu;
    const float bv = bias ? bias[n] : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < M) {
        float v = acc[j][r];
        if (epi) {
          v = v + bv;
          if (relu) v = v > 0.0f ? v : 0.0f;
        }
        out[m * C + n] = v;
      }
    }
  }
}


// ---------------------------------------------------------------------------
// Warp-specialized persistent form (the default).  One workgroup per CU, 12
// waves: PROD gather waves produce Z tiles into a 4-slot LDS ring, 12 - PROD
// MFMA waves consume them, so the HBM-bound gather and the matrix cores run
// at the same time instead of in alternating phases.
//  * a tile is 64 destination rows; a ring unit is a 128-column part of one
//    VIRTUAL segment of it, kept fp32 (64 x 128 floats + a pad chunk per row,
//    33 KB): every W fragment fetched from L2 feeds 64 rows (at 32 rows W's
//    re-read stream alone exceeded what L2 delivers to a CU), and the MFMA
//    waves split their A fragments into the x6 planes as they read them;
//  * virtual segments: a segment of F <= 256 columns is one; F = 256 FV
//    (gcn3's 2C-wide input, C5's d = 512 and its gcn3 at 1024) is FV
//    consecutive 256-column parts, each gathered as its own pass over the
//    segment's edge list (the list and its first 64 sources are reused, the
//    rows' 1 KB halves are what is read).  A finished row then fills only the
//    2 units of its part, so the 4-slot ring keeps a free slot ahead of the
//    MFMA waves at any F.  K order, and so every product, is unchanged;
//  * the unit stream: tile it of this workgroup (tile = blockIdx.x + it *
//    gridDim.x), virtual segment v, part hh -> unit u = (it * S FV + v) NH +
//    hh, ring slot u % 4, generation u / 4;
//  * gather wave p owns rows RW p..RW p + RW - 1 of each tile (RW = 64 /
//    PROD): it streams its rows' segment edges as one list (flushes at row
//    boundaries), gathering one float4 per lane per source row (1 KB per
//    wave-instruction, up to U rows in flight), and a finished row goes to
//    the virtual segment's NH units at once; the next segment's list and
//    first 64 sources load while this one gathers.  Before its first store
//    to a virtual segment's units it waits until the MFMA waves released
//    their slots' previous generation (consumed[slot] >= CONS g); after its
//    last it adds 1 to produced[slot] (release); gather waves never wait for
//    each other;
//  * MFMA wave c owns output columns 64c..64c+63 for all 64 rows (2 x 2
//    MFMA blocks): it waits for produced[slot] >= PROD (g + 1) (acquire), runs
//    the unit's K16 steps (24 MFMAs each) with the next step's W fragments
//    in flight (the W stream crosses unit and tile boundaries: it is
//    periodic in the segment order), then adds 1 to consumed[slot]; after a
//    tile's last unit it stores the tile.
//  * PROD = 8 (C <= 256: 4 MFMA waves) or 4 (C <= 512: 8 MFMA waves, each
//    gather wave 16 rows with two rowptr-window registers and more rows in
//    flight, so the bytes in flight per CU stay the same).
// Every wave walks the same unit sequence and units complete in order, so
// the waits cannot form a cycle; each spin is bounded anyway (a kernel that
// could hang the GPU is not an option): a wave whose bound runs out sets the
// call's status word (vector atomic OR into the caller's workspace) and
// stops; graphconv_status then poisons the call's outputs (stream-ordered).
// Arithmetic per element is the same as graphconv_fused_kernel's (same
// chains, split, K order, product order): bitwise the two-kernel result.
constexpr int WS_R = 64;                   // rows per tile
constexpr int WS_KC = 128;                 // Z columns per ring unit
constexpr int WS_FV = 256;                 // columns per virtual segment (at most)
constexpr int WS_LDF = WS_KC + 4;          // floats per ring row (+ one 16-B pad chunk: conflict-free)
constexpr int WS_SLOT = WS_R * WS_LDF;     // floats per ring slot
constexpr int WS_WAVES = 12;               // gather + MFMA waves per workgroup
constexpr int WS_CB = 2;                   // 32-column blocks per MFMA wave
constexpr int WS_NB = (140 * 1024) / (WS_SLOT * 4);  // ring slots that ~140 KB hold: 4
#ifndef GRL_WS_U
#define GRL_WS_U 12
#endif
#ifndef GRL_WS_U16
#define GRL_WS_U16 12
#endif
constexpr int WS_SPIN = 1 << 24;           // bounded waits (~0.5 s of s_sleep 1); the ws_spin path option overrides
constexpr int WS_STATUS_TIMEOUT = 1;       // status bit: a bounded wait ran out (results invalid)

// GRL_WS_STAMP=1 (diagnostic builds only): every wave adds up the cycles it
// spent waiting on the ring and its total, read back with grl_debug_ws_stats
#ifndef GRL_WS_STAMP
#define GRL_WS_STAMP 0
#endif
// GRL_WS_ONLY_ROLE (register-use diagnostics only, never a working build):
// 1 = compile the gather role alone, 2 = the MFMA role alone
#ifndef GRL_WS_ONLY_ROLE
#define GRL_WS_ONLY_ROLE 0
#endif
// GRL_WS_WHATIF (timing-only diagnostic builds, wrong results): 1 = the MFMA
// waves re-read two steps of W (L2-hot) instead of the stream, 2 = no A split,
// 4 = the gather alone (MFMA waves only release slots), 8 = the MFMA side
// alone (gather waves store zeros for the typed segments)
#ifndef GRL_WS_WHATIF
#define GRL_WS_WHATIF 0
#endif
#if GRL_WS_STAMP
__device__ unsigned long long g_ws_dbg[1024 * 12 * 2];
#endif

__device__ __forceinline__ int lds_load_acq(int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_add_rel(int* p, int v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until *p >= target (wave-uniform); false if the bound ran out, after
// recording it in *status (one lane, vector atomic to global memory)
__device__ __forceinline__ bool wait_ge(int* p, int target, unsigned long long* waited, int spin_limit,
                                        int* status) {
#if GRL_WS_STAMP
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  for (int spin = 0; spin < spin_limit; ++spin) {
    if (lds_load_acq(p) >= target) {
#if GRL_WS_STAMP
      *waited += __builtin_amdgcn_s_memtime() - t0;
#endif
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(status, WS_STATUS_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return false;
}

// KS: K16 steps of one virtual segment (its width / 16); FV: virtual segments
// per segment (F = 16 KS FV); PROD: gather waves (8: C <= 256, 4: C <= 512).
// EID (the data-gradient form over the typed transpose): entry e's DropEdge
// id is edge_base + eid[e] (its forward CSR position) instead of edge_base + e.
// Rows >= self_rows have no self term (a shard's transpose: its halo rows);
// the forward passes M.
#ifndef GRL_WS_DIAG_LB
#define GRL_WS_DIAG_LB (64 * WS_WAVES)  // register-use diagnostics: a smaller bound shows the unconstrained demand
#endif
template <int KS, bool VALS, bool EID = false, int FV = 1, int PROD = 8>
__global__ __launch_bounds__(GRL_WS_DIAG_LB) void graphconv_ws_kernel(
    int64_t M, int L, int hs, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ colidx,
    const float* __restrict__ vals, uint64_t edge_base, uint64_t self_base, const float* __restrict__ X,
    int64_t ldx, const uint16_t* __restrict__ Wf, const float* __restrict__ bias, int relu,
    float* __restrict__ out, int C, DropDev de, int64_t num_tiles, float* __restrict__ Zout, int64_t ldz,
    const int32_t* __restrict__ eid, int64_t self_rows, int spin_limit, int* __restrict__ status,
    int64_t self_row0) {
  constexpr int FVW = KS * 16;                // columns per virtual segment
  constexpr int F = FVW * FV;                 // columns per segment
  constexpr int KC = FVW < WS_KC ? FVW : WS_KC;  // Z columns per unit
  constexpr int NH = FVW / KC;                // units per virtual segment
  constexpr int KSU = KC / 16;                // K16 steps per unit
  constexpr int CONS = WS_WAVES - PROD;       // MFMA waves
  constexpr int CB = CONS * WS_CB;            // 32-column blocks of W's planes (C <= 32 CB)
  constexpr int RW = WS_R / PROD;             // rows per gather wave
  constexpr int U = RW > 8 ? GRL_WS_U16 : GRL_WS_U;  // neighbour rows in flight per gather wave
  static_assert(FV == 1 || FVW == WS_FV, "wide segments are cut into 256-column virtual segments");
  static_assert(NH < WS_NB, "a virtual segment's units are distinct ring slots, and one more is free");
  static_assert(PROD == 8 || PROD == 4, "8 gather + 4 MFMA waves, or 4 + 8 (two 8-row groups per gather wave)");
  __shared__ __attribute__((aligned(16))) float ring[WS_NB * WS_SLOT];
  __shared__ int produced[WS_NB], consumed[WS_NB];
  if (threadIdx.x < WS_NB) {
    produced[threadIdx.x] = 0;
    consumed[threadIdx.x] = 0;
  }
  __syncthreads();
  de = resolve_key(de);
  const int lane = threadIdx.x & 63;
  const int wave = uniform_i(threadIdx.x >> 6);
  const int S = L + hs;
  unsigned long long waited = 0;
#if GRL_WS_STAMP
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  auto stamp_out = [&]() {
    if (lane == 0 && blockIdx.x < 1024) {
      g_ws_dbg[(blockIdx.x * 12 + wave) * 2] = waited;
      g_ws_dbg[(blockIdx.x * 12 + wave) * 2 + 1] = __builtin_amdgcn_s_memtime() - t_start;
    }
  };
#else
  auto stamp_out = [&]() {};
#endif

#if GRL_WS_ONLY_ROLE == 2
  if (false) {
#else
  if (wave < PROD) {
#endif
    // =========================== gather waves ===========================
    // A gather wave's RW rows are NG groups of GR = 8; each group's edges of a
    // segment stream as one list (the rowptr window of 8 rows fits one
    // register), the groups one after the other.
    constexpr int GR = 8;
    constexpr int NG = RW / GR;
#ifndef GRL_WS_SC
#define GRL_WS_SC 4
#endif
    constexpr int SC = GRL_WS_SC;        // self rows loaded per step
    const int col = lane * 4;            // this lane's 4 columns of the virtual segment
    const bool col_ok = col < FVW;
    const int part = col / KC;           // the unit (part of the virtual segment) they belong to
    const int ucol = col - part * KC;    // column within that unit
    int u = 0;                           // first unit of the current virtual segment
    // segment lists: lanes < GR hold row lane's range start b and the
    // inclusive count incl; the first 64 entries' source rows / weights are
    // fetched one list ahead
    struct List {
      int b, incl, exc, total, sidx;
      float w;
    };
    auto make_list = [&](int rp, int t) {
      List ls;
      const int r = min(lane, GR - 1);
      ls.b = __shfl(rp, r * L + t);
      const int e1 = __shfl(rp, r * L + t + 1);  // all lanes: ds_bpermute reads active lanes only
      const int cnt = lane < GR ? e1 - ls.b : 0;
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < GR; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      ls.incl = incl;
      ls.exc = incl - cnt;
      ls.total = readlane_i(incl, GR - 1);
      return ls;
    };
    // list entries [c0, c0 + 64): source row and DropEdge weight (0 = dropped / past the end)
    auto fetch = [&](const List& ls, int c0, int& sidx, float& w) {
      const int pp = c0 + lane;
      int sl = 0;
#pragma unroll
      for (int i = 0; i < GR - 1; ++i) sl += pp >= readlane_i(ls.incl, i) ? 1 : 0;
      const int e = __shfl(ls.b, sl) + (pp - __shfl(ls.exc, sl));  // CSR position of entry pp
      sidx = 0;
      w = 0.0f;
      if (pp < ls.total) {
        sidx = colidx[e];
        const float v = VALS ? vals[e] : 1.0f;
        if (EID)
          w = de.active ? dropedge_weight(de, v, edge_base + (uint64_t)(uint32_t)eid[e]) : v;
        else
          w = de.active ? dropedge_weight(de, v, edge_base + (uint64_t)e) : v;
      }
    };
    for (int64_t tile = blockIdx.x; tile < num_tiles; tile += gridDim.x) {
      const int64_t rw0 = tile * WS_R + wave * RW;
      const int nvalid = (int)max<int64_t>(0, min<int64_t>(RW, M - rw0));
      // rowptr window of each group's rows (lane l: rowptr[(rw0 + 8 g) L + l], l <= 8 L; rows past M read as empty)
      int rp[NG];
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        const int nv = max(0, min(GR, nvalid - gi * GR));
        rp[gi] = lane <= GR * L ? rowptr[min<int64_t>((rw0 + gi * GR) * L + min(lane, nv * L), M * L)] : 0;
      }
      List cur = make_list(rp[0], 0);
      fetch(cur, 0, cur.sidx, cur.w);
      for (int s = 0; s < S; ++s) {
#pragma unroll 1
        for (int hv = 0; hv < FV; ++hv, u += NH) {
          // claim the virtual segment's NH slots (this wave's rows only), once, before the first store
          bool have = false;
          auto claim = [&]() -> bool {
            if (have) return true;
#pragma unroll
            for (int q = 0; q < NH; ++q)
              if (!wait_ge(&consumed[(u + q) % WS_NB], CONS * ((u + q) / WS_NB), &waited, spin_limit, status))
                return false;
            have = true;
            return true;
          };
          float* const dst = ring + ((u + part) % WS_NB) * WS_SLOT + ucol + wave * RW * WS_LDF;
          const float* const xs = X + hv * FVW + col;  // this lane's columns of the virtual segment
          // training forward (Zout): the row also goes to HBM for the weight
          // gradient, with non-temporal stores as spmm_kernel's
          float* const zrow = Zout ? Zout + rw0 * ldz + (int64_t)s * F + hv * FVW + col : nullptr;
          auto flush = [&](int r, const float4& v) {  // r: the wave's row
            if (col_ok) {
              *reinterpret_cast<float4*>(dst + r * WS_LDF) = v;
              if (zrow && r < nvalid) {
                f32x4_t t = {v.x, v.y, v.z, v.w};
                __builtin_nontemporal_store(t, reinterpret_cast<f32x4_t*>(zrow + (int64_t)r * ldz));
              }
            }
          };
          if (s < hs) {
            // identity block of A_pre (robust_gcn.py:58-65): the rows' own features, SC rows at a time
            // (a rolled loop: unrolled, the rows' loads and uniform DropEdge hashes crowd the registers)
#pragma unroll 1
            for (int i0 = 0; i0 < RW; i0 += SC) {
              float4 xv[SC];
#pragma unroll
              for (int i = 0; i < SC; ++i)
                xv[i] = (i0 + i < nvalid && rw0 + i0 + i < self_rows && col_ok)
                            ? *reinterpret_cast<const float4*>(xs + (self_row0 + rw0 + i0 + i) * ldx) : zero4();
              if (!claim()) return;
#pragma unroll
              for (int i = 0; i < SC; ++i) {
                float w = 1.0f;
                if (de.active && de.drop_self) w = dropedge_weight(de, 1.0f, self_base + (uint64_t)(rw0 + i0 + i));
                flush(i0 + i, w != 0.0f ? make_float4(w * xv[i].x, w * xv[i].y, w * xv[i].z, w * xv[i].w) : zero4());
              }
            }
          } else {
#if GRL_WS_WHATIF & 8
            // what-if: the MFMA side alone (typed segments are never gathered)
            if (!claim()) return;
            for (int r = 0; r < RW; ++r) flush(r, zero4());
            if (false)
#endif
#pragma unroll 1
            for (int gi = 0; gi < NG; ++gi) {
              // the next list (next group; else the next segment's first, unless the next virtual part
              // of this segment re-walks this list) and its first 64 entries load while this one gathers
              List nxt = cur;
              if (gi + 1 < NG) {
                nxt = make_list(rp[NG - 1], s - hs);  // NG <= 2: the next group is the last
                fetch(nxt, 0, nxt.sidx, nxt.w);
              } else if (hv + 1 < FV) {
                if (NG > 1) {
                  nxt = make_list(rp[0], s - hs);
                  fetch(nxt, 0, nxt.sidx, nxt.w);
                }
              } else if (s + 1 < S) {
                nxt = make_list(rp[0], s + 1 - hs);
                fetch(nxt, 0, nxt.sidx, nxt.w);
              }
              int row = gi * GR;  // the wave's row being summed
              int bound = readlane_i(cur.incl, 0);
              float4 a4 = zero4();
              for (int c0 = 0; c0 < cur.total; c0 += 64) {
                int sidx = cur.sidx;
                float w = cur.w;
                if (c0 > 0) fetch(cur, c0, sidx, w);  // rows with more than 64 segment edges together
                uint64_t kept = __ballot(w != 0.0f);
                while (kept) {
                  int jj[U];
#pragma unroll
                  for (int q = 0; q < U; ++q) {
                    if (kept) {
                      jj[q] = __builtin_ctzll(kept);
                      kept &= kept - 1;
                    } else {
                      jj[q] = -1;
                    }
                  }
                  float4 xv[U];
#pragma unroll
                  for (int q = 0; q < U; ++q) {
                    if (jj[q] >= 0) {
                      const int src = readlane_i(sidx, jj[q]);
                      // the source row's address is wave-uniform: a scalar base + the lane's column
                      // offset (global_load's saddr form, no 64-bit VALU add per gathered row)
                      // (src, ldx >= 0 and ldx < 2^30: an unsigned 32 x 32 -> 64-bit product of bytes)
                      const uint64_t ra = reinterpret_cast<uint64_t>(X + hv * FVW) +
                                          (uint64_t)(uint32_t)src * (uint32_t)(ldx * 4);
                      typedef __attribute__((address_space(1))) const float gfloat;
                      typedef __attribute__((address_space(1))) const f32x4_t gvec4;
                      gfloat* const rowp = (gfloat*)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ra >> 32)) << 32) |
                                                     (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ra));
                      xv[q] = zero4();
                      if (col_ok) {
                        // C > 256: streaming loads, so the gathered rows (no reuse to speak of in L2) evict
                        // less of W's 11 MB of planes (1.3 % at F = C = 512, profiles/r05_ab_wide_ntx.txt)
                        const f32x4_t t = PROD == 4 ? __builtin_nontemporal_load((gvec4*)(rowp + col))
                                                    : *(gvec4*)(rowp + col);
                        xv[q] = make_float4(t[0], t[1], t[2], t[3]);
                      }
                    }
                  }
#pragma unroll
                  for (int q = 0; q < U; ++q) {
                    if (jj[q] >= 0) {
                      const int pos = c0 + jj[q];
                      while (pos >= bound) {  // rows finished before this entry (wave-uniform)
                        if (!claim()) return;
                        flush(row, a4);
                        a4 = zero4();
                        ++row;
                        bound = readlane_i(cur.incl, row - gi * GR);
                      }
                      fma4(a4, readlane_f(w, jj[q]), xv[q]);
                    }
                  }
                }
              }
              if (!claim()) return;
              for (; row < (gi + 1) * GR; ++row) {
                flush(row, a4);
                a4 = zero4();
              }
              cur = nxt;
            }
          }
          if (lane == 0)
#pragma unroll
            for (int q = 0; q < NH; ++q) lds_add_rel(&produced[(u + q) % WS_NB], 1);
        }
      }
    }
    stamp_out();
  } else {
#if GRL_WS_ONLY_ROLE == 1
    return;
#endif
    // =========================== MFMA waves ===========================
    const int c = wave - PROD;
    const int l32 = lane & 31, h = lane >> 5;
    constexpr int WSTEP = CB * 3 * FG_FRAG;     // bf16 between K16 steps of W
    const int nsteps = S * KS * FV;             // one tile's K16 steps (the W stream's period)
    // uniform base (SGPRs) + the lane's 16 B: saddr loads
    const uint16_t* wbase = Wf + (int64_t)(c * WS_CB) * 3 * FG_FRAG;
    const int loff = lane * 8;
    auto load_b = [&](bf16x8_t (&bb)[WS_CB][3], int gstep) {
#if GRL_WS_WHATIF & 1
      gstep = gstep & 1;  // what-if (timing only): a 2-step W stream that stays in L2
#endif
      const uint16_t* w = wbase + (int64_t)gstep * WSTEP;
#pragma unroll
      for (int j = 0; j < WS_CB; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) bb[j][q] = *reinterpret_cast<const bf16x8_t*>(w + (j * 3 + q) * FG_FRAG + loff);
    };
    f32x16 acc[2][WS_CB];  // [row block][column block]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < WS_CB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    // 12 MFMAs of row block i against both column blocks, gemm_x6_kernel's product order
    auto mma = [&](int i, const bf16x8_t (&b)[WS_CB][3], const bf16x8_t (&a)[3]) {
#pragma unroll
      for (int j = 0; j < WS_CB; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][0], acc[i][j], 0, 0, 0);
      }
    };
    // this lane's 8 k (step ks) of row i*32 + l32 of a fp32 ring unit
    auto read_a = [&](const float* zs, int ks, int i, float4& v0, float4& v1) {
      const float* ar = zs + (i * 32 + l32) * WS_LDF + ks * 16 + h * 8;
      v0 = *reinterpret_cast<const float4*>(ar);
      v1 = *reinterpret_cast<const float4*>(ar + 4);
    };
    auto split_a = [&](const float4& v0, const float4& v1, bf16x8_t (&a)[3]) {
#if GRL_WS_WHATIF & 2
      a[0] = __builtin_bit_cast(bf16x8_t, make_uint4(__float_as_uint(v0.x), __float_as_uint(v0.y), __float_as_uint(v1.x), __float_as_uint(v1.y)));
      a[1] = __builtin_bit_cast(bf16x8_t, make_uint4(__float_as_uint(v0.z), __float_as_uint(v0.w), __float_as_uint(v1.z), __float_as_uint(v1.w)));
      a[2] = a[0];  // what-if (timing only): no split VALU
      return;
#endif
      uint2 p0, p1, p2, r0, r1, r2;
      split3(v0, p0, p1, p2);
      split3(v1, r0, r1, r2);
      a[0] = __builtin_bit_cast(bf16x8_t, make_uint4(p0.x, p0.y, r0.x, r0.y));
      a[1] = __builtin_bit_cast(bf16x8_t, make_uint4(p1.x, p1.y, r1.x, r1.y));
      a[2] = __builtin_bit_cast(bf16x8_t, make_uint4(p2.x, p2.y, r2.x, r2.y));
    };
    // scheduling hint for the region just written: 2 MFMAs, then 3 VALU / 1 MFMA
    auto interleave = [&]() {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
#pragma unroll
      for (int q = 0; q < 10; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    };
    bf16x8_t bb[2][WS_CB][3];
    int nxt = 0;  // K16 step (within the tile) of the next W fragments to load
    load_b(bb[0], nxt);
    nxt = nxt + 1 == nsteps ? 0 : nxt + 1;
    int u = 0;
    for (int64_t tile = blockIdx.x; tile < num_tiles; tile += gridDim.x) {
      for (int su = 0; su < S * FV * NH; ++su, ++u) {
        const int slot = u % WS_NB, g = u / WS_NB;
        const float* zs = ring + slot * WS_SLOT;
        if (!wait_ge(&produced[slot], PROD * (g + 1), &waited, spin_limit, status)) return;
#if GRL_WS_WHATIF & 4
        if (lane == 0) lds_add_rel(&consumed[slot], 1);  // what-if: the gather alone
        continue;
#endif
        // Software-pipelined by row block: the split of the next row block's
        // A fragments (VALU) is interleaved with the current row block's 12
        // MFMAs (an MFMA holds the SIMD's issue for 8 of its 32 cycles; the
        // VALU fits in the rest), instead of running between them.
        bf16x8_t pa[2][3];
        {
          float4 v0, v1;
          read_a(zs, 0, 0, v0, v1);
          split_a(v0, v1, pa[0]);
        }
#pragma unroll
        for (int ks = 0; ks < KSU; ++ks) {  // KSU is even: the stage of step ks is ks & 1
          load_b(bb[(ks + 1) & 1], nxt);
          nxt = nxt + 1 == nsteps ? 0 : nxt + 1;
          const int st = ks & 1;
          float4 v0, v1;
          read_a(zs, ks, 1, v0, v1);
          __builtin_amdgcn_sched_barrier(0);
          mma(0, bb[st], pa[0]);
          split_a(v0, v1, pa[1]);
          interleave();
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 1 < KSU) read_a(zs, ks + 1, 0, v0, v1);
          __builtin_amdgcn_sched_barrier(0);
          mma(1, bb[st], pa[1]);
          if (ks + 1 < KSU) split_a(v0, v1, pa[0]);
          interleave();
          __builtin_amdgcn_sched_barrier(0);
        }
        // the slot's A fragments are in registers once their reads returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) lds_add_rel(&consumed[slot], 1);
      }
      // tile done: bias + ReLU, as gemm_x6_kernel
      const int64_t m0 = tile * WS_R;
      const bool epi = bias != nullptr || relu;
      if (m0 + WS_R <= M) {  // whole tile (wave-uniform): row offsets are uniform multiples of C
#pragma unroll
        for (int j = 0; j < WS_CB; ++j) {
          const int n = (c * WS_CB + j) * 32 + l32;
          const float bv = (bias && n < C) ? bias[n] : 0.0f;
          float* const o = out + (m0 + 4 * h) * C + n;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float v = acc[i][j][r];
              if (epi) {
                v = v + bv;
                if (relu) v = v > 0.0f ? v : 0.0f;
              }
              if (n < C) o[(int64_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * C] = v;
              acc[i][j][r] = 0.0f;
            }
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < WS_CB; ++j) {
        const int n = (c * WS_CB + j) * 32 + l32;
        const float bv = (bias && n < C) ? bias[n] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t m = m0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (m < M && n < C) {
              float v = acc[i][j][r];
              if (epi) {
                v = v + bv;
                if (relu) v = v > 0.0f ? v : 0.0f;
              }
              out[m * C + n] = v;
            }
            acc[i][j][r] = 0.0f;
          }
      }
    }
    stamp_out();
  }
}

}  // namespace

#if GRL_WS_STAMP
extern "C" int grl_debug_ws_stats(unsigned long long* host, int64_t n) {
  GRL_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ws_dbg), (size_t)n * 8));
  return GRL_OK;
}
#endif

// The graphconv_fused path option 0 keeps grl_graphconv_fwd on the
// two-kernel path (A/B aid and tests).
bool graphconv_fused_enabled() { return opt(OPT_GRAPHCONV_FUSED) != 0; }

// The gathered width F: one virtual segment (64, 128, 256) or 2 / 4 of 256
// columns; the output width C <= 512 (C > 256: 4 gather + 8 MFMA waves); L
// <= 7 (a gather wave's rowptr window holds RW L + 1 entries in 1 or 2
// registers).  The phase-alternating kernel (fg_ws = 0) takes F <= 256, C
// <= 256 only; other shapes always run the persistent one.
bool graphconv_fused_shape_ok(int F, int C, int L) {
  return (F == 64 || F == 128 || F == 256 || F == 512 || F == 1024) && C >= 1 && C <= 512 && L >= 1 && L <= 7;
}

// 32-column blocks of W's planes: 8 for C <= 256, 16 for C <= 512
static int planes_cb(int C) { return C <= 256 ? FG_CB : 2 * FG_CB; }

// W's planes, then 256 B whose first word is the call's status
size_t graphconv_fused_ws_bytes(int64_t K, int C) { return (size_t)K * planes_cb(C) * 32 * 3 * 2 + 256; }

static int* ws_status(void* ws, int64_t K, int C) {
  return reinterpret_cast<int*>(static_cast<char*>(ws) + (size_t)K * planes_cb(C) * 32 * 3 * 2);
}

static int ws_spin_limit() {
  const int64_t v = opt(OPT_WS_SPIN);  // test / diagnostic aid: a tiny bound forces the timeout path
  return v > 0 ? (int)v : WS_SPIN;
}

// A persistent kernel whose bounded wait ran out left its outputs partly
// unwritten.  Stream-ordered handling (no host sync on the call): a
// follow-up kernel fills the call's outputs with NaN when the call's status
// word is set, and ORs the entry point's bit into the per-device sticky
// word, which grl_check() reads and clears at the caller's next sync point.
// ws_status_sync = 1 (debug aid) makes an eager call wait for its kernel and
// return GRL_E_TIMEOUT itself, as round 3's entry points did.
__device__ int g_grl_sticky;  // WS_WHO_* bits of the calls whose outputs were poisoned

constexpr int WS_WHO_FWD = 1, WS_WHO_FWD_TRAIN = 2, WS_WHO_BWD_DATA = 4;

__global__ void ws_poison_kernel(const int* __restrict__ status, float* __restrict__ a, int64_t na,
                                 float* __restrict__ b, int64_t nb, int who) {
  if (*status == 0) return;
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_fetch_or(&g_grl_sticky, who, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float nan = __builtin_nanf("");
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * blockDim.x)
    (i < na ? a[i] : b[i - na]) = nan;
}

static const char* who_name(int who) {
  return who == WS_WHO_FWD ? "grl_graphconv_fwd" : who == WS_WHO_FWD_TRAIN ? "grl_graphconv_fwd_train"
                                                                          : "grl_graphconv_bwd_data";
}

static int graphconv_status(const int* status, float* a, int64_t na, float* b, int64_t nb, hipStream_t st, int who) {
  const bool sync = opt(OPT_WS_STATUS_SYNC) != 0;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (sync) GRL_HIP(hipStreamIsCapturing(st, &cs));
  if (!sync || cs != hipStreamCaptureStatusNone) {
    hipLaunchKernelGGL(ws_poison_kernel, dim3(1024), dim3(256), 0, st, status, a, na, b, b ? nb : 0, who);
    GRL_LAUNCH_CHECK();
    return GRL_OK;
  }
  int h = 0;
  GRL_HIP(hipMemcpyAsync(&h, status, sizeof(int), hipMemcpyDeviceToHost, st));
  GRL_HIP(hipStreamSynchronize(st));
  if (h & WS_STATUS_TIMEOUT)
    GRL_FAIL(GRL_E_TIMEOUT, "%s: a wave of the persistent GraphConv kernel gave up waiting on its LDS ring "
             "(bound %d sleeps); the outputs are invalid", who_name(who), ws_spin_limit());
  return GRL_OK;
}

// One launch of the persistent kernel for gathered width F and output width
// C: the template instance for (F, C > 256) with or without edge values /
// eid (the data-gradient form); grid = one workgroup per CU (at most the
// tiles).
template <bool EID>
static void launch_ws(int F, int C, bool v, dim3 grid, hipStream_t st, int64_t M, int L, int hs,
                      const GrlTypedCsr* g, const float* X, int64_t ldx, const uint16_t* Wf, const float* bias,
                      int relu, float* out, DropDev d, int64_t tiles, float* Z, int64_t ldz, const int32_t* eid,
                      int64_t self_rows, int spin, int* status) {
#define GRL_WS_ARGS                                                                                                \
  grid, dim3(64 * WS_WAVES), 0, st, M, L, hs, g->rowptr, g->colidx, g->vals, g->edge_id_base, g->self_id_base, X, \
      ldx, Wf, bias, relu, out, C, d, tiles, Z, ldz, eid, self_rows, spin, status, g->self_row0
#define GRL_WS_ONE(KS_, FV_, PROD_)                                                                                \
  do {                                                                                                            \
    if (v)                                                                                                        \
      hipLaunchKernelGGL((graphconv_ws_kernel<KS_, true, EID, FV_, PROD_>), GRL_WS_ARGS);                         \
    else                                                                                                          \
      hipLaunchKernelGGL((graphconv_ws_kernel<KS_, false, EID, FV_, PROD_>), GRL_WS_ARGS);                        \
  } while (0)
#define GRL_WS_PRODS(KS_, FV_)       \
  do {                               \
    if (C <= 256)                    \
      GRL_WS_ONE(KS_, FV_, 8);       \
    else                             \
      GRL_WS_ONE(KS_, FV_, 4);       \
  } while (0)
#ifdef GRL_WS_DIAG_ONE  // register-use diagnostics only: one instance (F = 256 FV, PROD)
  GRL_WS_ONE(16, GRL_WS_DIAG_FV, GRL_WS_DIAG_PROD);
#else
  switch (F) {
    case 64: GRL_WS_PRODS(4, 1); break;
    case 128: GRL_WS_PRODS(8, 1); break;
    case 256: GRL_WS_PRODS(16, 1); break;
    case 512: GRL_WS_PRODS(16, 2); break;
    default: GRL_WS_PRODS(16, 4); break;  // 1024
  }
#endif
#undef GRL_WS_PRODS
#undef GRL_WS_ONE
#undef GRL_WS_ARGS
}

int graphconv_fused_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx, int F, const float* W, const float* bias,
                        int C, int relu, float* out, const GrlDropEdge* de, void* ws, hipStream_t st, float* Z) {
  const int hs = g->has_self ? 1 : 0;
  const int64_t K = (int64_t)(g->num_types + hs) * F;
  uint16_t* Wf = static_cast<uint16_t*>(ws);
  const int cbn = planes_cb(C);
  const int64_t n_el = K * cbn * 32;
  hipLaunchKernelGGL(fused_w_planes_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n_el, 256), 4096)), dim3(256), 0,
                     st, W, K, C, Wf, (int64_t)0, cbn);
  GRL_LAUNCH_CHECK();
  const int64_t M = g->num_rows;
  const int64_t tiles = ceil_div(M, FG_R);
  GRL_CHECK_ARG(tiles < 2147483647LL, "grl_graphconv_fwd: too many row tiles");
  const DropDev d = to_dev(de);
  const bool v = g->vals != nullptr;
  // the persistent kernel (Z out, wide shapes and row-range views: only it)
  if (opt(OPT_FG_WS) != 0 || Z || F > 256 || C > 256 || g->self_row0 != 0) {
    const int64_t ldz = K;
    const int64_t ws_tiles = ceil_div(M, WS_R);
    const int64_t grid = std::min<int64_t>(ws_tiles, (int64_t)device_cu_count());
    int* status = ws_status(ws, K, C);
    const int spin = ws_spin_limit();
    GRL_HIP(hipMemsetAsync(status, 0, sizeof(int), st));
    launch_ws<false>(F, C, v, dim3((unsigned)grid), st, M, g->num_types, hs, g, X, ldx, Wf, bias, relu, out, d,
                     ws_tiles, Z, ldz, nullptr, M, spin, status);
    GRL_LAUNCH_CHECK();
    return graphconv_status(status, out, M * C, Z, M * ldz, st, Z ? WS_WHO_FWD_TRAIN : WS_WHO_FWD);
  }
#define GRL_FUSED_LAUNCH(KS_)                                                                                        \
  do {                                                                                                               \
    if (v)                                                                                                           \
      hipLaunchKernelGGL((graphconv_fused_kernel<KS_, true>), dim3((unsigned)tiles), dim3(256), 0, st, M,            \
                         g->num_types, hs, g->rowptr, g->colidx, g->vals, g->edge_id_base, g->self_id_base, X, ldx,  \
                         Wf, bias, relu, out, C, d);                                                                 \
    else                                                                                                             \
      hipLaunchKernelGGL((graphconv_fused_kernel<KS_, false>), dim3((unsigned)tiles), dim3(256), 0, st, M,           \
                         g->num_types, hs, g->rowptr, g->colidx, g->vals, g->edge_id_base, g->self_id_base, X, ldx,  \
                         Wf, bias, relu, out, C, d);                                                                 \
  } while (0)
  if (F == 256)
    GRL_FUSED_LAUNCH(16);
  else if (F == 128)
    GRL_FUSED_LAUNCH(8);
  else
    GRL_FUSED_LAUNCH(4);
#undef GRL_FUSED_LAUNCH
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// dX = sum_s G_s W_s^T over the typed transpose gt (grl_graphconv_bwd_data):
// graphconv_ws_kernel with the rows' CSC segments, DropEdge ids through eid,
// and W's planes taken block-transposed.  Cin = G's width (the forward's C),
// Cout = dX's width (the forward's F).
int graphconv_fused_bwd_data(const GrlTypedCsr* gt, const int32_t* eid, const float* G, int64_t ldg, int64_t self_rows,
                             int Cin, const float* W, int Cout, float* dX, float* Gagg, const GrlDropEdge* de, void* ws,
                             hipStream_t st) {
  const int hs = gt->has_self ? 1 : 0;
  const int64_t K = (int64_t)(gt->num_types + hs) * Cin;
  uint16_t* Wf = static_cast<uint16_t*>(ws);
  const int cbn = planes_cb(Cout);
  const int64_t n_el = K * cbn * 32;
  hipLaunchKernelGGL(fused_w_planes_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n_el, 256), 4096)), dim3(256), 0,
                     st, W, K, Cout, Wf, (int64_t)Cin, cbn);
  GRL_LAUNCH_CHECK();
  const int64_t M = gt->num_rows;
  const int64_t ws_tiles = ceil_div(M, WS_R);
  GRL_CHECK_ARG(ws_tiles < 2147483647LL, "grl_graphconv_bwd_data: too many row tiles");
  const int64_t grid = std::min<int64_t>(ws_tiles, (int64_t)device_cu_count());
  const DropDev d = to_dev(de);
  const bool v = gt->vals != nullptr;
  int* status = ws_status(ws, K, Cout);
  const int spin = ws_spin_limit();
  GRL_HIP(hipMemsetAsync(status, 0, sizeof(int), st));
  launch_ws<true>(Cin, Cout, v, dim3((unsigned)grid), st, M, gt->num_types, hs, gt, G, ldg, Wf, nullptr, 0, dX, d,
                  ws_tiles, Gagg, K, eid, self_rows, spin, status);
  GRL_LAUNCH_CHECK();
  return graphconv_status(status, dX, M * Cout, Gagg, M * K, st, WS_WHO_BWD_DATA);
}

}  // namespace grl

namespace grl {
namespace {
// grl_check's read-and-clear in ONE atomic exchange, its old value written
// to a pinned host word: a poison kernel on another stream that lands
// between a read and a separate clear would lose its report.
__global__ void sticky_take_kernel(int* __restrict__ host_word) {
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_exchange(&g_grl_sticky, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(host_word, old, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
}  // namespace
}  // namespace grl

namespace grl {
namespace {
// grl_check's pinned host words: one per host thread at a time (virtual ranks
// check concurrently).  A thread takes a word from a process-wide free list
// (allocating only when the list is empty) and gives it back when it exits,
// so a session that starts fresh threads per run reuses the same few words
// instead of leaking one per thread.  Portable + coherent: usable whichever
// device a later check targets.
std::mutex g_word_mu;
std::vector<int*> g_free_words;
struct CheckWord {
  int* p = nullptr;
  ~CheckWord() {
    if (p) {
      std::lock_guard<std::mutex> lk(g_word_mu);
      g_free_words.push_back(p);
    }
  }
};
}  // namespace
}  // namespace grl

extern "C" int grl_check(grl_stream_t stream) {
  using namespace grl;
  hipStream_t st = as_stream(stream);
  thread_local CheckWord held;
  if (!held.p) {
    {
      std::lock_guard<std::mutex> lk(g_word_mu);
      if (!g_free_words.empty()) {
        held.p = g_free_words.back();
        g_free_words.pop_back();
      }
    }
    if (!held.p) {
      void* p = nullptr;
      GRL_HIP(hipHostMalloc(&p, sizeof(int), hipHostMallocCoherent | hipHostMallocPortable));
      held.p = static_cast<int*>(p);
    }
  }
  int* const word = held.p;
  *reinterpret_cast<volatile int*>(word) = 0;
  hipLaunchKernelGGL(sticky_take_kernel, dim3(1), dim3(64), 0, st, word);
  GRL_LAUNCH_CHECK();
  GRL_HIP(hipStreamSynchronize(st));
  const int h = *reinterpret_cast<volatile int*>(word);
  if (h == 0) return GRL_OK;
  GRL_FAIL(GRL_E_TIMEOUT, "%s%s%s%s%s: a wave of the persistent GraphConv kernel gave up waiting on its LDS ring "
           "(bound %d sleeps); those calls' outputs were set to NaN",
           (h & WS_WHO_FWD) ? "grl_graphconv_fwd" : "", (h & WS_WHO_FWD) && (h & ~WS_WHO_FWD) ? ", " : "",
           (h & WS_WHO_FWD_TRAIN) ? "grl_graphconv_fwd_train" : "",
           (h & WS_WHO_FWD_TRAIN) && (h & WS_WHO_BWD_DATA) ? ", " : "",
           (h & WS_WHO_BWD_DATA) ? "grl_graphconv_bwd_data" : "", ws_spin_limit());
}
