// One GraphConv layer forward in ONE kernel for gfx950 (inference):
//
//   out = relu?( (A_drop X) W + bias )
//       gnn/models/networks/robust_gcn.py:45-51 (new_V = matmul(A_pre, V);
//       matmul(new_V, h_weights) + bias) and the F.relu of drop_robust_gcn.py:76.
//
// The two-kernel path (grl_typed_spmm_fwd, then the x6 GEMM) writes Z =
// A_drop X to HBM and reads it back: 7.2 GB each way at C3 (N = 1M, L = 6,
// F = 256).  Here Z never leaves the CU:
//  * a workgroup (4 waves) owns a tile of 32 destination rows and walks the
//    K dimension one typed segment (F columns of Z) at a time:
//      gather:  each wave sums its 8 rows' segment-t neighbour rows (one
//               float4 per lane, one 1 KB row per wave-instruction, 8 rows
//               in flight, the rows' edge lists streamed as one list with
//               flushes at row boundaries), splits each finished Z row into
//               three bf16 planes (the exact x6 split) and stores it in LDS;
//      multiply: each wave owns 64 output columns and multiplies the 32 x F
//               Z tile with its W slice on v_mfma_f32_32x32x16_bf16, six
//               plane products per K16 step into fp32 accumulators; W comes
//               pre-split in MFMA fragment order straight from L2 into
//               registers (one coalesced 1 KB load per fragment), the next
//               step's fragments in flight during the current step's MFMAs;
//  * 48 KB of LDS per workgroup, so three workgroups share a CU and one's
//    gather overlaps another's MFMAs;
//  * bias + ReLU in the epilogue; only out (N x C) is written.
// Arithmetic: each Z element is the same fmaf chain as spmm_kernel (CSR
// order, the same DropEdge weights), split and multiplied in the same K16
// order and product order as gemm_x6_kernel, so the result is bitwise that
// of the two-kernel path (tests/test_gpu_graphconv.py).
#include "grl_internal.h"

#include <cstdlib>

namespace grl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

constexpr int FG_R = 32;                  // destination rows per tile
constexpr int FG_WAVES = 4;               // waves per workgroup
constexpr int FG_RW = FG_R / FG_WAVES;    // rows per wave in the gather
constexpr int FG_LD = 256;                // bf16 per Z-tile plane row (F <= 256)
constexpr int FG_PLANE = FG_R * FG_LD;    // bf16 per plane
#ifndef GRL_FG_U
#define GRL_FG_U 8
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
// n = 32 cb + (lane & 31)), zero for n >= C.  Scalar split as
// split_planes_kernel (linear.hip).
__global__ void fused_w_planes_kernel(const float* __restrict__ W, int64_t K, int C, uint16_t* __restrict__ Wf) {
  const int64_t total = K * FG_CB * 32;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7), lane = (int)((i >> 3) & 63);
    const int64_t rest = i >> 9;
    const int cb = (int)(rest % FG_CB);
    const int64_t ks = rest / FG_CB;
    const int64_t k = ks * 16 + 8 * (lane >> 5) + e;
    const int n = cb * 32 + (lane & 31);
    const float v = n < C ? W[k * C + n] : 0.0f;
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

// 16-B chunk c of Z-tile row r sits at chunk c ^ (r & 15): the fragment reads
// (ds_read_b128: lane groups of 16 rows at one chunk) and the row stores
// (ds_write_b64) are both conflict-free.
__device__ __forceinline__ int zoff(int r, int chunk) { return r * FG_LD + ((chunk ^ (r & 15)) << 3); }

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
  const int S = L + hs;

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

  for (int s = 0; s < S; ++s) {
    // ---------------- gather: Z segment s of this wave's rows ----------------
    if (s < hs) {
      // identity block of A_pre (robust_gcn.py:58-65): the node's own row
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
    } else {
      const int t = s - hs;
      // lanes < FG_RW: edge range of row rw0 + lane in segment t
      int b = 0, cnt = 0;
      if (lane < FG_RW && rw0 + lane < M) {
        const int64_t q = (rw0 + lane) * L + t;
        b = rowptr[q];
        cnt = rowptr[q + 1] - b;
      }
      int incl = cnt;
#pragma unroll
      for (int d = 1; d < FG_RW; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      const int exc = incl - cnt;
      const int total = readlane_i(incl, FG_RW - 1);
      int slot = 0;
      int bound = readlane_i(incl, 0);  // end position of row `slot` in the combined list
      float4 a4 = zero4();
      for (int c0 = 0; c0 < total; c0 += 64) {
        const int p = c0 + lane;
        int sl = 0;
#pragma unroll
        for (int i = 0; i < FG_RW - 1; ++i) sl += p >= readlane_i(incl, i) ? 1 : 0;
        const int e = __shfl(b, sl) + (p - __shfl(exc, sl));  // CSR position of list entry p
        int sidx = 0;
        float w = 0.0f;
        if (p < total) {
          sidx = colidx[e];
          const float v = VALS ? vals[e] : 1.0f;
          w = de.active ? dropedge_weight(de, v, edge_base + (uint64_t)e) : v;
        }
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
                bound = readlane_i(incl, slot);
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
    }
    __syncthreads();

    // ---------------- multiply: acc += Zs(32 x F) W_s(F x 64 cols of this wave) ----------------
    {
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
    }
    __syncthreads();
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

}  // namespace

// GRL_GRAPHCONV_FUSED=0 (read on every call) keeps grl_graphconv_fwd on the
// two-kernel path (A/B aid and tests).
bool graphconv_fused_enabled() {
  const char* e = getenv("GRL_GRAPHCONV_FUSED");
  return !(e && e[0] == '0');
}

bool graphconv_fused_shape_ok(int F, int C) { return (F == 256 || F == 128 || F == 64) && C >= 1 && C <= 256; }

size_t graphconv_fused_ws_bytes(int64_t K) { return (size_t)K * FG_CB * 32 * 3 * 2 + 256; }

int graphconv_fused_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx, int F, const float* W, const float* bias,
                        int C, int relu, float* out, const GrlDropEdge* de, void* ws, hipStream_t st) {
  const int hs = g->has_self ? 1 : 0;
  const int64_t K = (int64_t)(g->num_types + hs) * F;
  uint16_t* Wf = static_cast<uint16_t*>(ws);
  const int64_t n_el = K * FG_CB * 32;
  hipLaunchKernelGGL(fused_w_planes_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n_el, 256), 4096)), dim3(256), 0,
                     st, W, K, C, Wf);
  GRL_LAUNCH_CHECK();
  const int64_t M = g->num_rows;
  const int64_t tiles = ceil_div(M, FG_R);
  GRL_CHECK_ARG(tiles < 2147483647LL, "grl_graphconv_fwd: too many row tiles");
  const DropDev d = to_dev(de);
  const bool v = g->vals != nullptr;
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

}  // namespace grl
