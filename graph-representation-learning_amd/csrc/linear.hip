// fp32 post-aggregation linear on the gfx950 matrix cores.
//
// Replaces  V_out = torch.matmul(new_V, self.h_weights) + self.bias
// (gnn/models/networks/robust_gcn.py:50) and optionally the F.relu applied
// to the layer output (gnn/models/networks/drop_robust_gcn.py:76,80,85).
//
// v_mfma_f32_32x32x2_f32: exact f32 products (one rounding per fmaf), the
// only MFMA use in the engine.  Block tile 128 x 128, K staged 32 deep
// through LDS; 4 waves, each owning a 64 x 64 sub-tile (2 x 2 MFMA tiles,
// 64 accumulator registers).  Inside a K-step of 8 the two half-waves take
// k = 4h + s (s = 0..3) so every operand fragment is one ds_read_b128; the
// sum over k is the same set of products in a different order.
#include "grl_internal.h"

namespace grl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int LDA = BK + 4;  // 144 B row stride: conflict-free ds_read_b128
constexpr int LDB = BK + 4;

template <bool ALIGNED>
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ Z, int64_t ldz,
                                                     const float* __restrict__ W, const float* __restrict__ bias,
                                                     float* __restrict__ out, int64_t M, int K, int C, int relu) {
  __shared__ __attribute__((aligned(16))) float As[BM * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LDB];  // transposed: Bs[n][k]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int l32 = lane & 31, h = lane >> 5;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  for (int k0 = 0; k0 < K; k0 += BK) {
    // ---- stage A tile: BM x BK (rows of Z) --------------------------------
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = tid + it * 256;  // 1024 float4 slots
      const int r = idx >> 3, c4 = (idx & 7) * 4;
      const int64_t gm = m0 + r;
      const int gk = k0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gm < M) {
        const float* p = Z + gm * ldz + gk;
        if (ALIGNED) {
          if (gk < K) v = *reinterpret_cast<const float4*>(p);
        } else {
          if (gk + 0 < K) v.x = p[0];
          if (gk + 1 < K) v.y = p[1];
          if (gk + 2 < K) v.z = p[2];
          if (gk + 3 < K) v.w = p[3];
        }
      }
      *reinterpret_cast<float4*>(&As[r * LDA + c4]) = v;
    }
    // ---- stage B tile: BK x BN of W, stored transposed ---------------------
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = tid + it * 256;
      const int kr = idx >> 5, c4 = (idx & 31) * 4;
      const int gk = k0 + kr;
      const int gn = n0 + c4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gk < K) {
        const float* p = W + (int64_t)gk * C + gn;
        if (ALIGNED) {
          if (gn < C) v = *reinterpret_cast<const float4*>(p);
        } else {
          if (gn + 0 < C) v.x = p[0];
          if (gn + 1 < C) v.y = p[1];
          if (gn + 2 < C) v.z = p[2];
          if (gn + 3 < C) v.w = p[3];
        }
      }
      Bs[(c4 + 0) * LDB + kr] = v.x;
      Bs[(c4 + 1) * LDB + kr] = v.y;
      Bs[(c4 + 2) * LDB + kr] = v.z;
      Bs[(c4 + 3) * LDB + kr] = v.w;
    }
    __syncthreads();

#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
      float4 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = *reinterpret_cast<const float4*>(&As[(wm * 64 + i * 32 + l32) * LDA + kk + 4 * h]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b[j] = *reinterpret_cast<const float4*>(&Bs[(wn * 64 + j * 32 + l32) * LDB + kk + 4 * h]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }

  // ---- epilogue: bias (+ReLU), C/D map col = lane&31, row = (r&3)+8(r>>2)+4h
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int gn = n0 + wn * 64 + j * 32 + l32;
    if (gn >= C) continue;
    const float bv = bias ? bias[gn] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < M) {
          float v = acc[i][j][r] + bv;
          if (relu) v = v > 0.0f ? v : 0.0f;
          out[gm * C + gn] = v;
        }
      }
    }
  }
}

}  // namespace
}  // namespace grl

using namespace grl;

extern "C" int grl_linear_fwd(const float* Z, int64_t ldz, const float* W, const float* bias, float* out, int64_t M,
                              int32_t K, int32_t C, int32_t relu, grl_stream_t stream) {
  GRL_CHECK_ARG(M >= 0 && K >= 0 && C >= 0, "grl_linear_fwd: negative size");
  GRL_CHECK_ARG(ldz >= K, "grl_linear_fwd: ldz (%lld) < K (%d)", (long long)ldz, K);
  if (M == 0 || C == 0) return GRL_OK;
  GRL_CHECK_ARG(Z && W && out, "grl_linear_fwd: NULL pointer");
  GRL_CHECK_ARG(ceil_div(M, BM) < 2147483647LL && ceil_div(C, BN) < 65536, "grl_linear_fwd: grid too large");
  const bool aligned = (reinterpret_cast<uintptr_t>(Z) % 16 == 0) && (reinterpret_cast<uintptr_t>(W) % 16 == 0) &&
                       (ldz % 4 == 0) && (K % 4 == 0) && (C % 4 == 0);
  const dim3 grid((unsigned)ceil_div(M, BM), (unsigned)ceil_div(C, BN));
  if (aligned)
    hipLaunchKernelGGL(linear_kernel<true>, grid, dim3(256), 0, as_stream(stream), Z, ldz, W, bias, out, M, K, C,
                       relu);
  else
    hipLaunchKernelGGL(linear_kernel<false>, grid, dim3(256), 0, as_stream(stream), Z, ldz, W, bias, out, M, K, C,
                       relu);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
