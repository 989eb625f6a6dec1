// emb1 = Linear(4369 -> net_size) + ReLU over bag-of-characters rows
// (gnn/models/networks/drop_robust_gcn.py:36,64; the rows come from
// TextlineEncoding, textline_encoding.py:23-42: character counts plus four
// box features, ~7 nonzeros in 4369).
//
//   out[m, :] = relu(bias + sum_{k : V[m,k] != 0, ascending k} V[m,k] * Wt[k, :])
//
// A dense GEMM would spend 2*K*C flops per row on zeros; here one wave scans
// its row 64 entries per lane-load, ballots the nonzeros and gathers only those
// rows of Wt (K x C, L2-resident: 4.5 MB at 4369 x 256).  V is read once,
// coalesced; no CSR is built and nothing syncs with the host, so the model's
// forward stays capturable in a HIP graph.  Sums are one fmaf per nonzero in
// ascending k (deterministic).  The backward (dW = V^T (g * [out > 0]), db)
// is grl_linear_bwd_weight on the MFMA GEMM.
#include "grl_internal.h"

namespace grl {
namespace {

constexpr int U = 8;      // nonzero rows of Wt in flight per wave
constexpr int SCAN = 24;  // 64-entry chunks of a V row loaded together
constexpr int CAP = 512;  // (k, v) list entries per wave in LDS

// Two phases per row, so that the row's latency is a few load rounds rather
// than one per nonzero-holding chunk: (1) scan the row SCAN chunks at a time,
// appending its nonzeros (k ascending) to a per-wave LDS list; (2) walk the
// list U entries at a time, gathering those Wt rows together.  The list is
// flushed early when it would overflow (dense rows), which keeps the order.
template <int CPL>  // output columns per lane: C <= 64 * CPL
__global__ __launch_bounds__(256) void bag_linear_kernel(const float* __restrict__ V, int64_t ldv, int64_t M, int K,
                                                         const float* __restrict__ Wt, int C,
                                                         const float* __restrict__ bias, int relu,
                                                         float* __restrict__ out, int64_t ldo) {
  __shared__ int list_k[4][CAP];
  __shared__ float list_v[4][CAP];
  const int lane = threadIdx.x & 63;
  int* const lk = list_k[threadIdx.x >> 6];
  float* const lv = list_v[threadIdx.x >> 6];
  const uint64_t below = (1ull << lane) - 1;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t m = wave; m < M; m += nwaves) {
    float acc[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) acc[c] = 0.0f;
    int cnt = 0;  // wave-uniform list length
    auto flush = [&]() {
      __builtin_amdgcn_wave_barrier();
      for (int i0 = 0; i0 < cnt; i0 += U) {
        float w[U][CPL], vj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = i0 + u < cnt;
          vj[u] = ok ? lv[i0 + u] : 0.0f;
          const float* wrow = Wt + (int64_t)(ok ? lk[i0 + u] : 0) * C;
#pragma unroll
          for (int cc = 0; cc < CPL; ++cc) {
            const int col = lane + 64 * cc;
            w[u][cc] = (ok && col < C) ? wrow[col] : 0.0f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (i0 + u < cnt) {
#pragma unroll
            for (int cc = 0; cc < CPL; ++cc) acc[cc] = fmaf(vj[u], w[u][cc], acc[cc]);
          }
      }
      __builtin_amdgcn_wave_barrier();
      cnt = 0;
    };
    const float* vrow = V + m * ldv;
    for (int kb = 0; kb < K; kb += 64 * SCAN) {
      float vs[SCAN];  // SCAN chunks of the row in flight at once
#pragma unroll
      for (int c = 0; c < SCAN; ++c) {
        const int k = kb + 64 * c + lane;
        vs[c] = k < K ? vrow[k] : 0.0f;
      }
#pragma unroll
      for (int c = 0; c < SCAN; ++c) {
        const uint64_t nz = __ballot(vs[c] != 0.0f);
        if (nz) {
          const int n = __popcll(nz);
          if (cnt + n > CAP) flush();
          if (vs[c] != 0.0f) {
            const int pos = cnt + __popcll(nz & below);
            lk[pos] = kb + 64 * c + lane;
            lv[pos] = vs[c];
          }
          cnt += n;
        }
      }
    }
    flush();
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int col = lane + 64 * c;
      if (col < C) {
        float x = acc[c] + (bias ? bias[col] : 0.0f);
        if (relu) x = x > 0.0f ? x : 0.0f;
        out[m * ldo + col] = x;
      }
    }
  }
}

template <int CPL>
void launch_bag(const float* V, int64_t ldv, int64_t M, int K, const float* Wt, int C, const float* bias, int relu,
                float* out, hipStream_t st) {
  const int64_t blocks = std::min<int64_t>(ceil_div(M, 4), (int64_t)device_cu_count() * 16);
  hipLaunchKernelGGL((bag_linear_kernel<CPL>), dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, V, ldv,
                     M, K, Wt, C, bias, relu, out, (int64_t)C);
}

}  // namespace
}  // namespace grl

using namespace grl;

extern "C" int grl_bag_linear_fwd(const float* V, int64_t ldv, int64_t M, int32_t K, const float* Wt, int32_t C,
                                  const float* bias, int32_t relu, float* out, grl_stream_t stream) {
  TraceRange trace_("grl_bag_linear_fwd");
  GRL_CHECK_ARG(M >= 0 && K >= 0 && ldv >= K, "grl_bag_linear_fwd: bad sizes (M %lld, K %d, ldv %lld)", (long long)M,
                K, (long long)ldv);
  GRL_CHECK_ARG(C >= 1 && C <= 512, "grl_bag_linear_fwd: output width %d outside [1, 512]", C);
  if (M == 0) return GRL_OK;
  GRL_CHECK_ARG((V || K == 0) && Wt && out, "grl_bag_linear_fwd: NULL pointer");
  hipStream_t st = as_stream(stream);
  if (C <= 64)
    launch_bag<1>(V, ldv, M, K, Wt, C, bias, relu, out, st);
  else if (C <= 128)
    launch_bag<2>(V, ldv, M, K, Wt, C, bias, relu, out, st);
  else if (C <= 256)
    launch_bag<4>(V, ldv, M, K, Wt, C, bias, relu, out, st);
  else
    launch_bag<8>(V, ldv, M, K, Wt, C, bias, relu, out, st);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
