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
// ascending k (deterministic).  The weight gradient (dWt = V^T g', db = sum g',
// g' = g * [out > 0]) is sparse too (grl_bag_linear_bwd_weight below): only
// the nonzeros of V cost a row of g'.
#include "grl_internal.h"

#include <cstdlib>

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


// dWt[k, :] = sum_{m : V[m,k] != 0, ascending m} V[m,k] g'[m, :]  (db: k = K, V = 1)
//
// A workgroup owns DW_KB columns of V and one range of rows (blockIdx.y; the
// ranges' partials are added in range order by bag_dw_reduce_kernel).  Per
// chunk of DW_ROWS rows: (1) scan -- wave w reads columns 4w..4w+3, lane =
// row, and ballots append the nonzeros to an LDS list column by column
// entries in ascending row order);
// the next chunk's loads are issued before (2) accumulate -- the whole
// workgroup walks the list DW_U entries at a time (thread t owns output
// columns t, t+256; two batches of DW_U rows of g' in flight), summing each
// column's run in registers (one fmaf per nonzero, ascending rows) and adding
// the run to the column's LDS total (chunk by chunk).  Deterministic; g' (M x C) is read once per nonzero, V
// once.  A dense GEMM would spend 2*M*K*C flops on zeros (224 GFLOP at
// M = 100k, K = 4369, C = 256).
constexpr int DW_KB = 16;
constexpr int DW_ROWS = 256;  // chunk height (A/B 64 / 128 / 256 at M = 100k: 1.83 / 1.62 / 1.52 ms)
constexpr int DW_U = 16;
// ent_key packs (column in block << 8) | row in chunk
static_assert(DW_ROWS <= 256 && DW_KB <= 16, "bag_dw_kernel's ent_key holds the row in 8 bits");
// LDS per workgroup: ent_key + ent_v (2 x 4 x DW_KB x DW_ROWS B) + acc_s (4 x DW_KB x 256 x CPT B) + 16 B.
// CPT = 2 (C in (256, 512]) needs 65,552 B: more than 64 KiB, within gfx950's 160 KB per workgroup.
static_assert(2 * 4 * DW_KB * DW_ROWS + 4 * DW_KB * 256 * 2 + 16 <= 160 * 1024, "bag_dw_kernel<2> exceeds gfx950 LDS");

template <int CPT>  // output columns per thread: C <= 256 * CPT
__global__ __launch_bounds__(256) void bag_dw_kernel(const float* __restrict__ V, int64_t ldv, int64_t M, int K,
                                                     int Keff, const float* __restrict__ g,
                                                     const float* __restrict__ relu_out, int C,
                                                     int64_t rows_per_split, float* __restrict__ part) {
  constexpr int Q = DW_ROWS / 64;
  __shared__ int ent_key[DW_KB * DW_ROWS];  // (column in block << 8) | row in chunk
  __shared__ float ent_v[DW_KB * DW_ROWS];
  __shared__ int cnt_s[4];
  __shared__ float acc_s[DW_KB][256 * CPT];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int k0 = blockIdx.x * DW_KB;
  const int64_t r_lo = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r_hi = min(M, r_lo + rows_per_split);
#pragma unroll
  for (int j = 0; j < DW_KB; ++j)
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) acc_s[j][t + 256 * cc] = 0.0f;
  // lane = row; wave w's columns 4w..4w+3
  auto load = [&](float (&vs)[Q][4], int64_t r0) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int64_t row = r0 + 64 * q + lane;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int k = k0 + 4 * w + jj;
        vs[q][jj] = (row < r_hi && k < Keff) ? (k < K ? V[row * ldv + k] : 1.0f) : 0.0f;
      }
    }
  };
  float vs[Q][4];
  load(vs, r_lo);
  for (int64_t r0 = r_lo; r0 < r_hi; r0 += DW_ROWS) {
    // list order: column (wave w holds 4w..4w+3), then row ascending -- each
    // column is one run of the list
    const uint64_t below = (1ull << lane) - 1;
    uint64_t nz[4][Q];
    int wtot = 0;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        nz[jj][q] = __ballot(vs[q][jj] != 0.0f);
        wtot += __popcll(nz[jj][q]);
      }
    if (lane == 0) cnt_s[w] = wtot;
    __syncthreads();
    int pos = 0, total = 0;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      if (ww == w) pos = total;
      total += cnt_s[ww];
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (vs[q][jj] != 0.0f) {
          const int p = pos + __popcll(nz[jj][q] & below);
          ent_key[p] = ((4 * w + jj) << 8) | (64 * q + lane);
          ent_v[p] = vs[q][jj];
        }
        pos += __popcll(nz[jj][q]);
      }
    __syncthreads();
    if (r0 + DW_ROWS < r_hi) load(vs, r0 + DW_ROWS);  // in flight under the accumulation
    // two batches of DW_U rows of g' in flight: batch i+1 is issued before batch i is added
    float gv[2][DW_U][CPT], vv[2][DW_U];
    int kk[2][DW_U];
    auto fetch = [&](int b, int i0) {
#pragma unroll
      for (int u = 0; u < DW_U; ++u) {
        const bool ok = i0 + u < total;
        const int key = ok ? ent_key[i0 + u] : 0;
        vv[b][u] = ok ? ent_v[i0 + u] : 0.0f;
        kk[b][u] = key >> 8;
        const int64_t row = r0 + (key & 255);
#pragma unroll
        for (int cc = 0; cc < CPT; ++cc) {
          const int c = min(t + 256 * cc, C - 1);
          float x = g[row * C + c];
          if (relu_out && !(relu_out[row * C + c] > 0.0f)) x = 0.0f;
          gv[b][u][cc] = x;
        }
      }
    };
    // the run of the current column sums in registers; it is added to the
    // column's LDS total when the column changes (kk is workgroup-uniform)
    float run[CPT];
    int cur = -1;
#pragma unroll
    for (int cc = 0; cc < CPT; ++cc) run[cc] = 0.0f;
    auto close_run = [&]() {
      if (cur >= 0)
#pragma unroll
        for (int cc = 0; cc < CPT; ++cc) acc_s[cur][t + 256 * cc] += run[cc];
    };
    auto add = [&](int b, int i0) {
#pragma unroll
      for (int u = 0; u < DW_U; ++u)
        if (i0 + u < total) {
          if (kk[b][u] != cur) {
            close_run();
            cur = kk[b][u];
#pragma unroll
            for (int cc = 0; cc < CPT; ++cc) run[cc] = 0.0f;
          }
#pragma unroll
          for (int cc = 0; cc < CPT; ++cc) run[cc] = fmaf(vv[b][u], gv[b][u][cc], run[cc]);
        }
    };
    if (total > 0) fetch(0, 0);
    for (int i0 = 0; i0 < total; i0 += 2 * DW_U) {
      if (i0 + DW_U < total) fetch(1, i0 + DW_U);
      add(0, i0);
      if (i0 + DW_U < total) {
        if (i0 + 2 * DW_U < total) fetch(0, i0 + 2 * DW_U);
        add(1, i0 + DW_U);
      }
    }
    close_run();
    __syncthreads();  // the list is refilled by the next chunk
  }
#pragma unroll
  for (int j = 0; j < DW_KB; ++j) {
    const int k = k0 + j;
    if (k < Keff)
#pragma unroll
      for (int cc = 0; cc < CPT; ++cc) {
        const int c = t + 256 * cc;
        if (c < C) part[((int64_t)blockIdx.y * Keff + k) * C + c] = acc_s[j][c];
      }
  }
}

// dWt / db = the row ranges' partials added in range order
__global__ void bag_dw_reduce_kernel(const float* __restrict__ part, int S, int K, int Keff, int C,
                                     float* __restrict__ dWt, float* __restrict__ db) {
  const int64_t n = (int64_t)Keff * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.0f;
    for (int s = 0; s < S; ++s) a += part[(int64_t)s * n + i];
    if (i < (int64_t)K * C)
      dWt[i] = a;
    else
      db[i - (int64_t)K * C] = a;
  }
}

// Row splits of the sparse dW: up to 128 ranges of >= 512 rows, and at most
// DW_PART_BUDGET bytes of fp32 partials (every split writes its whole
// Keff x C slab, which the ordered reduce reads back).  A workgroup walks its
// range's chunks one after another, so the split count is the kernel's
// parallelism: at M = 100k, K = 4369, C = 256 (kernel + reduce,
// tools/probe_bag_dw_splits.py, profiles/r03_probe_bag_dw_splits.json)
// S = 16 / 29 / 64 / 128 / 196 take 3.41 / 2.33 / 1.70 / 1.52 / 1.57 ms; a
// 128 MB budget (S = 29 there) cost the 100k-node train step 0.9 ms, so the
// budget is 1 GiB (S = 128: 573 MB at C = 256; C = 512: S = 120, 1.07 GB).
constexpr int64_t DW_PART_BUDGET = 1ll << 30;
int bag_dw_splits(int64_t M, int64_t Keff, int64_t C) {
  const int64_t by_mem = std::max<int64_t>(1, DW_PART_BUDGET / std::max<int64_t>(1, Keff * C * 4));
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(128, by_mem), ceil_div(M, 512)));
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

extern "C" size_t grl_bag_linear_bwd_weight_workspace_size(int64_t M, int32_t K, int32_t C) {
  if (M <= 0 || K < 0 || C <= 0) return 0;
  return (size_t)bag_dw_splits(M, (int64_t)K + 1, C) * (size_t)(K + 1) * (size_t)C * 4;
}

extern "C" int grl_bag_linear_bwd_weight(const float* V, int64_t ldv, const float* g, const float* relu_out,
                                         float* dWt, float* db, int64_t M, int32_t K, int32_t C, void* workspace,
                                         size_t workspace_bytes, grl_stream_t stream) {
  TraceRange trace_("grl_bag_linear_bwd_weight");
  GRL_CHECK_ARG(M >= 0 && K >= 0 && ldv >= K, "grl_bag_linear_bwd_weight: bad sizes (M %lld, K %d, ldv %lld)",
                (long long)M, K, (long long)ldv);
  GRL_CHECK_ARG(C >= 1 && C <= 512, "grl_bag_linear_bwd_weight: output width %d outside [1, 512]", C);
  GRL_CHECK_ARG(dWt || K == 0, "grl_bag_linear_bwd_weight: NULL dWt");
  hipStream_t st = as_stream(stream);
  if (M == 0) {  // no rows: zero gradients
    if (K) GRL_HIP(hipMemsetAsync(dWt, 0, (size_t)K * C * 4, st));
    if (db) GRL_HIP(hipMemsetAsync(db, 0, (size_t)C * 4, st));
    return GRL_OK;
  }
  GRL_CHECK_ARG((V || K == 0) && g, "grl_bag_linear_bwd_weight: NULL pointer");
  const int Keff = K + (db ? 1 : 0);
  if (Keff == 0) return GRL_OK;
  const int S = bag_dw_splits(M, (int64_t)K + 1, C);  // the size query's split count (db or not)
  const size_t need = (size_t)S * (size_t)Keff * (size_t)C * 4;
  if (!workspace || workspace_bytes < need)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_bag_linear_bwd_weight: workspace %zu < %zu", workspace_bytes, need);
  float* part = static_cast<float*>(workspace);
  const int64_t rps = ceil_div(M, (int64_t)S);
  const dim3 grid((unsigned)ceil_div((int64_t)Keff, (int64_t)DW_KB), (unsigned)ceil_div(M, rps));
  if (C <= 256)
    hipLaunchKernelGGL((bag_dw_kernel<1>), grid, dim3(256), 0, st, V, ldv, M, K, Keff, g, relu_out, C, rps,
                       part);
  else
    hipLaunchKernelGGL((bag_dw_kernel<2>), grid, dim3(256), 0, st, V, ldv, M, K, Keff, g, relu_out, C, rps,
                       part);
  GRL_LAUNCH_CHECK();
  const int64_t n = (int64_t)Keff * C;
  hipLaunchKernelGGL(bag_dw_reduce_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, (int64_t)256), 8192)),
                     dim3(256), 0, st, part, (int)grid.y, K, Keff, C, dWt, db);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
