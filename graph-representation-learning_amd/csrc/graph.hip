// Graph-format kernels: dense adjacency -> typed CSR (the sparse drop-in for
// GraphConv.preprocess_adj, gnn/models/networks/robust_gcn.py:53-72),
// typed CSR -> CSC for the backward pass, and the seeded synthetic
// Erdos-Renyi / R-MAT generators of the benchmark configs.
//
// None of this is on the per-layer hot path: a graph is converted once per
// forward (the reference calls preprocess_adj once per forward in
// efficient_mode, drop_robust_gcn.py:69) and reused by all three GraphConv
// layers and their backward.
#include <hipcub/hipcub.hpp>

#include "grl_internal.h"

namespace grl {
namespace {

// ---------------------------------------------------------------------------
// dense -> typed CSR
// ---------------------------------------------------------------------------
// One wavefront per (b, n, t) row; 64 consecutive m per ballot.
__global__ __launch_bounds__(256) void dense_count_kernel(const float* __restrict__ A, int64_t B, int64_t N, int L,
                                                          int64_t sb, int64_t sn, int64_t st, int64_t sm,
                                                          int32_t* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const int64_t rows = B * N * L;
  const int64_t wave0 = (int64_t)blockIdx.x * 4 + uniform_i(threadIdx.x >> 6);
  for (int64_t r = wave0; r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t t = r % L;
    const int64_t bn = r / L;
    const int64_t n = bn % N;
    const int64_t b = bn / N;
    const float* row = A + b * sb + n * sn + t * st;
    int cnt = 0;
    for (int64_t m0 = 0; m0 < N; m0 += 64) {
      const int64_t m = m0 + lane;
      const bool nz = m < N && row[m * sm] != 0.0f;
      cnt += __popcll(__ballot(nz));
    }
    if (lane == 0) counts[r] = cnt;
  }
}

__global__ __launch_bounds__(256) void dense_fill_kernel(const float* __restrict__ A, int64_t B, int64_t N, int L,
                                                         int64_t sb, int64_t sn, int64_t st, int64_t sm,
                                                         const int32_t* __restrict__ rowptr,
                                                         int32_t* __restrict__ colidx, float* __restrict__ vals) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t rows = B * N * L;
  const int64_t wave0 = (int64_t)blockIdx.x * 4 + uniform_i(threadIdx.x >> 6);
  for (int64_t r = wave0; r < rows; r += (int64_t)gridDim.x * 4) {
    const int64_t t = r % L;
    const int64_t bn = r / L;
    const int64_t n = bn % N;
    const int64_t b = bn / N;
    const float* row = A + b * sb + n * sn + t * st;
    int pos = rowptr[r];
    for (int64_t m0 = 0; m0 < N; m0 += 64) {
      const int64_t m = m0 + lane;
      const float v = m < N ? row[m * sm] : 0.0f;
      const bool nz = v != 0.0f;
      const uint64_t bal = __ballot(nz);
      if (nz) {
        const int o = pos + __popcll(bal & lt_mask);
        colidx[o] = (int32_t)(b * N + m);
        if (vals) vals[o] = v;
      }
      pos += __popcll(bal);
    }
  }
}

__global__ void set_tail_zero(int32_t* p) { *p = 0; }


__global__ void iota_kernel(int32_t* __restrict__ v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (int32_t)i;
}

// largest s with rowptr[s] <= e  (rowptr nondecreasing, rowptr[0] = 0 <= e)
__device__ __forceinline__ int64_t segment_of(const int32_t* __restrict__ rowptr, int64_t nseg, int32_t e) {
  int64_t lo = 0, hi = nseg;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (rowptr[mid] <= e)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__global__ void csc_gather_kernel(const int32_t* __restrict__ rowptr, int64_t nseg, int S, int hs,
                                  const int32_t* __restrict__ eid, const float* __restrict__ vals_in, int64_t nnz,
                                  int32_t* __restrict__ zrow, float* __restrict__ vals_out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t e = eid[i];
    const int64_t s = segment_of(rowptr, nseg, e);
    const int64_t n = s / S, t = s % S;
    zrow[i] = (int32_t)(n * (S + hs) + hs + t);
    if (vals_out) vals_out[i] = vals_in[e];
  }
}

// colptr[c] = first position whose key >= c   (c in [0, ncols])
__global__ void lower_bound_ptr_kernel(const int32_t* __restrict__ keys, int64_t nnz, int64_t ncols,
                                       int32_t* __restrict__ colptr) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c <= ncols; c += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < c)
        lo = mid + 1;
      else
        hi = mid;
    }
    colptr[c] = (int32_t)lo;
  }
}

int bits_for(uint64_t maxval) {  // bits needed to represent values in [0, maxval]
  int b = 0;
  while (b < 64 && (maxval >> b) != 0) ++b;
  return b < 1 ? 1 : b;
}

// ---------------------------------------------------------------------------
// synthetic graphs
// ---------------------------------------------------------------------------
struct SynthDev {
  int kind, L;
  int64_t N, C;
  uint64_t seed;
  int64_t rb, re;
  int scale;
};

// R-MAT quadrant thresholds (a, a+b, a+b+c) * 2^32 for a,b,c,d = .57,.19,.19,.05
constexpr uint64_t kRmatA = 2448131358ull;    // floor(0.57 * 2^32)
constexpr uint64_t kRmatAB = 3264175144ull;   // floor(0.76 * 2^32)
constexpr uint64_t kRmatABC = 4080218931ull;  // floor(0.95 * 2^32)

__device__ __forceinline__ void synth_edge(const SynthDev& s, uint64_t k, int64_t& src, int64_t& dst, int& type) {
  const uint64_t h1 = synth_bits(s.seed, k, 1);
  type = (int)(((h1 & 0xFFFFFFFFull) * (uint64_t)s.L) >> 32);
  if (s.kind == 0) {
    const uint64_t h0 = synth_bits(s.seed, k, 0);
    src = (int64_t)(((h0 & 0xFFFFFFFFull) * (uint64_t)s.N) >> 32);
    dst = (int64_t)(((h0 >> 32) * (uint64_t)s.N) >> 32);
  } else {
    int64_t u = 0, v = 0;
    for (int lvl = 0; lvl < s.scale; ++lvl) {
      const uint64_t h = synth_bits(s.seed, k, 2 + (lvl >> 1));
      const uint64_t r = (lvl & 1) ? (h >> 32) : (h & 0xFFFFFFFFull);
      const int q = r < kRmatA ? 0 : (r < kRmatAB ? 1 : (r < kRmatABC ? 2 : 3));
      u = (u << 1) | (q >> 1);
      v = (v << 1) | (q & 1);
    }
    src = u;
    dst = v;
  }
}

__global__ __launch_bounds__(256) void synth_count_kernel(SynthDev s, unsigned long long* __restrict__ count) {
  __shared__ unsigned int block_cnt;
  if (threadIdx.x == 0) block_cnt = 0;
  __syncthreads();
  unsigned int mine = 0;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < s.C; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t src, dst;
    int t;
    synth_edge(s, (uint64_t)k, src, dst, t);
    mine += (src >= s.rb && src < s.re) ? 1u : 0u;
  }
  atomicAdd(&block_cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(count, (unsigned long long)block_cnt);
}

__global__ __launch_bounds__(256) void synth_emit_kernel(SynthDev s, unsigned long long* __restrict__ cursor,
                                                         uint64_t* __restrict__ keys, int64_t cap) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < s.C; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t src, dst;
    int t;
    synth_edge(s, (uint64_t)k, src, dst, t);
    if (src >= s.rb && src < s.re) {
      const unsigned long long o = atomicAdd(cursor, 1ull);
      if ((int64_t)o < cap) keys[o] = ((uint64_t)(src - s.rb) * (uint64_t)s.L + (uint64_t)t) * (uint64_t)s.N + (uint64_t)dst;
    }
  }
}

__global__ __launch_bounds__(256) void synth_degree_kernel(SynthDev s, int32_t* __restrict__ deg) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < s.C; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t src, dst;
    int t;
    synth_edge(s, (uint64_t)k, src, dst, t);
    if (src >= s.rb && src < s.re) atomicAdd(deg + (src - s.rb), 1);  // integer: order-independent
  }
}

__global__ void synth_split_kernel(const uint64_t* __restrict__ ukeys, const int64_t* __restrict__ nnz_p, int64_t N,
                                   int32_t* __restrict__ colidx) {
  const int64_t nnz = *nnz_p;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * blockDim.x)
    colidx[i] = (int32_t)(ukeys[i] % (uint64_t)N);
}

// rowptr[s] = first unique key >= s*N, s in [0, nseg]
__global__ void synth_rowptr_kernel(const uint64_t* __restrict__ ukeys, const int64_t* __restrict__ nnz_p,
                                    int64_t nseg, int64_t N, int32_t* __restrict__ rowptr) {
  const int64_t nnz = *nnz_p;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= nseg; s += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t target = (uint64_t)s * (uint64_t)N;
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (ukeys[mid] < target)
        lo = mid + 1;
      else
        hi = mid;
    }
    rowptr[s] = (int32_t)lo;
  }
}

int grid_for(int64_t n, int per_block = 256, int64_t cap = 65536) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, per_block), cap));
}

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int synth_validate(const GrlSynthSpec* spec, SynthDev& s) {
  GRL_CHECK_ARG(spec != nullptr, "synth: spec is NULL");
  GRL_CHECK_ARG(spec->kind == 0 || spec->kind == 1, "synth: kind must be 0 (ER) or 1 (R-MAT)");
  GRL_CHECK_ARG(spec->num_types >= 1 && spec->num_types <= 63, "synth: num_types in [1, 63]");
  GRL_CHECK_ARG(spec->num_nodes >= 1 && spec->num_nodes <= 2147483647LL, "synth: num_nodes in [1, 2^31)");
  GRL_CHECK_ARG(spec->num_candidates >= 0, "synth: negative num_candidates");
  GRL_CHECK_ARG(0 <= spec->row_begin && spec->row_begin <= spec->row_end && spec->row_end <= spec->num_nodes,
                "synth: bad row range [%lld, %lld)", (long long)spec->row_begin, (long long)spec->row_end);
  s.kind = spec->kind;
  s.L = spec->num_types;
  s.N = spec->num_nodes;
  s.C = spec->num_candidates;
  s.seed = spec->seed;
  s.rb = spec->row_begin;
  s.re = spec->row_end;
  s.scale = 0;
  if (s.kind == 1) {
    GRL_CHECK_ARG((s.N & (s.N - 1)) == 0, "synth: R-MAT needs num_nodes = 2^scale");
    while ((1LL << s.scale) < s.N) ++s.scale;
  }
  const uint64_t rows = (uint64_t)(s.re - s.rb);
  GRL_CHECK_ARG(rows == 0 || rows * (uint64_t)s.L <= (~0ull) / (uint64_t)s.N, "synth: key overflow");
  GRL_CHECK_ARG(rows * (uint64_t)s.L < 2147483647ull, "synth: too many segments for int32 rowptr");
  return GRL_OK;
}

}  // namespace
}  // namespace grl

using namespace grl;

// ------------------------------- dense -> CSR -------------------------------
extern "C" size_t grl_dense_to_csr_workspace_size(int64_t num_segments) {
  size_t temp = 0;
  int32_t* dummy = nullptr;
  const int64_t n = num_segments + 1;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, temp, dummy, dummy, (int)std::max<int64_t>(n, 1)) != hipSuccess)
    return 0;
  return align_up((size_t)n * sizeof(int32_t)) + align_up(temp);
}

extern "C" int grl_dense_to_csr_rowptr(const float* A, int64_t B, int64_t N, int32_t L, const int64_t strides[4],
                                       int32_t* rowptr, void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  GRL_CHECK_ARG(B >= 0 && N >= 0 && L >= 1 && strides != nullptr, "grl_dense_to_csr_rowptr: bad shape");
  GRL_CHECK_ARG(rowptr != nullptr, "grl_dense_to_csr_rowptr: rowptr is NULL");
  if ((double)B * (double)N * (double)L * (double)N >= 2147483647.0)
    GRL_FAIL(GRL_E_OVERFLOW, "grl_dense_to_csr_rowptr: B*N*L*N >= 2^31 entries cannot be indexed by int32");
  const int64_t rows = B * N * L;
  const size_t need = grl_dense_to_csr_workspace_size(rows);
  if (workspace_bytes < need || (need && !workspace))
    GRL_FAIL(GRL_E_WORKSPACE, "grl_dense_to_csr_rowptr: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  int32_t* counts = reinterpret_cast<int32_t*>(workspace);
  void* temp = static_cast<char*>(workspace) + align_up((size_t)(rows + 1) * sizeof(int32_t));
  size_t temp_bytes = workspace_bytes - align_up((size_t)(rows + 1) * sizeof(int32_t));
  if (rows > 0) {
    GRL_CHECK_ARG(A != nullptr, "grl_dense_to_csr_rowptr: A is NULL");
    hipLaunchKernelGGL(dense_count_kernel, dim3(grid_for(rows, 4)), dim3(256), 0, st, A, B, N, L, strides[0],
                       strides[1], strides[2], strides[3], counts);
    GRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(set_tail_zero, dim3(1), dim3(1), 0, st, counts + rows);
  GRL_LAUNCH_CHECK();
  GRL_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, rowptr, (int)(rows + 1), st));
  return GRL_OK;
}

extern "C" int grl_dense_to_csr_fill(const float* A, int64_t B, int64_t N, int32_t L, const int64_t strides[4],
                                     const int32_t* rowptr, int32_t* colidx, float* vals, grl_stream_t stream) {
  GRL_CHECK_ARG(B >= 0 && N >= 0 && L >= 1 && strides != nullptr, "grl_dense_to_csr_fill: bad shape");
  const int64_t rows = B * N * L;
  if (rows == 0) return GRL_OK;
  GRL_CHECK_ARG(A && rowptr && colidx, "grl_dense_to_csr_fill: NULL pointer");
  hipLaunchKernelGGL(dense_fill_kernel, dim3(grid_for(rows, 4)), dim3(256), 0, as_stream(stream), A, B, N, L,
                     strides[0], strides[1], strides[2], strides[3], rowptr, colidx, vals);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// ------------------------------- CSR -> CSC ---------------------------------
extern "C" size_t grl_csr_to_csc_workspace_size(int64_t nnz, int64_t num_cols) {
  size_t temp = 0;
  int32_t* dummy = nullptr;
  const int n = (int)std::max<int64_t>(nnz, 1);
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, temp, dummy, dummy, dummy, dummy, n, 0,
                                         bits_for((uint64_t)std::max<int64_t>(num_cols - 1, 1))) != hipSuccess)
    return 0;
  return 2 * align_up((size_t)n * sizeof(int32_t)) + align_up(temp);
}

extern "C" int grl_csr_to_csc(const GrlTypedCsr* g, int64_t num_cols, int32_t* colptr, int32_t* zrow, int32_t* eid,
                              float* vals_out, void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  GRL_CHECK_ARG(g != nullptr && num_cols >= 0 && colptr != nullptr, "grl_csr_to_csc: bad arguments");
  GRL_CHECK_ARG(g->num_types >= 1, "grl_csr_to_csc: num_types must be >= 1");
  GRL_CHECK_ARG(g->nnz < 2147483647LL, "grl_csr_to_csc: nnz exceeds int32");
  GRL_CHECK_ARG(g->self_row0 == 0, "grl_csr_to_csc: a row-range view (self_row0 %lld) has no transpose of its own",
                (long long)g->self_row0);
  hipStream_t st = as_stream(stream);
  const int64_t nnz = g->nnz;
  const size_t need = grl_csr_to_csc_workspace_size(nnz, num_cols);
  if (workspace_bytes < need || !workspace)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_csr_to_csc: workspace %zu < %zu", workspace_bytes, need);
  const int nn = (int)std::max<int64_t>(nnz, 1);
  int32_t* vals_iota = reinterpret_cast<int32_t*>(workspace);
  int32_t* keys_out = reinterpret_cast<int32_t*>(static_cast<char*>(workspace) + align_up((size_t)nn * 4));
  void* temp = static_cast<char*>(workspace) + 2 * align_up((size_t)nn * 4);
  size_t temp_bytes = workspace_bytes - 2 * align_up((size_t)nn * 4);
  if (nnz > 0) {
    GRL_CHECK_ARG(g->colidx && zrow && eid, "grl_csr_to_csc: NULL pointer");
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(nnz)), dim3(256), 0, st, vals_iota, nnz);
    GRL_LAUNCH_CHECK();
    GRL_HIP(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, g->colidx, keys_out, vals_iota, eid, (int)nnz, 0,
                                               bits_for((uint64_t)std::max<int64_t>(num_cols - 1, 1)), st));
    const int hs = g->has_self ? 1 : 0;
    hipLaunchKernelGGL(csc_gather_kernel, dim3(grid_for(nnz)), dim3(256), 0, st, g->rowptr,
                       g->num_rows * g->num_types, g->num_types, hs, eid, g->vals, nnz, zrow,
                       g->vals ? vals_out : nullptr);
    GRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(lower_bound_ptr_kernel, dim3(grid_for(num_cols + 1)), dim3(256), 0, st, keys_out, nnz, num_cols,
                     colptr);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// ------------------------------- synthetic ----------------------------------
extern "C" int grl_synth_count(const GrlSynthSpec* spec, int64_t* count, grl_stream_t stream) {
  SynthDev s;
  int rc = synth_validate(spec, s);
  if (rc) return rc;
  GRL_CHECK_ARG(count != nullptr, "grl_synth_count: count is NULL");
  hipStream_t st = as_stream(stream);
  GRL_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), st));
  if (s.C > 0) {
    hipLaunchKernelGGL(synth_count_kernel, dim3(grid_for(s.C, 256, 16384)), dim3(256), 0, st, s,
                       reinterpret_cast<unsigned long long*>(count));
    GRL_LAUNCH_CHECK();
  }
  return GRL_OK;
}

extern "C" int grl_synth_degrees(const GrlSynthSpec* spec, int32_t* deg, grl_stream_t stream) {
  SynthDev s;
  int rc = synth_validate(spec, s);
  if (rc) return rc;
  if (s.C == 0 || s.re == s.rb) return GRL_OK;
  GRL_CHECK_ARG(deg != nullptr, "grl_synth_degrees: deg is NULL");
  hipLaunchKernelGGL(synth_degree_kernel, dim3(grid_for(s.C, 256, 16384)), dim3(256), 0, as_stream(stream), s, deg);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

extern "C" size_t grl_synth_workspace_size(const GrlSynthSpec* spec, int64_t count) {
  SynthDev s;
  if (synth_validate(spec, s)) return 0;
  const int n = (int)std::max<int64_t>(count, 1);
  const int end_bit = bits_for((uint64_t)(s.re - s.rb) * (uint64_t)s.L * (uint64_t)s.N);
  size_t t_sort = 0, t_uniq = 0;
  uint64_t* d = nullptr;
  int64_t* cnt = nullptr;
  if (hipcub::DeviceRadixSort::SortKeys(nullptr, t_sort, d, d, n, 0, end_bit) != hipSuccess) return 0;
  if (hipcub::DeviceSelect::Unique(nullptr, t_uniq, d, d, cnt, n) != hipSuccess) return 0;
  return 3 * align_up((size_t)n * 8) + align_up(16) + align_up(std::max(t_sort, t_uniq));
}

extern "C" int grl_synth_build(const GrlSynthSpec* spec, int64_t count, int32_t* rowptr, int32_t* colidx,
                               int64_t* nnz, void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  SynthDev s;
  int rc = synth_validate(spec, s);
  if (rc) return rc;
  GRL_CHECK_ARG(count >= 0 && count < 2147483647LL, "grl_synth_build: count must be in [0, 2^31)");
  GRL_CHECK_ARG(rowptr && nnz, "grl_synth_build: NULL pointer");
  const size_t need = grl_synth_workspace_size(spec, count);
  if (workspace_bytes < need || !workspace)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_synth_build: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const int n = (int)std::max<int64_t>(count, 1);
  char* w = static_cast<char*>(workspace);
  uint64_t* keys = reinterpret_cast<uint64_t*>(w);
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + align_up((size_t)n * 8));
  uint64_t* ukeys = reinterpret_cast<uint64_t*>(w + 2 * align_up((size_t)n * 8));
  unsigned long long* cursor = reinterpret_cast<unsigned long long*>(w + 3 * align_up((size_t)n * 8));
  void* temp = w + 3 * align_up((size_t)n * 8) + align_up(16);
  size_t temp_bytes = workspace_bytes - (3 * align_up((size_t)n * 8) + align_up(16));
  const int64_t nseg = (s.re - s.rb) * s.L;
  GRL_HIP(hipMemsetAsync(nnz, 0, sizeof(int64_t), st));
  if (count > 0) {
    GRL_CHECK_ARG(colidx != nullptr, "grl_synth_build: colidx is NULL");
    GRL_HIP(hipMemsetAsync(cursor, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(synth_emit_kernel, dim3(grid_for(s.C, 256, 16384)), dim3(256), 0, st, s, cursor, keys, count);
    GRL_LAUNCH_CHECK();
    const int end_bit = bits_for((uint64_t)(s.re - s.rb) * (uint64_t)s.L * (uint64_t)s.N);
    GRL_HIP(hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, sorted, (int)count, 0, end_bit, st));
    GRL_HIP(hipcub::DeviceSelect::Unique(temp, temp_bytes, sorted, ukeys, nnz, (int)count, st));
    hipLaunchKernelGGL(synth_split_kernel, dim3(grid_for(count)), dim3(256), 0, st, ukeys, nnz, s.N, colidx);
    GRL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(synth_rowptr_kernel, dim3(grid_for(nseg + 1)), dim3(256), 0, st, ukeys, nnz, nseg, s.N, rowptr);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
