// fp32 GEMMs of the GraphConv linear on the gfx950 matrix cores.
//
// Forward:  V_out = new_V @ h_weights + bias   (gnn/models/networks/robust_gcn.py:50)
//           [+ F.relu]                          (drop_robust_gcn.py:76,80,85)
// Backward (autograd MmBackward0 of robust_gcn.py:50, ReLU mask fused):
//           dZ = (g * [out > 0]) @ h_weights^T
//           dW = new_V^T @ (g * [out > 0]),  db = sum_rows(g * [out > 0])
//
// One templated kernel, v_mfma_f32_32x32x2_f32 (exact f32 products, one
// rounding per fmaf): block tile 128 x 128, K staged 32 deep through LDS in
// the operand's natural global layout (every global load and LDS store is a
// float4; no transposing stores).  An operand whose K index is contiguous is
// read as one ds_read_b128 fragment per k-step of 8 (the two half-waves take
// k = 4h + s); one whose M/N index is contiguous as four ds_read_b32 (lanes on
// consecutive addresses, conflict-free).  The next K tile is loaded into
// registers while the current one is multiplied.  4 waves, each a 64 x 64
// sub-tile = 2 x 2 MFMA tiles = 64 accumulator registers.  Long reductions
// (dW sums over all N nodes) split K over blockIdx.z into fp32 slabs that a
// second pass adds in split order: deterministic, no atomics.
#include "grl_internal.h"


#include <cstdlib>

// GRL_X6T_WHATIF (diagnostic builds with -DGRL_DIAG only; timing, wrong
// results): the dW GEMM without its split VALU (1), without its operand
// stream after two steps (2), without its per-step barrier (4)
#if !defined(GRL_DIAG) || !defined(GRL_X6T_WHATIF)
#undef GRL_X6T_WHATIF
#define GRL_X6T_WHATIF 0
#endif
// register sets of the dW GEMM's staged rows: 1, the loads one K16 step ahead
// of their LDS stash; 2 (diagnostic builds: -DGRL_DIAG -DGRL_X6T_NR=2), two
// steps -- measured neutral (profiles/r06_ab_dw_nr2.txt): the operand stream
// costs the kernel power, not latency
#if !defined(GRL_DIAG) || !defined(GRL_X6T_NR)
#undef GRL_X6T_NR
#define GRL_X6T_NR 1
#endif

namespace grl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BM = 128, BN = 128;



enum Epilogue { EPI_STORE = 0, EPI_BIAS = 1, EPI_SLAB = 2 };

struct GemmArgs {
  const float* A;
  int64_t lda;
  const float* Amask;  // optional: A element multiplied by [Amask > 0] (same indexing as A)
  const float* B;
  int64_t ldb;
  const float* Bmask;  // optional, same indexing as B
  float* C;
  int64_t ldc;
  const float* bias;
  int64_t M, N, K;
  int64_t k_per_split;
  int relu;
  // tile grid (set by launch_gemm): mt x nt output tiles x zt K-splits,
  // launched as one dimension; inner_n: which tile index runs fastest
  int64_t mt, nt, zt;
  int inner_n;
  // rows the x6-vs-fp32 path choice is made for (0: M): a node-range shard
  // passes the whole graph's row count, so it takes the one-GPU call's path
  int64_t path_rows;
};


// XCD-aware tile order.  Workgroups are dealt to the 8 XCDs round-robin
// (blockIdx % 8; speed only, never relied on for correctness), and each XCD
// walks a contiguous run of the tile order u with the operand-sharing index
// fastest, so the tiles that read the same A rows (inner_n: forward, dZ) or
// the same B rows (dW) run together on one XCD and hit its L2 instead of
// re-reading HBM once per tile (dZ: 14 N tiles share each 1 GB row block).
__device__ __forceinline__ void tile_of(const GemmArgs& p, int64_t& mi, int64_t& ni, int64_t& zi) {
  const int64_t T = p.mt * p.nt * p.zt;
  const int64_t L = blockIdx.x;
  const int64_t q = T / 8, r = T % 8, x = L % 8, s = L / 8;
  const int64_t u = x * q + (x < r ? x : r) + s;
  if (p.inner_n) {
    ni = u % p.nt;
    mi = (u / p.nt) % p.mt;
  } else {
    mi = u % p.mt;
    ni = (u / p.mt) % p.nt;
  }
  zi = u / (p.mt * p.nt);
}

__device__ __forceinline__ float4 masked(float4 v, float4 mk) {
  v.x = mk.x > 0.f ? v.x : 0.f;
  v.y = mk.y > 0.f ? v.y : 0.f;
  v.z = mk.z > 0.f ? v.z : 0.f;
  v.w = mk.w > 0.f ? v.w : 0.f;
  return v;
}

// One operand tile (ROWS x BK) staged as ROWS*BK/4 float4 slots, SLOTS per
// thread.  KC: image [row][k] (k contiguous, stride LDK); RC: image [k][row]
// (row contiguous, stride LDR).  Global addresses are per-thread pointers
// advanced by one K tile per step; interior tiles load with no per-element
// branches (clamped + selected loads only on edge tiles).
template <bool KC, bool ALIGNED, bool MASK, int BK, int ROWS = BM>
struct Operand {
  static constexpr int LDK = BK + 4;
  static constexpr int LDR = ROWS + 4;
  static constexpr int RQ = ROWS / 4;  // float4 slots per k row of the [k][row] image
  static constexpr int SLOTS = ROWS * BK / 4 / 256;
  const float* base;
  const float* mask;
  int64_t ld, rows_total, row0;
  int64_t kstep;  // element stride per unit of k
  float4 reg[SLOTS];

  __device__ __forceinline__ void slot(int idx, int64_t& row, int& kin) const {
    if (KC) {
      row = row0 + idx / (BK / 4);
      kin = (idx % (BK / 4)) * 4;
    } else {
      row = row0 + (idx % RQ) * 4;
      kin = idx / RQ;
    }
  }
  __device__ __forceinline__ int lds_off(int idx) const {
    return KC ? (idx / (BK / 4)) * LDK + (idx % (BK / 4)) * 4 : (idx / RQ) * LDR + (idx % RQ) * 4;
  }
  __device__ __forceinline__ void fetch(int tid, int64_t k0, int64_t kend, bool interior) {
#pragma unroll
    for (int it = 0; it < SLOTS; ++it) {
      int64_t row;
      int kin;
      slot(tid + it * 256, row, kin);
      const int64_t k = k0 + kin;
      if (interior) {
        const int64_t off = KC ? row * ld + k : k * ld + row;
        float4 v = *reinterpret_cast<const float4*>(base + off);
        if (MASK) v = masked(v, *reinterpret_cast<const float4*>(mask + off));
        reg[it] = v;
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t r = KC ? row : row + e;
          const int64_t kk = KC ? k + e : k;
          const bool ok = r < rows_total && kk < kend;
          const int64_t off = ok ? (KC ? r * ld + kk : kk * ld + r) : 0;
          float x = base[off];
          if (MASK) x = mask[off] > 0.f ? x : 0.f;
          t[e] = ok ? x : 0.f;
        }
        reg[it] = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
  }
  __device__ __forceinline__ void stash(float* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < SLOTS; ++it) *reinterpret_cast<float4*>(&lds[lds_off(tid + it * 256)]) = reg[it];
  }
  // fragment of row `row` (0..ROWS-1 within the tile) for k = kk + 4h + s, s = 0..3
  __device__ __forceinline__ static float4 frag(const float* lds, int row, int kk, int h) {
    if (KC) return *reinterpret_cast<const float4*>(&lds[row * LDK + kk + 4 * h]);
    const float* c = &lds[(kk + 4 * h) * LDR + row];
    return make_float4(c[0], c[LDR], c[2 * LDR], c[3 * LDR]);
  }
  static constexpr int lds_floats() { return KC ? ROWS * LDK : BK * LDR; }
};

// A(m, k): A_KC ? A[m*lda + k] : A[k*lda + m]
// B(k, n): B_KC ? B[n*ldb + k] : B[k*ldb + n]
// TBN: the tile's columns, 128 (four 64 x 64 wave tiles) or 64 (four 64 x 32:
// narrow outputs -- the classifier's 56, f/g/h's 160 -- compute half the
// padding).  Every element's accumulation is the same either way (one
// accumulator, k in the same order): the choice never changes bits.
template <bool A_KC, bool B_KC, int EPI, bool ALIGNED, bool MASK_A, bool MASK_B, int BK, int TBN = BN>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs p) {
  using OA = Operand<A_KC, ALIGNED, MASK_A, BK>;
  using OB = Operand<B_KC, ALIGNED, MASK_B, BK, TBN>;
  constexpr int NJ = TBN / 64;  // 32-column accumulators per wave
  constexpr int WN = 32 * NJ;   // wave tile columns
  constexpr int STAGE = OA::lds_floats() + OB::lds_floats();
  constexpr int SMEM = STAGE > 4 * 64 * 32 ? STAGE : 4 * 64 * 32;  // epilogue staging: 64 x 32 per wave
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  static_assert(TBN == 64 || TBN == 128, "tile columns: 64 or 128");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int l32 = lane & 31, h = lane >> 5;
  int64_t mi, ni, zi;
  tile_of(p, mi, ni, zi);
  const int64_t m0 = mi * BM;
  const int64_t n0 = ni * TBN;
  const int64_t kbeg = zi * p.k_per_split;
  const int64_t kend = min(p.K, kbeg + p.k_per_split);

  OA oa;
  oa.base = p.A;
  oa.mask = p.Amask;
  oa.ld = p.lda;
  oa.rows_total = p.M;
  oa.row0 = m0;
  OB ob;
  ob.base = p.B;
  ob.mask = p.Bmask;
  ob.ld = p.ldb;
  ob.rows_total = p.N;
  ob.row0 = n0;
  const bool rows_in = ALIGNED && (m0 + BM <= p.M) && (n0 + TBN <= p.N);

  f32x16 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  auto mma_step = [&](const float* As, const float* Bs) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
      float4 a[2], b[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = OA::frag(As, wm * 64 + i * 32 + l32, kk, h);
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = OB::frag(Bs, wn * WN + j * 32 + l32, kk, h);
      // component-major: consecutive MFMAs hit the four independent
      // accumulators, so none waits on the previous one's result (the
      // per-accumulator k order is unchanged: results are bitwise the same)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(reinterpret_cast<const float*>(&a[i])[c],
                                                             reinterpret_cast<const float*>(&b[j])[c], acc[i][j],
                                                             0, 0, 0);
    }
  };

  if (kbeg < kend) {
    const bool in0 = rows_in && kbeg + BK <= kend;
    oa.fetch(tid, kbeg, kend, in0);
    ob.fetch(tid, kbeg, kend, in0);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    oa.stash(smem, tid);
    ob.stash(smem + OA::lds_floats(), tid);
    __syncthreads();
    const int64_t kn = k0 + BK;
    if (kn < kend) {  // next tile in flight during the MFMAs
      const bool in = rows_in && kn + BK <= kend;
      oa.fetch(tid, kn, kend, in);
      ob.fetch(tid, kn, kend, in);
    }
    mma_step(smem, smem + OA::lds_floats());
    __syncthreads();
  }

  // ---- epilogue: C/D map col = lane&31, row = (r&3) + 8(r>>2) + 4h --------
  float* Cz = p.C + (EPI == EPI_SLAB ? zi * p.M * p.ldc : 0);
  // Through LDS, one 64 x 32 half of the wave's sub-tile at a time, so that
  // every lane stores whole float4 rows (a register holds one column of four
  // rows; scalar stores cost 4x the store instructions on a 7 GB output).
  if ((p.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(Cz) & 15) == 0) {
    float* stage = smem + wave * (64 * 32);  // 4 x 2048 floats
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) stage[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 32 + l32] = acc[i][j][r];
      __syncthreads();
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = (lane >> 3) + 8 * it, c4 = (lane & 7) * 4;
        const int64_t gm = m0 + wm * 64 + row;
        const int64_t gn = n0 + wn * WN + j * 32 + c4;
        if (gm >= p.M || gn >= p.N) continue;
        float4 v = *reinterpret_cast<const float4*>(&stage[row * 32 + c4]);
        float* vp = reinterpret_cast<float*>(&v);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = vp[e];
          if (EPI == EPI_BIAS) {
            if (p.bias && gn + e < p.N) x += p.bias[gn + e];
            if (p.relu) x = x > 0.0f ? x : 0.0f;
          }
          vp[e] = x;
        }
        if (gn + 3 < p.N) {
          *reinterpret_cast<float4*>(&Cz[gm * p.ldc + gn]) = v;
        } else {
          for (int e = 0; gn + e < p.N; ++e) Cz[gm * p.ldc + gn + e] = vp[e];
        }
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int64_t gn = n0 + wn * WN + j * 32 + l32;
    if (gn >= p.N) continue;
    const float bv = (EPI == EPI_BIAS && p.bias) ? p.bias[gn] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < p.M) {
          float v = acc[i][j][r] + bv;
          if (EPI == EPI_BIAS && p.relu) v = v > 0.0f ? v : 0.0f;
          Cz[gm * p.ldc + gn] = v;
        }
      }
    }
  }
}

// sum_{z < splits} slab[z*stride + i] in split order; loads are issued 8
// slabs ahead of the adds (a chain of dependent loads is latency-bound).
__device__ __forceinline__ float ordered_slab_sum(const float* __restrict__ slab, int64_t stride, int splits,
                                                  int64_t i) {
  float s = 0.0f;
  int z = 0;
  for (; z + 8 <= splits; z += 8) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = slab[(int64_t)(z + u) * stride + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; z < splits; ++z) s += slab[(int64_t)z * stride + i];
  return s;
}

// out[i] = sum_{z < splits} slab[z][i]  (split order: deterministic)
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int64_t n, int splits, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = ordered_slab_sum(slab, n, splits, i);
}

// Split-K epilogue of the forward / data-gradient GEMMs:
// out[m*ldo + n] = epi(sum_{z < splits} slab[z][m][n] (+ bias[n])), split order.
__global__ void slab_reduce_epi_kernel(const float* __restrict__ slab, int64_t M, int64_t N, int splits,
                                       float* __restrict__ out, int64_t ldo, const float* __restrict__ bias,
                                       int relu) {
  const int64_t n_all = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x) {
    float s = ordered_slab_sum(slab, n_all, splits, i);
    const int64_t m = i / N, n = i - m * N;
    if (bias) s += bias[n];
    if (relu) s = s > 0.0f ? s : 0.0f;
    out[m * ldo + n] = s;
  }
}

// partial[z][c] = sum over rows [z*rows_per, ...) of g[r][c] * [mask[r][c] > 0],
// added in row order; loads are issued 8 rows ahead of the adds (latency).
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ g, const float* __restrict__ mask,
                                                              int64_t M, int64_t C, int64_t rows_per,
                                                              float* __restrict__ partial) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t z = blockIdx.y;
  if (c >= C) return;
  const int64_t r0 = z * rows_per, r1 = min(M, r0 + rows_per);
  float s = 0.0f;
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = g[(r + u) * C + c];
      if (mask) x[u] = mask[(r + u) * C + c] > 0.0f ? x[u] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; r < r1; ++r) {
    const float x = g[r * C + c];
    s += (!mask || mask[r * C + c] > 0.0f) ? x : 0.0f;
  }
  partial[z * C + c] = s;
}

// g_eff[r][c] = relu_out[r][c] > 0 ? g[r][c] : 0, and partial[z][c] = the sum
// of g_eff over rows [z*rows_per, ...) in colsum_partial_kernel's order (so a
// db reduced from it is bitwise that kernel's on g_eff).  g_eff may alias g.
__global__ __launch_bounds__(256) void relu_grad_colsum_kernel(const float* g, const float* __restrict__ relu_out,
                                                                float* g_eff, int64_t M, int64_t C, int64_t rows_per,
                                                                float* __restrict__ partial) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t z = blockIdx.y;
  if (c >= C) return;
  const int64_t r0 = z * rows_per, r1 = min(M, r0 + rows_per);
  float s = 0.0f;
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float v = g[(r + u) * C + c];
      x[u] = relu_out[(r + u) * C + c] > 0.0f ? v : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) g_eff[(r + u) * C + c] = x[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; r < r1; ++r) {
    const float x = relu_out[r * C + c] > 0.0f ? g[r * C + c] : 0.0f;
    g_eff[r * C + c] = x;
    s += x;
  }
  if (partial) partial[z * C + c] = s;
}

// ---------------------------------------------------------------------------
// Large-tile path for the big GraphConv shapes (M in the millions): 256 x 256
// block tile, 8 waves (2 along M x 4 along N, each 128 x 64 = 4 x 2 MFMA
// 32x32 tiles, 128 accumulator registers), one block per CU.  K is staged 16
// deep through THREE LDS stages (96 KB) filled by global_load_lds_dwordx4
// (LDS-DMA: no VGPR staging, no ds_write pass); tile t+1's DMA stays in
// flight across the barrier (counted `s_waitcnt vmcnt(4)`, raw s_barrier --
// cdna_hip_programming.md "Pipelining across barriers").  Measured at C3:
// forward 7.97 -> 7.56 ms, dZ 8.0 -> 7.55 ms; dW (both operands M/N
// contiguous) stays on the 128^2 kernel (7.8 ms vs 10.6 here).
// Preconditions (big_ok): 16-B aligned operands and leading dimensions,
// K % 16 == 0, M, N >= 4, no operand masks.
constexpr int LB_M = 256, LB_N = 256;
constexpr int LP_K = 16, LP_STAGE = LB_M * LP_K;  // floats per operand stage

template <bool KC>
struct PipeOperand {
  const float* base;
  int64_t ld, rows_total, row0;
  //  KC: row = 16 floats = 4 chunks; 16 rows per 1 KB instruction; chunk c of
  //      row r at c ^ (r & 3).   RC: one k row (256 floats) per instruction.
  __device__ __forceinline__ void issue(float* lds, int wave, int lane, int64_t k0) const {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int inst = wave * 2 + q;  // 16 per operand stage
      const float* src;
      if (KC) {
        const int r = inst * 16 + (lane >> 2);
        const int c = (lane & 3) ^ (r & 3);
        int64_t row = row0 + r;
        row = row < rows_total ? row : rows_total - 1;
        src = base + row * ld + k0 + c * 4;
      } else {
        int64_t col = row0 + lane * 4;
        col = col + 3 < rows_total ? col : rows_total - 4;
        src = base + (k0 + inst) * ld + col;
      }
      // Issued from asm so that the compiler's waitcnt pass does not see an
      // LDS write in flight and wait vmcnt(0) before every ds_read (which
      // would serialize the pipeline); ordering is the counted vmcnt +
      // s_barrier in the kernel.  M0 = the wave-uniform LDS byte address.
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          (uint32_t)reinterpret_cast<uintptr_t>(lds + inst * 256));
      uint32_t keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\t"
          "s_mov_b32 m0, %2\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\t"
          "s_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(dst)
          : "memory");
    }
  }
  __device__ __forceinline__ static float4 frag(const float* lds, int row, int kk, int h) {
    if (KC) {
      const int c = (kk >> 2) + h;
      return *reinterpret_cast<const float4*>(&lds[row * LP_K + ((c ^ (row & 3)) << 2)]);
    }
    const float* q = &lds[(kk + 4 * h) * LB_N + row];
    return make_float4(q[0], q[LB_N], q[2 * LB_N], q[3 * LB_N]);
  }
};

template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
}

template <bool A_KC, bool B_KC, int EPI, int S>
__global__ __launch_bounds__(512) void gemm256p_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[S * 2 * LP_STAGE];  // S stages x (A, B), 32 KB each
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int l32 = lane & 31, h = lane >> 5;
  int64_t mi, ni, zi;
  tile_of(p, mi, ni, zi);
  const int64_t m0 = mi * LB_M, n0 = ni * LB_N;
  const int64_t kbeg = zi * p.k_per_split;
  const int64_t kend = min(p.K, kbeg + p.k_per_split);
  const int64_t nk = kend > kbeg ? (kend - kbeg) / LP_K : 0;
  const PipeOperand<A_KC> oa{p.A, p.lda, p.M, m0};
  const PipeOperand<B_KC> ob{p.B, p.ldb, p.N, n0};

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  auto stage_ptr = [&](int64_t t) { return smem + (int)(t % S) * 2 * LP_STAGE; };
  for (int64_t t = 0; t < S - 1 && t < nk; ++t) {
    oa.issue(stage_ptr(t), wave, lane, kbeg + t * LP_K);
    ob.issue(stage_ptr(t) + LP_STAGE, wave, lane, kbeg + t * LP_K);
  }
  for (int64_t t = 0; t < nk; ++t) {
    // tile t landed (the next min(S-2, nk-1-t) tiles' DMA, 4 instructions
    // per wave each, may stay in flight); every wave's reads of the stage
    // about to be refilled (tile t-1) are retired
    const int64_t ahead = nk - 1 - t;
    if (S >= 4 && ahead >= 2)
      wait_vm_lgkm0<8>();
    else if (ahead >= 1)
      wait_vm_lgkm0<4>();
    else
      wait_vm_lgkm0<0>();
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < nk) {
      float* nx = stage_ptr(t + S - 1);
      oa.issue(nx, wave, lane, kbeg + (t + S - 1) * LP_K);
      ob.issue(nx + LP_STAGE, wave, lane, kbeg + (t + S - 1) * LP_K);
    }
    const float* cur = stage_ptr(t);
#pragma unroll
    for (int kk = 0; kk < LP_K; kk += 8) {
      float4 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = PipeOperand<A_KC>::frag(cur, wm * 128 + i * 32 + l32, kk, h);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = PipeOperand<B_KC>::frag(cur + LP_STAGE, wn * 64 + j * 32 + l32, kk, h);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(reinterpret_cast<const float*>(&a[i])[c],
                                                             reinterpret_cast<const float*>(&b[j])[c], acc[i][j],
                                                             0, 0, 0);
    }
  }

  float* Cz = p.C + (EPI == EPI_SLAB ? zi * p.M * p.ldc : 0);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t gn = n0 + wn * 64 + j * 32 + l32;
    if (gn >= p.N) continue;
    const float bv = (EPI == EPI_BIAS && p.bias) ? p.bias[gn] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < p.M) {
          float v = acc[i][j][r] + bv;
          if (EPI == EPI_BIAS && p.relu) v = v > 0.0f ? v : 0.0f;
          Cz[gm * p.ldc + gn] = v;
        }
      }
  }
}


// ---------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores by exact three-way splitting ("x6").
// Every fp32 operand value v is written as v = v0 + v1 + v2 with
// v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1) (round to nearest
// even; the differences are exact by Sterbenz, and 3 x 8 significant bits
// hold all 24 of an fp32, so the split is exact for 2^-100 <= |v| < 3.39e38;
// below, the third part is a bf16 subnormal, off by <= 2^-133: tests/test_x6_split.py).
// Products of two bf16 are exact in fp32; of the nine a_i b_j the six with
// i + j <= 2 are accumulated (v_mfma_f32_32x32x16_bf16, fp32 accumulators);
// the three dropped terms are <= ~2^-24 |a b| each -- the size of one fp32
// rounding.  One 32x32x16 bf16 MFMA costs 32 SIMD cycles against 8 x 64 for
// the same K on v_mfma_f32_32x32x2_f32, so six of them take 0.375x the
// matrix-core time of the fp32 instruction (MI355X_MICROARCH.md: f32 MFMA =
// 1/16 of bf16).
//
// A (M x K, K contiguous: Z for the forward, g for dZ) is split inside the
// kernel while it is staged into LDS; B arrives pre-split (split_planes_kernel,
// once per call: W is 1.8 MB) as three bf16 planes [3][Np][K] with K
// contiguous.  256 x 256 block tile, 8 waves of 128 x 64 (4 x 2 MFMA tiles,
// 128 accumulators), K staged 16 deep through two LDS plane stages (48 KB
// each: 3 planes x (A, B) x 256 rows x 32 B), one barrier per stage.  A and
// B arrive by LDS-DMA (layout and pipeline at gemm_x6_kernel below).
// Preconditions (x6_shape_ok + aligned): K % 16 == 0, 16-B aligned A,
// lda % 4 == 0, no operand masks.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

constexpr int X6_K = 16;
constexpr int X6_PLANE = 256 * X6_K;  // bf16 elements per plane per operand stage
constexpr int X6_STAGE = 6 * X6_PLANE;  // A planes then B planes

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  f32x2_t p = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(p, bf16x2_t));
}
__device__ __forceinline__ float lo_f(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_f(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// v -> three planes of 4 bf16 (v == p0 + p1 + p2 exactly)
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

// planes[p][n][k] (n < Np, k < K; zero for n >= N) of B(k, n) = B_KC ? B[n*ldb + k] : B[k*ldb + n]
__global__ void split_planes_kernel(const float* __restrict__ B, int64_t ldb, int b_kc, int64_t N, int64_t K,
                                    int64_t Np, uint16_t* __restrict__ planes) {
  const int64_t total = Np * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / K, k = i - n * K;
    const float v = n < N ? (b_kc ? B[n * ldb + k] : B[k * ldb + n]) : 0.0f;
    const uint32_t h0 = pack_bf16(v, 0.0f) & 0xFFFFu;
    const float r1 = v - lo_f(h0);
    const uint32_t h1 = pack_bf16(r1, 0.0f) & 0xFFFFu;
    const float r2 = r1 - lo_f(h1);
    const uint32_t h2 = pack_bf16(r2, 0.0f) & 0xFFFFu;
    planes[i] = (uint16_t)h0;
    planes[total + i] = (uint16_t)h1;
    planes[2 * total + i] = (uint16_t)h2;
  }
}

// global -> LDS DMA of one 16 B chunk per lane (lane l lands at lds_base + 16 l).
// Issued from asm so that hipcc's waitcnt pass neither sees nor waits on it;
// completion is ordered by the kernel's counted `s_waitcnt vmcnt`.
__device__ __forceinline__ void dma16(const void* src, const void* lds_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds_base));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(dst)
      : "memory");
}

// LDS: two plane stages (48 KB each: A planes 0-2, B planes 3-5, 256 rows x
// 16 k bf16) + three A landing slots (16 KB each: [wave][2 instr][lane] x 16 B
// of fp32, each lane reading back only what it fetched itself).
// Step t:  barrier | DMA B(t+1) -> stage (t+1)&1, DMA A(t+2) -> slot (t+2)%3 |
//          MFMAs on stage t&1 | vmcnt(2): own A(t+1), B(t+1) landed |
//          split own A(t+1) from its slot into stage (t+1)&1.
// A's loads get two compute phases to land, B's (L2-resident planes) one.
constexpr int X6_SLOT = 512 * 8;  // floats per landing slot (16 KB)

template <int EPI>
__global__ __launch_bounds__(512) void gemm_x6_kernel(GemmArgs p, const uint16_t* __restrict__ Bp, int64_t Np) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * X6_STAGE];  // 2 plane stages x 48 KB
  __shared__ __attribute__((aligned(16))) float land[3 * X6_SLOT];      // 3 landing slots x 16 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int l32 = lane & 31, h = lane >> 5;
  int64_t mi, ni, zi;
  tile_of(p, mi, ni, zi);
  const int64_t m0 = mi * LB_M, n0 = ni * LB_N;
  const int64_t K = p.K;
  const int64_t nk = K / X6_K;

  // A: this lane's two float4 (idx = tid + 512 i: row idx >> 2, 4 k at (idx & 3) * 4)
  const int64_t r0 = min<int64_t>(m0 + (tid >> 2), p.M - 1);
  const int64_t r1 = min<int64_t>(m0 + ((tid + 512) >> 2), p.M - 1);
  const float* a_src0 = p.A + r0 * p.lda + (tid & 3) * 4;
  const float* a_src1 = p.A + r1 * p.lda + (tid & 3) * 4;
  // 16-B half h of a 32-B plane row r sits at position h ^ ((r >> 3) & 1): the
  // ds_read_b128 lane groups {0-3,12-15,20-27}, ... then hit 16 distinct
  // slots (2-way bank conflicts without it; MI355X_MICROARCH.md §LDS)
  auto sw = [](int r, int k) { return r * X6_K + ((((k >> 3) ^ (r >> 3)) & 1) << 3) + (k & 7); };
  const int a_off0 = sw(tid >> 2, (tid & 3) * 4);
  const int a_off1 = sw((tid + 512) >> 2, (tid & 3) * 4);
  // B: chunk c = (3 wave + j) * 64 + lane of 1536 per stage: plane c / 512,
  // n = (c % 512) / 2, 8 k at (c & 1) * 8; lands at B region + 8 c
  const int64_t plane_stride = Np * K;
  const uint16_t* b_src[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int c = (wave * 3 + j) * 64 + lane;
    const int n = (c & 511) >> 1;
    b_src[j] = Bp + (c >> 9) * plane_stride + (n0 + n) * K + (((c & 1) ^ (n >> 3)) & 1) * 8;
  }
  float* const my_land = land + wave * 512;  // 2 x 1 KB per wave; + slot * X6_SLOT, + 256 per instr, + 4 lane

  auto issue_a = [&](int64_t t) {
    float* sl = my_land + (int)(t % 3) * X6_SLOT;
    dma16(a_src0 + t * X6_K, sl);
    dma16(a_src1 + t * X6_K, sl + 256);
  };
  auto issue_b = [&](int64_t t, uint16_t* st) {
    uint16_t* bb = st + 3 * X6_PLANE + wave * 3 * 512;
#pragma unroll
    for (int j = 0; j < 3; ++j) dma16(b_src[j] + t * X6_K, bb + j * 512);
  };
  auto stash_a = [&](int64_t t, uint16_t* st) {
    const float* sl = my_land + (int)(t % 3) * X6_SLOT + lane * 4;
    const float4 v0 = *reinterpret_cast<const float4*>(sl);
    const float4 v1 = *reinterpret_cast<const float4*>(sl + 256);
    uint2 q0, q1, q2;
    split3(v0, q0, q1, q2);
    *reinterpret_cast<uint2*>(st + a_off0) = q0;
    *reinterpret_cast<uint2*>(st + X6_PLANE + a_off0) = q1;
    *reinterpret_cast<uint2*>(st + 2 * X6_PLANE + a_off0) = q2;
    split3(v1, q0, q1, q2);
    *reinterpret_cast<uint2*>(st + a_off1) = q0;
    *reinterpret_cast<uint2*>(st + X6_PLANE + a_off1) = q1;
    *reinterpret_cast<uint2*>(st + 2 * X6_PLANE + a_off1) = q2;
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  if (nk > 0) {
    issue_a(0);
    issue_b(0, smem);
    if (nk > 1) {
      issue_a(1);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stash_a(0, smem);
  }
  for (int64_t t = 0; t < nk; ++t) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    uint16_t* cur = smem + (int)(t & 1) * X6_STAGE;
    uint16_t* nxt = smem + (int)((t + 1) & 1) * X6_STAGE;
    if (t + 1 < nk) issue_b(t + 1, nxt);
    if (t + 2 < nk) issue_a(t + 2);
    {
      bf16x8_t a_[4][3], b_[2][3];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          a_[i][q] = *reinterpret_cast<const bf16x8_t*>(cur + q * X6_PLANE + sw(wm * 128 + i * 32 + l32, h * 8));
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          b_[j][q] = *reinterpret_cast<const bf16x8_t*>(cur + (3 + q) * X6_PLANE + sw(wn * 64 + j * 32 + l32, h * 8));
      // small terms first (i + j = 2, then 1, then the leading product)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][2], b_[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][1], b_[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][1], b_[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][0], acc[i][j], 0, 0, 0);
        }
    }
    if (t + 1 < nk) {
      if (t + 2 < nk)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A(t+2) may stay in flight
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stash_a(t + 1, nxt);
    }
  }
  float* Cz = p.C;
  if (m0 + LB_M <= p.M) {  // whole row tile (uniform): row offsets are uniform multiples of ldc
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t gn = n0 + wn * 64 + j * 32 + l32;
      const float bv = (EPI == EPI_BIAS && p.bias && gn < p.N) ? p.bias[gn] : 0.0f;
      float* const o = Cz + (m0 + wm * 128 + 4 * h) * p.ldc + gn;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r] + bv;
          if (EPI == EPI_BIAS && p.relu) v = v > 0.0f ? v : 0.0f;
          if (gn < p.N) o[(int64_t)(i * 32 + (r & 3) + 8 * (r >> 2)) * p.ldc] = v;
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t gn = n0 + wn * 64 + j * 32 + l32;
    if (gn >= p.N) continue;
    const float bv = (EPI == EPI_BIAS && p.bias) ? p.bias[gn] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < p.M) {
          float v = acc[i][j][r] + bv;
          if (EPI == EPI_BIAS && p.relu) v = v > 0.0f ? v : 0.0f;
          Cz[gm * p.ldc + gn] = v;
        }
      }
  }
}

// ---------------------------------------------------------------------------
// x6 for the weight gradient dW = Z^T g (grl_linear_bwd_weight at large M):
// both operands are M/N-contiguous (A(m, k) = Z[k][m], B(k, n) = g[k][n], k =
// node).  Each K16 step's rows are split into bf16 planes stored as they lie,
// [16 k][256 m] (512 B per k row; the 8-B group at column m of row k sits at
// m ^ ((k & 3) << 5), so stores and reads are bank-conflict free), and the
// MFMA fragments (8 consecutive k of one column) come out of
// ds_read_b64_tr_b16, the gfx950 transposing LDS read: per 16-lane group a
// 4 k x 16 column block, lane i receiving column i (cdna_hip_programming.md
// T10).  K (the node count) is split over blockIdx.z into fp32 slabs added in
// split order afterwards (deterministic).  Register-staged: the next step's
// loads are in flight during the MFMAs.  Preconditions (x6t_ok): 16-B
// aligned operands, lda, ldb, M, N multiples of 4.
typedef short i16x4_t __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) uint16_t lds_u16;

// tr_pair on an LDS-space pointer (p0 = plane + k * 256 + swizzled column):
// the second block row is a constant 2 KB further, so with the stage and the
// plane also constants both reads fold into one base VGPR + ds offsets
__device__ __forceinline__ bf16x8_t tr_pair3(const lds_u16* p0) {
  typedef __attribute__((address_space(3))) i16x4_t lds_v4;
  const i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p0);
  const i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0 + 4 * 256));
  typedef short i16x8_t __attribute__((ext_vector_type(8)));
  const i16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// The K16 loop is unrolled over the two stages, fragment reads from per-lane
// LDS offsets fixed for the kernel (the stage and plane as immediates): the
// rolled loop recomputed ~40 address adds per step (round 4,
// profiles/r04_ab_dw_u2.txt).
template <int EPI>
__global__ __launch_bounds__(512) void gemm_x6t_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * X6_STAGE];  // 2 stages x (A, B) x 3 planes x 8 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int l32 = lane & 31, h = lane >> 5;
  int64_t mi, ni, zi;
  tile_of(p, mi, ni, zi);
  const int64_t m0 = mi * LB_M, n0 = ni * LB_N;
  const int64_t kbeg = zi * p.k_per_split;
  const int64_t kend = min(p.K, kbeg + p.k_per_split);
  const int64_t nk = kend > kbeg ? (kend - kbeg + X6_K - 1) / X6_K : 0;

  // staging: float4 f = tid + 512 i of each operand: k row f >> 6, 4 columns at (f & 63) * 4
  // the staged k rows are wave-uniform: row offsets and the range checks stay scalar
  const int kr0 = __builtin_amdgcn_readfirstlane(tid >> 6), kr1 = kr0 + 8;
  const int col = (tid & 63) * 4;
  const int64_t am = min<int64_t>(m0 + col, p.M - 4), bn = min<int64_t>(n0 + col, p.N - 4);
  const float* __restrict__ a_base = p.A + am;
  const float* __restrict__ b_base = p.B + bn;
  const int st_off0 = kr0 * 256 + (col ^ ((kr0 & 3) << 5));
  const int st_off1 = kr1 * 256 + (col ^ ((kr1 & 3) << 5));
  // register sets of staged rows: set j holds step t's rows for t = j (mod NR); NR = 2 puts the loads
  // two K16 steps ahead of their LDS stash (one step of MFMAs would leave an HBM miss's latency exposed)
  constexpr int NR = GRL_X6T_NR;
  float4 ra0[NR], ra1[NR], rb0[NR], rb1[NR];
  bool in0[NR], in1[NR];  // the staged rows lie inside this split's K range
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // Rows past the split's end are loaded clamped (from kbeg) and zeroed only
  // when stashed, after the next step's MFMAs: zeroing right after the loads
  // made hipcc branch on the loaded registers and wait vmcnt(0) for them
  // there, exposing the whole load latency on every K16 step
  // (cdna_hip_programming.md, "register or load" selects).
#define X6T_LOAD(t, j)                                                                                    \
  do {                                                                                                    \
    const int64_t k_ = kbeg + (t) * X6_K;                                                                 \
    in0[j] = k_ + kr0 < kend;                                                                             \
    in1[j] = k_ + kr1 < kend;                                                                             \
    const int64_t r0_ = in0[j] ? k_ + kr0 : kbeg;                                                         \
    const int64_t r1_ = in1[j] ? k_ + kr1 : kbeg;                                                         \
    ra0[j] = *reinterpret_cast<const float4*>(a_base + r0_ * p.lda);                                      \
    ra1[j] = *reinterpret_cast<const float4*>(a_base + r1_ * p.lda);                                      \
    rb0[j] = *reinterpret_cast<const float4*>(b_base + r0_ * p.ldb);                                      \
    rb1[j] = *reinterpret_cast<const float4*>(b_base + r1_ * p.ldb);                                      \
  } while (0)
#if GRL_X6T_WHATIF & 1  /* what-if (timing only): no split VALU, the raw bits as planes */
#define X6T_SPLIT3(v, q0_, q1_, q2_)                                                                      \
  do {                                                                                                    \
    q0_ = make_uint2(__float_as_uint((v).x), __float_as_uint((v).y));                                     \
    q1_ = make_uint2(__float_as_uint((v).z), __float_as_uint((v).w));                                     \
    q2_ = q0_;                                                                                            \
  } while (0)
#else
#define X6T_SPLIT3(v, q0_, q1_, q2_) split3(v, q0_, q1_, q2_)
#endif
#define X6T_SPLIT(v, base, off)                                                                           \
  do {                                                                                                    \
    uint2 q0_, q1_, q2_;                                                                                  \
    X6T_SPLIT3(v, q0_, q1_, q2_);                                                                         \
    *reinterpret_cast<uint2*>((base) + (off)) = q0_;                                                      \
    *reinterpret_cast<uint2*>((base) + X6_PLANE + (off)) = q1_;                                           \
    *reinterpret_cast<uint2*>((base) + 2 * X6_PLANE + (off)) = q2_;                                       \
  } while (0)
#define X6T_STASH(st, j)                                                                                  \
  do {                                                                                                    \
    if (!in0[j]) ra0[j] = rb0[j] = zero4; /* wave-uniform: only a split's last K16 step branches */       \
    if (!in1[j]) ra1[j] = rb1[j] = zero4;                                                                 \
    X6T_SPLIT(ra0[j], (st), st_off0);                                                                     \
    X6T_SPLIT(ra1[j], (st), st_off1);                                                                     \
    X6T_SPLIT(rb0[j], (st) + 3 * X6_PLANE, st_off0);                                                      \
    X6T_SPLIT(rb1[j], (st) + 3 * X6_PLANE, st_off1);                                                      \
  } while (0)

  // this lane's transposed-read coordinates: k = 8h + ((lane & 15) >> 2),
  // column = block base + 16 ((lane >> 4) & 1) + 4 (lane & 3)
  const int tk = 8 * h + ((lane & 15) >> 2);
  const int tc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  if (nk > 0) {
    X6T_LOAD(0, 0);
    X6T_STASH(smem, 0);
#pragma unroll
    for (int j = 1; j <= NR; ++j)
      if (nk > j) X6T_LOAD(j, j % NR);
  }
  __syncthreads();
  {
    const lds_u16* s3 = (const lds_u16*)smem;
    const int sx = (tk & 3) << 5;
    int oa[4], ob[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) oa[i] = tk * 256 + ((wm * 128 + i * 32 + tc) ^ sx);
#pragma unroll
    for (int j = 0; j < 2; ++j) ob[j] = tk * 256 + ((wn * 64 + j * 32 + tc) ^ sx);
    // step t reads LDS stage S = t & 1 and stashes register set J = (t + 1) % NR into the other stage:
    // both constants of the body (the loop is unrolled by two, and NR is 1 or 2)
    auto step = [&](int64_t t, auto stage, auto rset) {
      constexpr int S = decltype(stage)::value;
      constexpr int J = decltype(rset)::value;  // (t + 1) % NR
      const lds_u16* cur = s3 + S * X6_STAGE;
      bf16x8_t a_[4][3], b_[2][3];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) a_[i][q] = tr_pair3(cur + q * X6_PLANE + oa[i]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) b_[j][q] = tr_pair3(cur + (3 + q) * X6_PLANE + ob[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][2], b_[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][1], b_[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][1], b_[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_[i][0], b_[j][0], acc[i][j], 0, 0, 0);
        }
      if (t + 1 < nk) {
        X6T_STASH(smem + (S ^ 1) * X6_STAGE, J);  // the other stage: last read in step t-1
#if GRL_X6T_WHATIF & 2
        if (t + 1 + NR < nk && t < 2) X6T_LOAD(t + 1 + NR, J);  // what-if: no Z / g stream after the first steps
#else
        if (t + 1 + NR < nk) X6T_LOAD(t + 1 + NR, J);
#endif
      }
#if GRL_X6T_WHATIF & 4
      __builtin_amdgcn_s_waitcnt(0);  // what-if: no barrier (races; timing only)
#else
      __syncthreads();
#endif
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    int64_t t = 0;
    if constexpr (NR == 1) {
      for (; t + 1 < nk; t += 2) {
        step(t, I0{}, I0{});
        step(t + 1, I1{}, I0{});
      }
      if (t < nk) step(t, I0{}, I0{});
    } else {  // NR == 2: the register set to stash is (t + 1) & 1 = the other LDS stage's parity
      for (; t + 1 < nk; t += 2) {
        step(t, I0{}, I1{});
        step(t + 1, I1{}, I0{});
      }
      if (t < nk) step(t, I0{}, I1{});
    }
  }
#undef X6T_LOAD
#undef X6T_SPLIT
#undef X6T_STASH
  float* Cz = p.C + (EPI == EPI_SLAB ? zi * p.M * p.ldc : 0);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t gn = n0 + wn * 64 + j * 32 + l32;
    if (gn >= p.N) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t gm = m0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < p.M) Cz[gm * p.ldc + gn] = acc[i][j][r];
      }
  }
}

bool al16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

constexpr int GEMM_BK = 32;

template <bool A_KC, bool B_KC, int EPI, int TBN = BN>
int launch_gemm(GemmArgs a, int splits, bool aligned, hipStream_t st) {
  if (a.M == 0 || a.N == 0) return GRL_OK;
  a.mt = ceil_div(a.M, BM);
  a.nt = ceil_div(a.N, TBN);
  a.zt = splits;
  // the operand worth sharing is the one with more rows per tile: A (M x K
  // rows of Z / g) for the forward and dZ, B (the K x N slab of g) for dW
  a.inner_n = (A_KC ? 1 : 0);
  GRL_CHECK_ARG(a.mt * a.nt * a.zt < 2147483647LL, "gemm: grid too large");
  const dim3 grid((unsigned)(a.mt * a.nt * a.zt));
  const bool ma = a.Amask != nullptr, mb = a.Bmask != nullptr;
#define GRL_GEMM(AL, MA, MB) \
  hipLaunchKernelGGL((gemm_kernel<A_KC, B_KC, EPI, AL, MA, MB, GEMM_BK, TBN>), grid, dim3(256), 0, st, a)
  if (aligned) {
    if (ma) GRL_GEMM(true, true, false); else if (mb) GRL_GEMM(true, false, true); else GRL_GEMM(true, false, false);
  } else {
    if (ma) GRL_GEMM(false, true, false); else if (mb) GRL_GEMM(false, false, true); else GRL_GEMM(false, false, false);
  }
#undef GRL_GEMM
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

int pick_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ceil_div(M, BM) * ceil_div(N, BN);
  const int64_t want = (int64_t)device_cu_count() * 4;  // ~4 blocks per CU
  int64_t s = std::max<int64_t>(1, want / std::max<int64_t>(tiles, 1));
  // each split keeps >= 4 K tiles (1 or 2 measured the same on the C1 step, profiles/r05_ab_c1_dw_splits.txt)
  s = std::min<int64_t>(s, ceil_div(K, 4 * GEMM_BK));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 256));
}

// The output-stationary fp32 GEMM (forward, data gradient; the x6 path's
// fallback) sums K in fixed chunks of whole K tiles -- their size chosen
// from K and the WHOLE call's output tiles (path_rows), never from the rows
// at hand: about kFp32WantBlocks workgroups, at most kFp32MaxChunks chunks --
// one chunk per K split into fp32 slabs that a second pass adds in chunk
// order with the bias / ReLU epilogue.  So every element is the same fp32
// operations whatever M is, and a node-range shard's rows equal the whole
// graph's.  Small calls get the chunks' parallelism (a lone
// workgroup walking all of K is bound by load latency: a 74-node page is one
// 128-row tile; its 1792-deep GraphConv GEMM runs as 56 one-tile chunks);
// M whose slabs would exceed kFp32SlabCap runs in row blocks that fit.  (Summing the chunks inside one
// workgroup instead -- a second accumulator set -- cost 1 wave per SIMD at
// 225-251 VGPRs: the classifier's 100k rows ran 5x slower than hipBLASLt.)
// Calls made for at least kFp32OnePassTiles output tiles -- counted on the
// whole graph's rows (path_rows), so every shard and row block of that graph
// decides alike -- fill the chip without the chunks and walk all of K in one
// accumulator instead: the slabs of K = 512 at 100k rows were 16 chunks of
// one K tile each, 1.6 GB of slab traffic for a 13 GFLOP GEMM.
constexpr int64_t kFp32MaxChunks = 64;
constexpr int64_t kFp32WantBlocks = 1024;  // ~4 workgroups per CU
constexpr size_t kFp32SlabCap = (size_t)256 << 20;
constexpr int64_t kFp32OnePassTiles = 256;

int64_t path_rows_of(int64_t M, int64_t path_rows) { return std::max<int64_t>(M, path_rows); }

// output tiles of the whole call (path_rows) the arithmetic is chosen for
int64_t fp32_path_tiles(int64_t M, int64_t path_rows, int64_t N) {
  return ceil_div(path_rows_of(M, path_rows), BM) * ceil_div(std::max<int64_t>(N, 1), BN);
}

int64_t fp32_chunk_tiles(int64_t tiles, int64_t K) {
  const int64_t kt = std::max<int64_t>(1, ceil_div(K, GEMM_BK));
  const int64_t want = std::max<int64_t>(1, ceil_div(kFp32WantBlocks, std::max<int64_t>(tiles, 1)));
  return ceil_div(kt, std::min<int64_t>(std::min<int64_t>(want, kFp32MaxChunks), kt));
}

int fp32_chunks(int64_t tiles, int64_t K) {
  return (int)ceil_div(std::max<int64_t>(1, ceil_div(K, GEMM_BK)), fp32_chunk_tiles(tiles, K));
}

// rows per slab pass: all of M, or the BM-multiple whose `chunks` slabs fit kFp32SlabCap
int64_t fp32_block_rows(int64_t M, int64_t N, int chunks) {
  const int64_t per_row = (int64_t)chunks * std::max<int64_t>(N, 1) * 4;
  const int64_t cap = std::max<int64_t>(BM, (int64_t)kFp32SlabCap / per_row / BM * BM);
  return std::min<int64_t>(M, cap);
}

// K splits of the fp32 output GEMM: 1 (one pass, no slabs) for calls of
// kFp32OnePassTiles tiles, else the chunk count
int pick_splits_small(int64_t M, int64_t path_rows, int64_t N, int64_t K) {
  const int64_t tiles = fp32_path_tiles(M, path_rows, N);
  return tiles >= kFp32OnePassTiles ? 1 : fp32_chunks(tiles, K);
}

// row blocks of the db column sum: ~16 rows each (>= 1 block, <= 1024); a block's rows are a chain of
// dependent load rounds, so small M wants short blocks (a 296-row C1 batch: 19 blocks, 2 rounds each)
int colsum_splits(int64_t M) { return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(M, 16), 1024)); }

size_t small_ws_bytes(int64_t M, int64_t path_rows, int64_t N, int64_t K) {
  const int s = pick_splits_small(M, path_rows, N, K);
  return s > 1 ? (size_t)s * (size_t)fp32_block_rows(M, N, s) * (size_t)N * 4 + 256 : 0;
}

// Large-tile path selection (the fp32 fallback when the x6 path is off).
bool big_ok(const GemmArgs& a, bool aligned) {
  return aligned && !a.Amask && !a.Bmask && a.K % LP_K == 0 && a.M >= 4 && a.N >= 4 &&
         2.0 * (double)a.M * (double)a.N * (double)a.K >= 1.6e10;
}

template <bool A_KC, bool B_KC, int EPI>
int launch_gemm256p(GemmArgs a, int splits, hipStream_t st) {
  a.mt = ceil_div(a.M, LB_M);
  a.nt = ceil_div(a.N, LB_N);
  a.zt = splits;
  a.inner_n = A_KC ? 1 : 0;
  GRL_CHECK_ARG(a.mt * a.nt * a.zt < 2147483647LL, "gemm: grid too large");
  hipLaunchKernelGGL((gemm256p_kernel<A_KC, B_KC, EPI, 3>), dim3((unsigned)(a.mt * a.nt * a.zt)), dim3(512), 0, st,
                     a);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// Split-bf16 ("x6") path selection.  The gemm_x6 path option 0 keeps the
// fp32-MFMA kernels (A/B aid and tests; a workspace query and the call it
// sizes must see the same setting).
bool x6_enabled() { return opt(OPT_GEMM_X6) != 0; }

bool x6_shape_ok(int64_t M, int64_t N, int64_t K) {
  return x6_enabled() && K % X6_K == 0 && K > 0 && M >= 4 && N >= 4 &&
         2.0 * (double)M * (double)N * (double)K >= 1.6e10;
}

int64_t x6_np(int64_t N) { return ceil_div(N, LB_N) * LB_N; }

// workspace of the x6 path: B's three bf16 planes
size_t x6_ws_bytes(int64_t M, int64_t N, int64_t K) {
  return x6_shape_ok(M, N, K) ? (size_t)3 * (size_t)x6_np(N) * (size_t)K * 2 + 256 : 0;
}

// The path choice for an M-row call made on behalf of `path_rows` rows (a
// node-range shard's rows of a graph of path_rows nodes; 0: M itself): the
// size floor is the whole call's, so every shard takes the one-GPU path.
// (The x6 kernels clamp their A rows, so any M >= 1 is safe on them.)
bool x6_path_ok(int64_t M, int64_t path_rows, int64_t N, int64_t K) {
  return M >= 1 && x6_shape_ok(path_rows_of(M, path_rows), N, K);
}
size_t x6_ws_bytes_p(int64_t M, int64_t path_rows, int64_t N, int64_t K) {
  return M >= 1 ? x6_ws_bytes(path_rows_of(M, path_rows), N, K) : 0;
}

template <bool B_KC>
int split_b_planes(const GemmArgs& a, uint16_t* planes, hipStream_t st) {
  const int64_t Np = x6_np(a.N);
  const int64_t n_el = Np * a.K;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n_el, 256), 4096)), dim3(256), 0,
                     st, a.B, a.ldb, B_KC ? 1 : 0, a.N, a.K, Np, planes);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// the x6 GEMM on B planes already split into `planes`
int launch_x6_gemm(GemmArgs a, const uint16_t* planes, hipStream_t st) {
  const int64_t Np = x6_np(a.N);
  a.mt = ceil_div(a.M, LB_M);
  a.nt = Np / LB_N;
  a.zt = 1;
  a.inner_n = 1;
  a.k_per_split = a.K;
  GRL_CHECK_ARG(a.mt * a.nt < 2147483647LL, "gemm: grid too large");
  const dim3 grid((unsigned)(a.mt * a.nt));
  if (a.bias || a.relu)
    hipLaunchKernelGGL(gemm_x6_kernel<EPI_BIAS>, grid, dim3(512), 0, st, a, planes, Np);
  else
    hipLaunchKernelGGL(gemm_x6_kernel<EPI_STORE>, grid, dim3(512), 0, st, a, planes, Np);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

template <bool B_KC>
int launch_x6(GemmArgs a, void* ws, hipStream_t st) {
  uint16_t* planes = static_cast<uint16_t*>(ws);
  const int rc = split_b_planes<B_KC>(a, planes, st);
  return rc ? rc : launch_x6_gemm(a, planes, st);
}

// The output GEMM on 64-column tiles when that computes less padding (N mod
// 128 in 1..64: the classifier's 56 columns, f/g/h's 160); same bits.
template <bool A_KC, bool B_KC, int EPI>
int launch_out_gemm(const GemmArgs& a, int splits, bool aligned, hipStream_t st) {
  const int64_t rem = a.N % BN;
  return rem != 0 && rem <= 64 ? launch_gemm<A_KC, B_KC, EPI, 64>(a, splits, aligned, st)
                               : launch_gemm<A_KC, B_KC, EPI, BN>(a, splits, aligned, st);
}

// Output-stationary GEMM with optional split-K through `ws` (slab layout
// [split][M][N], then one ordered reduce applying bias / ReLU).
template <bool A_KC, bool B_KC>
int run_output_gemm(GemmArgs a, bool aligned, const char* who, void* ws, size_t ws_bytes, hipStream_t st) {
  if (A_KC && aligned && !a.Amask && !a.Bmask && x6_path_ok(a.M, a.path_rows, a.N, a.K) && ws && al16(ws) &&
      ws_bytes >= x6_ws_bytes_p(a.M, a.path_rows, a.N, a.K))  // large M: fp32 on the bf16 matrix cores
    return launch_x6<B_KC>(a, ws, st);
  if (a.path_rows == 0 && big_ok(a, aligned)) {  // forward and dZ at large M: the pipelined 256^2 LDS-DMA tile
    a.k_per_split = std::max<int64_t>(a.K, 1);
    return a.bias || a.relu ? launch_gemm256p<A_KC, B_KC, EPI_BIAS>(a, 1, st)
                            : launch_gemm256p<A_KC, B_KC, EPI_STORE>(a, 1, st);
  }
  const int splits = pick_splits_small(a.M, a.path_rows, a.N, a.K);
  if (splits == 1) {
    a.k_per_split = std::max<int64_t>(a.K, 1);
    return a.bias || a.relu ? launch_out_gemm<A_KC, B_KC, EPI_BIAS>(a, 1, aligned, st)
                            : launch_out_gemm<A_KC, B_KC, EPI_STORE>(a, 1, aligned, st);
  }
  const size_t need = small_ws_bytes(a.M, a.path_rows, a.N, a.K);
  if (!ws || ws_bytes < need) GRL_FAIL(GRL_E_WORKSPACE, "%s: workspace %zu < %zu", who, ws_bytes, need);
  float* const out = a.C;
  const int64_t ldo = a.ldc;
  const float* const bias = a.bias;
  const int relu = a.relu;
  const float* const A0 = a.A;
  const float* const Amask0 = a.Amask;
  const int64_t M = a.M;
  const int64_t R = fp32_block_rows(M, a.N, splits);
  a.C = static_cast<float*>(ws);
  a.ldc = a.N;
  a.bias = nullptr;
  a.relu = 0;
  a.k_per_split = fp32_chunk_tiles(fp32_path_tiles(M, a.path_rows, a.N), a.K) * GEMM_BK;  // one chunk per split
  const int used = (int)ceil_div(a.K, a.k_per_split);
  for (int64_t r0 = 0; r0 < M; r0 += R) {  // row blocks: the same chunks, so the same bits, as one pass
    const int64_t rows = std::min<int64_t>(R, M - r0);
    // A(m, k) = A_KC ? A[m * lda + k] : A[k * lda + m]: row m of the block is m + r0
    a.A = A0 + (A_KC ? r0 * a.lda : r0);
    a.Amask = Amask0 ? Amask0 + (A_KC ? r0 * a.lda : r0) : nullptr;
    a.M = rows;
    int rc = launch_out_gemm<A_KC, B_KC, EPI_SLAB>(a, used, aligned, st);
    if (rc) return rc;
    const int64_t n = rows * a.N;
    hipLaunchKernelGGL(slab_reduce_epi_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, 256), 4096)), dim3(256),
                       0, st, a.C, rows, a.N, used, out + r0 * ldo, ldo, bias, relu);
    GRL_LAUNCH_CHECK();
  }
  return GRL_OK;
}

}  // namespace
}  // namespace grl

using namespace grl;

// x6-sized calls need W's planes; the others the fp32 path's slabs (at most kFp32SlabCap)
extern "C" size_t grl_linear_fwd_ex_workspace_size(int64_t M, int32_t K, int32_t C, int64_t path_rows) {
  if (M <= 0 || K <= 0 || C <= 0) return 0;
  return x6_path_ok(M, path_rows, C, K) ? x6_ws_bytes_p(M, path_rows, C, K) : small_ws_bytes(M, path_rows, C, K);
}

extern "C" size_t grl_linear_fwd_workspace_size(int64_t M, int32_t K, int32_t C) {
  return grl_linear_fwd_ex_workspace_size(M, K, C, 0);
}

extern "C" int grl_linear_fwd_ex(const float* Z, int64_t ldz, const float* W, int32_t w_layout, const float* bias,
                                 float* out, int64_t M, int32_t K, int32_t C, int32_t relu, int64_t path_rows,
                                 void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  TraceRange trace_("grl_linear_fwd");
  GRL_CHECK_ARG(M >= 0 && K >= 0 && C >= 0 && path_rows >= 0, "grl_linear_fwd: negative size");
  GRL_CHECK_ARG(ldz >= K, "grl_linear_fwd: ldz (%lld) < K (%d)", (long long)ldz, K);
  GRL_CHECK_ARG(w_layout == 0 || w_layout == 1, "grl_linear_fwd: w_layout must be 0 ([K][C]) or 1 ([C][K])");
  if (M == 0 || C == 0) return GRL_OK;
  GRL_CHECK_ARG(Z && W && out, "grl_linear_fwd: NULL pointer");
  GemmArgs a{};
  a.A = Z;
  a.lda = ldz;
  a.B = W;
  a.ldb = w_layout ? K : C;
  a.C = out;
  a.ldc = C;
  a.bias = bias;
  a.M = M;
  a.N = C;
  a.K = K;
  a.relu = relu;
  a.path_rows = path_rows;
  const bool aligned = al16(Z) && al16(W) && ldz % 4 == 0 && C % 4 == 0 && K % 4 == 0;
  hipStream_t st = as_stream(stream);
  return w_layout ? run_output_gemm<true, true>(a, aligned, "grl_linear_fwd", workspace, workspace_bytes, st)
                  : run_output_gemm<true, false>(a, aligned, "grl_linear_fwd", workspace, workspace_bytes, st);
}

extern "C" int grl_linear_fwd(const float* Z, int64_t ldz, const float* W, const float* bias, float* out, int64_t M,
                              int32_t K, int32_t C, int32_t relu, void* workspace, size_t workspace_bytes,
                              grl_stream_t stream) {
  return grl_linear_fwd_ex(Z, ldz, W, 0, bias, out, M, K, C, relu, 0, workspace, workspace_bytes, stream);
}

static size_t ws_align(size_t b) { return (b + 255) & ~(size_t)255; }

// the two-kernel form's workspace for a graph whose GEMM path is chosen for path_rows rows
static size_t graphconv_two_kernel_ws(const GrlTypedCsr* g, int F, int C) {
  const int64_t K = (int64_t)(g->num_types + (g->has_self ? 1 : 0)) * F;
  return ws_align((size_t)g->num_rows * (size_t)K * 4) +
         grl_linear_fwd_ex_workspace_size(g->num_rows, (int32_t)K, C, g->path_rows);
}

// grl_graphconv_fwd takes the fused kernel when its arithmetic equals the
// two-kernel path's (the linear on the x6 GEMM: large graphs, 16-B aligned W,
// C % 4 == 0), the shapes fit it (F in {64, 128, 256, 512, 1024}, C <= 512), X rows are
// float4-aligned and no heavy row is split (the split path sums chunk
// partials, a different order).
static bool fused_path(const GrlTypedCsr* g, const float* X, int64_t ldx, int F, const float* W, int C) {
  const int64_t K = (int64_t)(g->num_types + (g->has_self ? 1 : 0)) * F;
  return graphconv_fused_enabled() && graphconv_fused_shape_ok(F, C, g->num_types) &&
         x6_path_ok(g->num_rows, g->path_rows, C, K) &&
         al16(W) && C % 4 == 0 && al16(X) && ldx % 4 == 0 && ldx < (1LL << 30) &&  // gather: 32-bit row bytes
         (!g->split || g->split->num_heavy == 0);
}

extern "C" size_t grl_graphconv_fwd_workspace_query(const GrlTypedCsr* g, const float* X, int64_t ldx, int32_t F,
                                                   const float* W, int32_t C) {
  if (!g || g->num_rows <= 0 || g->num_types < 1 || F <= 0 || C <= 0) return 0;
  const int64_t K = (int64_t)(g->num_types + (g->has_self ? 1 : 0)) * F;
  if (K > 2147483647LL) return 0;
  if (fused_path(g, X, ldx, F, W, C)) return graphconv_fused_ws_bytes(K, C);
  return graphconv_two_kernel_ws(g, F, C);
}

extern "C" size_t grl_graphconv_fwd_workspace_size(int64_t num_rows, int32_t num_types, int32_t has_self, int32_t F,
                                                   int32_t C) {
  if (num_rows <= 0 || num_types < 1 || F <= 0 || C <= 0) return 0;
  const int64_t K = (int64_t)(num_types + (has_self ? 1 : 0)) * F;
  if (K > 2147483647LL) return 0;
  return ws_align((size_t)num_rows * (size_t)K * 4) + grl_linear_fwd_workspace_size(num_rows, (int32_t)K, C);
}


extern "C" int grl_graphconv_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx, int32_t F, const float* W,
                                 const float* bias, int32_t C, int32_t relu, float* out, const GrlDropEdge* de,
                                 void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  TraceRange trace_("grl_graphconv_fwd");
  GRL_CHECK_ARG(g != nullptr, "grl_graphconv_fwd: graph is NULL");
  GRL_CHECK_ARG(g->num_rows >= 0 && g->num_types >= 1 && g->num_types <= 63,
                "grl_graphconv_fwd: num_types must be in [1, 63] (got %d)", g->num_types);
  GRL_CHECK_ARG(F > 0 && ldx >= F && C > 0, "grl_graphconv_fwd: need F > 0, ldx >= F, C > 0");
  const int64_t M = g->num_rows;
  if (M == 0) return GRL_OK;
  GRL_CHECK_ARG(X && W && out && g->rowptr && (g->nnz == 0 || g->colidx), "grl_graphconv_fwd: NULL pointer");
  const int hs = g->has_self ? 1 : 0;
  const int64_t K64 = (int64_t)(g->num_types + hs) * F;
  GRL_CHECK_ARG(K64 <= 2147483647LL, "grl_graphconv_fwd: (has_self + num_types) * F exceeds int32");
  const int32_t K = (int32_t)K64;
  hipStream_t st = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  GRL_CHECK_ARG(ws == nullptr || al16(ws), "grl_graphconv_fwd: workspace must be 16-B aligned");
  const size_t zfull = ws_align((size_t)M * (size_t)K * 4);
  if (fused_path(g, X, ldx, F, W, C) && ws && workspace_bytes >= graphconv_fused_ws_bytes(K, C)) {
    // one kernel: Z never leaves the CU (graphconv.hip)
    GRL_CHECK_ARG(g->nnz < 2147483647LL, "grl_graphconv_fwd: nnz %lld exceeds int32", (long long)g->nnz);
    return graphconv_fused_fwd(g, X, ldx, F, W, bias, C, relu, out, de, ws, st);
  }
  if (ws && workspace_bytes >= graphconv_two_kernel_ws(g, F, C)) {
    // whole graph: Z in the workspace, then the linear (its workspace behind Z)
    float* Z = reinterpret_cast<float*>(ws);
    int rc = grl_typed_spmm_fwd(g, X, ldx, F, Z, de, stream);
    if (rc) return rc;
    return grl_linear_fwd_ex(Z, K, W, 0, bias, out, M, K, C, relu, g->path_rows, ws + zfull, workspace_bytes - zfull,
                             stream);
  }
  // Row chunks: Z for R rows at a time (bounded memory), on the x6 GEMM only,
  // whose per-element arithmetic does not depend on M -- so the result is
  // bitwise that of the whole-graph call.
  const bool x6 = x6_path_ok(M, g->path_rows, C, K) && al16(W) && C % 4 == 0;
  if (!x6 || (g->split && g->split->num_heavy > 0) || !ws)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_graphconv_fwd: workspace %zu < %zu (row chunking needs the x6 GEMM shape and no "
             "heavy-row split plan)", workspace_bytes, grl_graphconv_fwd_workspace_size(M, g->num_types, hs, F, C));
  const size_t planes_bytes = ws_align(x6_ws_bytes_p(M, g->path_rows, C, K));
  const int64_t per_row = (int64_t)K * 4;
  int64_t R = workspace_bytes > planes_bytes ? (int64_t)((workspace_bytes - planes_bytes) / per_row) : 0;
  R = R / LB_M * LB_M;
  if (R < LB_M)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_graphconv_fwd: workspace %zu holds fewer than %d rows of Z", workspace_bytes, LB_M);
  uint16_t* planes = reinterpret_cast<uint16_t*>(ws);
  float* Z = reinterpret_cast<float*>(ws + planes_bytes);
  GemmArgs a{};
  a.B = W;
  a.ldb = C;
  a.N = C;
  a.K = K;
  a.bias = bias;
  a.relu = relu;
  a.lda = K;
  a.ldc = C;
  int rc = split_b_planes<false>(a, planes, st);
  if (rc) return rc;
  for (int64_t r0 = 0; r0 < M; r0 += R) {
    const int64_t rows = std::min<int64_t>(R, M - r0);
    rc = spmm_fwd_rows(g, r0, rows, X, ldx, F, Z, de, st);
    if (rc) return rc;
    a.A = Z;
    a.M = rows;
    a.C = out + r0 * C;
    rc = launch_x6_gemm(a, planes, st);
    if (rc) return rc;
  }
  return GRL_OK;
}

// The data gradient of one GraphConv layer by reassociation (see grl.h):
// dX = sum_s (A_drop,s^T G) W_s^T on the one-kernel GraphConv over the typed
// transpose.  Eligible when the forward's x6 GEMM shape would be (large
// graphs), C in {64, 128, 256, 512, 1024}, F <= 512, L <= 7, G rows float4-aligned and no
// heavy-row split plan on the transpose.
static bool bwd_data_path(const GrlTypedCsr* gt, const float* G, int64_t ldg, int C, const float* W, int F) {
  const int64_t K = (int64_t)(gt->num_types + (gt->has_self ? 1 : 0)) * C;
  return gt->self_row0 == 0 && graphconv_fused_enabled() && graphconv_fused_shape_ok(C, F, gt->num_types) && x6_shape_ok(gt->num_rows, F, K) &&
         al16(W) && F % 4 == 0 && al16(G) && ldg % 4 == 0 && ldg < (1LL << 30) &&
         (!gt->split || gt->split->num_heavy == 0) &&
         K <= 2147483647LL && gt->nnz < 2147483647LL;
}

extern "C" size_t grl_graphconv_bwd_data_workspace_query(const GrlTypedCsr* gt, const float* G, int64_t ldg, int32_t C,
                                                        const float* W, int32_t F) {
  if (!gt || gt->num_rows <= 0 || gt->num_types < 1 || C <= 0 || F <= 0) return 0;
  if (!bwd_data_path(gt, G, ldg, C, W, F)) return 0;
  return graphconv_fused_ws_bytes((int64_t)(gt->num_types + (gt->has_self ? 1 : 0)) * C, F);
}

extern "C" int grl_graphconv_bwd_data(const GrlTypedCsr* gt, const int32_t* eid, const float* G, int64_t ldg,
                                      int64_t g_rows, int32_t C, const float* W, int32_t F, float* dX, float* G_agg,
                                      const GrlDropEdge* de, void* workspace, size_t workspace_bytes,
                                      grl_stream_t stream) {
  TraceRange trace_("grl_graphconv_bwd_data");
  GRL_CHECK_ARG(gt != nullptr, "grl_graphconv_bwd_data: graph is NULL");
  GRL_CHECK_ARG(gt->num_rows >= 0 && gt->num_types >= 1 && gt->num_types <= 63,
                "grl_graphconv_bwd_data: num_types must be in [1, 63] (got %d)", gt->num_types);
  GRL_CHECK_ARG(C > 0 && ldg >= C && F > 0 && g_rows >= 0 && g_rows <= gt->num_rows,
                "grl_graphconv_bwd_data: need C > 0, ldg >= C, F > 0, 0 <= g_rows <= num_rows");
  if (gt->num_rows == 0) return GRL_OK;
  // (an empty node-range shard: no G rows and no entries, so its empty G is never read)
  GRL_CHECK_ARG((G || (g_rows == 0 && gt->nnz == 0)) && W && dX && gt->rowptr && (gt->nnz == 0 || (gt->colidx && eid)),
                "grl_graphconv_bwd_data: NULL pointer");
  if (!bwd_data_path(gt, G, ldg, C, W, F))
    GRL_FAIL(GRL_E_UNSUPPORTED, "grl_graphconv_bwd_data: shape outside the one-kernel path (C %d, F %d, L %d, rows "
             "%lld; see grl_graphconv_bwd_data_workspace_query)", C, F, gt->num_types, (long long)gt->num_rows);
  const size_t need = graphconv_fused_ws_bytes((int64_t)(gt->num_types + (gt->has_self ? 1 : 0)) * C, F);
  if (!workspace || !al16(workspace) || workspace_bytes < need)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_graphconv_bwd_data: workspace %zu < %zu (16-B aligned)", workspace_bytes, need);
  return graphconv_fused_bwd_data(gt, eid, G, ldg, g_rows, C, W, F, dX, G_agg, de, workspace, as_stream(stream));
}

extern "C" int grl_graphconv_fwd_train(const GrlTypedCsr* g, const float* X, int64_t ldx, int32_t F, const float* W,
                                       const float* bias, int32_t C, int32_t relu, float* out, float* Z,
                                       const GrlDropEdge* de, void* workspace, size_t workspace_bytes,
                                       grl_stream_t stream) {
  TraceRange trace_("grl_graphconv_fwd_train");
  GRL_CHECK_ARG(g != nullptr, "grl_graphconv_fwd_train: graph is NULL");
  GRL_CHECK_ARG(g->num_rows >= 0 && g->num_types >= 1 && g->num_types <= 63,
                "grl_graphconv_fwd_train: num_types must be in [1, 63] (got %d)", g->num_types);
  GRL_CHECK_ARG(F > 0 && ldx >= F && C > 0, "grl_graphconv_fwd_train: need F > 0, ldx >= F, C > 0");
  const int64_t M = g->num_rows;
  if (M == 0) return GRL_OK;
  GRL_CHECK_ARG(X && W && out && Z && g->rowptr && (g->nnz == 0 || g->colidx), "grl_graphconv_fwd_train: NULL pointer");
  const int hs = g->has_self ? 1 : 0;
  const int64_t K64 = (int64_t)(g->num_types + hs) * F;
  GRL_CHECK_ARG(K64 <= 2147483647LL, "grl_graphconv_fwd_train: (has_self + num_types) * F exceeds int32");
  const int32_t K = (int32_t)K64;
  char* ws = static_cast<char*>(workspace);
  GRL_CHECK_ARG(ws == nullptr || al16(ws), "grl_graphconv_fwd_train: workspace must be 16-B aligned");
  if (fused_path(g, X, ldx, F, W, C) && al16(Z) && ws && workspace_bytes >= graphconv_fused_ws_bytes(K, C)) {
    GRL_CHECK_ARG(g->nnz < 2147483647LL, "grl_graphconv_fwd_train: nnz %lld exceeds int32", (long long)g->nnz);
    return graphconv_fused_fwd(g, X, ldx, F, W, bias, C, relu, out, de, ws, as_stream(stream), Z);
  }
  const int rc = grl_typed_spmm_fwd(g, X, ldx, F, Z, de, stream);
  return rc ? rc : grl_linear_fwd_ex(Z, K, W, 0, bias, out, M, K, C, relu, g->path_rows, workspace, workspace_bytes,
                                     stream);
}

extern "C" size_t grl_linear_bwd_data_workspace_size(int64_t M, int32_t K, int32_t C) {
  if (M <= 0 || K <= 0 || C <= 0) return 0;
  return x6_shape_ok(M, K, C) ? x6_ws_bytes(M, K, C) : small_ws_bytes(M, 0, K, C);
}

extern "C" int grl_linear_bwd_data(const float* g, const float* relu_out, const float* W, float* dZ, int64_t lddz,
                                   int64_t M, int32_t K, int32_t C, void* workspace, size_t workspace_bytes,
                                   grl_stream_t stream) {
  TraceRange trace_("grl_linear_bwd_data");
  GRL_CHECK_ARG(M >= 0 && K >= 0 && C >= 0 && lddz >= K, "grl_linear_bwd_data: bad sizes");
  if (M == 0 || K == 0) return GRL_OK;
  GRL_CHECK_ARG(g && W && dZ, "grl_linear_bwd_data: NULL pointer");
  GemmArgs a{};
  a.A = g;  // (M x C), k index = c contiguous
  a.lda = C;
  a.Amask = relu_out;
  a.B = W;  // B(k=c, n=kk) = W[kk][c]: K-contiguous rows of W
  a.ldb = C;
  a.C = dZ;
  a.ldc = lddz;
  a.M = M;
  a.N = K;
  a.K = C;
  const bool aligned = al16(g) && al16(W) && (!relu_out || al16(relu_out)) && C % 4 == 0;
  return run_output_gemm<true, true>(a, aligned, "grl_linear_bwd_data", workspace, workspace_bytes,
                                     as_stream(stream));
}

namespace grl {
namespace {
// x6t (split-bf16 dW) selection: same switch and size floor as the forward
bool x6t_shape_ok(int64_t M, int64_t K, int64_t C) {  // M nodes, K = rows of dW, C = its columns
  return x6_enabled() && M >= 16 && K >= 4 && C >= 4 && K % 4 == 0 && C % 4 == 0 &&
         2.0 * (double)M * (double)K * (double)C >= 1.6e10;
}

// K splits of the x6t dW: at most two 256 x 256 workgroups per CU (one is
// resident per CU at 96 KB of LDS, so the grid runs in two full rounds rather
// than two and a sliver), >= 16 K16 steps each (1, 3 and 4 rounds were
// measured slower, profiles/r04_ab_dw_split_whatif.txt)
constexpr int64_t X6T_ROUNDS = 2;
int x6t_splits(int64_t M, int64_t K, int64_t C) {
  const int64_t tiles = ceil_div(K, LB_M) * ceil_div(C, LB_N);
  int64_t s = (X6T_ROUNDS * (int64_t)device_cu_count()) / tiles;
  s = std::min<int64_t>(s, ceil_div(M, 16 * X6_K));
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 512));
}

// slabs reserved in the dW workspace: enough for whichever path runs
int wgt_slab_splits(int64_t M, int64_t K, int64_t C) {
  int s = pick_splits(K, C, M);
  if (x6t_shape_ok(M, K, C)) s = std::max(s, x6t_splits(M, K, C));
  return s;
}

}  // namespace
}  // namespace grl

extern "C" size_t grl_linear_bwd_weight_workspace_size(int64_t M, int32_t K, int32_t C) {
  const int s = wgt_slab_splits(M, K, C);
  const int zs = colsum_splits(M);
  return (size_t)s * (size_t)K * (size_t)C * 4 + (size_t)zs * (size_t)C * 4 + 512;
}

extern "C" size_t grl_relu_grad_workspace_size(int64_t M, int32_t C) {
  return (size_t)grl::colsum_splits(M) * (size_t)std::max<int32_t>(C, 0) * 4 + 256;
}

extern "C" int grl_relu_grad(const float* g, const float* relu_out, float* g_eff, float* db, int64_t M, int32_t C,
                             void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  using namespace grl;
  TraceRange trace_("grl_relu_grad");
  GRL_CHECK_ARG(M >= 0 && C >= 0, "grl_relu_grad: bad sizes");
  if (C == 0) return GRL_OK;
  if (M == 0) {  // no rows (an empty node-range shard): nothing to mask, db = 0
    if (db && hipMemsetAsync(db, 0, (size_t)C * sizeof(float), as_stream(stream)) != hipSuccess)
      GRL_FAIL(GRL_E_HIP, "grl_relu_grad: hipMemsetAsync failed");
    return GRL_OK;
  }
  GRL_CHECK_ARG(g && relu_out && g_eff, "grl_relu_grad: NULL pointer");
  const size_t need = grl_relu_grad_workspace_size(M, C);
  if (db && (!workspace || workspace_bytes < need))
    GRL_FAIL(GRL_E_WORKSPACE, "grl_relu_grad: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  const int zs = colsum_splits(M);
  const int64_t rows_per = ceil_div(std::max<int64_t>(M, 1), zs);
  float* part = db ? static_cast<float*>(workspace) : nullptr;
  // (a 16-B-per-lane variant measured no faster: 0.64 vs 0.61 ms at M = 1M, C = 256)
  hipLaunchKernelGGL(relu_grad_colsum_kernel, dim3((unsigned)ceil_div(C, 256), (unsigned)zs), dim3(256), 0, st, g,
                     relu_out, g_eff, M, (int64_t)C, rows_per, part);
  GRL_LAUNCH_CHECK();
  if (db) {
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)ceil_div(C, 256)), dim3(256), 0, st, part, (int64_t)C, zs,
                       db);
    GRL_LAUNCH_CHECK();
  }
  return GRL_OK;
}

extern "C" int grl_linear_bwd_weight(const float* Z, int64_t ldz, const float* g, const float* relu_out, float* dW,
                                     float* db, int64_t M, int32_t K, int32_t C, void* workspace,
                                     size_t workspace_bytes, grl_stream_t stream) {
  TraceRange trace_("grl_linear_bwd_weight");
  GRL_CHECK_ARG(M >= 0 && K >= 0 && C >= 0 && ldz >= K, "grl_linear_bwd_weight: bad sizes");
  if (K == 0 || C == 0) return GRL_OK;
  if (M == 0) {  // no rows (an empty node-range shard): dW = 0, db = 0
    GRL_CHECK_ARG(dW, "grl_linear_bwd_weight: NULL pointer");
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(dW, 0, (size_t)K * C * sizeof(float), st) != hipSuccess ||
        (db && hipMemsetAsync(db, 0, (size_t)C * sizeof(float), st) != hipSuccess))
      GRL_FAIL(GRL_E_HIP, "grl_linear_bwd_weight: hipMemsetAsync failed");
    return GRL_OK;
  }
  GRL_CHECK_ARG(Z && g && dW, "grl_linear_bwd_weight: NULL pointer");
  const size_t need = grl_linear_bwd_weight_workspace_size(M, K, C);
  if (!workspace || workspace_bytes < need)
    GRL_FAIL(GRL_E_WORKSPACE, "grl_linear_bwd_weight: workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = as_stream(stream);
  float* slab = static_cast<float*>(workspace);
  GemmArgs a{};
  a.A = Z;  // A(m=kk, k=row) = Z[row][kk]: rows of Z are M-contiguous for fixed k
  a.lda = ldz;
  a.B = g;  // B(k=row, n=c) = g[row][c]
  a.ldb = C;
  a.Bmask = relu_out;
  a.ldc = C;
  a.M = K;
  a.N = C;
  a.K = M;
  const bool aligned = al16(Z) && al16(g) && (!relu_out || al16(relu_out)) && ldz % 4 == 0 && C % 4 == 0 && K % 4 == 0;
  int used;
  if (aligned && !relu_out && x6t_shape_ok(M, K, C)) {  // large M: fp32 on the bf16 matrix cores
    // (a v_mfma_f32_16x16x32_bf16 form -- 128 x 256 tiles, 32-deep stages, conflict-free transposed reads,
    // with or without the next stage's split interleaved -- was 10 % slower at C3: 5.31 / 5.38 vs 4.81 ms,
    // profiles/r05_ab_dw16.txt; 16 x 16 fragments cost a third more LDS reads per flop here)
    const int splits = x6t_splits(M, K, C);
    a.C = splits > 1 ? slab : dW;
    a.k_per_split = ceil_div(ceil_div(M, splits), X6_K) * X6_K;
    used = (int)ceil_div(M, a.k_per_split);
    a.mt = ceil_div(a.M, LB_M);
    a.nt = ceil_div(a.N, LB_N);
    a.zt = used;
    a.inner_n = 0;
    GRL_CHECK_ARG(a.mt * a.nt * a.zt < 2147483647LL, "gemm: grid too large");
    const dim3 grid((unsigned)(a.mt * a.nt * a.zt));
    if (used > 1)
      hipLaunchKernelGGL(gemm_x6t_kernel<EPI_SLAB>, grid, dim3(512), 0, st, a);
    else
      hipLaunchKernelGGL(gemm_x6t_kernel<EPI_STORE>, grid, dim3(512), 0, st, a);
    GRL_LAUNCH_CHECK();
  } else {
    const int splits = pick_splits(K, C, M);
    a.C = splits > 1 ? slab : dW;
    a.k_per_split = ceil_div(ceil_div(M, splits), GEMM_BK) * GEMM_BK;
    used = (int)ceil_div(M, a.k_per_split);
    const int rc = used > 1 ? launch_gemm<false, false, EPI_SLAB>(a, used, aligned, st)
                            : launch_gemm<false, false, EPI_STORE>(a, 1, aligned, st);
    if (rc) return rc;
  }
  if (used > 1) {
    const int64_t n = (int64_t)K * C;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, 256), 65536)), dim3(256), 0,
                       st, slab, n, used, dW);
    GRL_LAUNCH_CHECK();
  }
  if (db) {
    const int zs = colsum_splits(M);
    float* part = slab + (size_t)wgt_slab_splits(M, K, C) * K * C;
    const int64_t rows_per = ceil_div(std::max<int64_t>(M, 1), zs);
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)ceil_div(C, 256), (unsigned)zs), dim3(256), 0, st, g,
                       relu_out, M, C, rows_per, part);
    GRL_LAUNCH_CHECK();
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)ceil_div(C, 256)), dim3(256), 0, st, part, (int64_t)C, zs,
                       db);
    GRL_LAUNCH_CHECK();
  }
  return GRL_OK;
}
