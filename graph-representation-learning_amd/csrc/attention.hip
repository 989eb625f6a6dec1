// NodeSelfAtten (gnn/models/networks/robust_gcn.py:78-99) as fused fp32
// MFMA kernels, flash-style: the B x N x N score matrix never exists.
//
//   S = Q K^T            Q = f(V), K = g(V): [B, N, dk]   (no 1/sqrt(dk), :94)
//   P = softmax_rows(S)                                    (:84, :94)
//   out = gamma * (P H) + V                                (:95-96), H = h(V): [B, N, dv]
//
// Layout trick.  With v_mfma_f32_32x32x2_f32 the accumulator's column is the
// lane (lane & 31) and its rows live in registers.  We compute the
// TRANSPOSED products S^T = K Q^T and O^T = H^T P^T, so every lane owns one
// query: the online-softmax max / sum are in-lane over 16 registers plus one
// exchange with lane ^ 32 (the two half-waves hold the two key halves), and
// the rescale of O^T is lane-local.  The P registers feed the second MFMA
// directly as its B operand when the k index of step s in half h is the key
// kappa(s, h) = (s & 3) + 8 (s >> 2) + 4 h -- exactly the key that register s
// of that half holds.  Products are exact fp32; sums are fp32.
//
// Backward (deterministic, no atomics), with dO = gamma * d_out and
// D = rowsum(dO * O_norm) precomputed on the host side:
//   kernel A (query-stationary): recompute P, dP^T = H dO^T, dS = P (dP - D),
//            dQ^T += K^T dS^T
//   kernel B (key-stationary):   recompute S with keys on lanes, dP likewise,
//            dH^T += dO^T P,  dK^T += Q^T dS
//   dk <= 16 with a workspace: kernel A's dQ is folded into kernel B's dK
//   pass instead (attn_bwd_kq_x6_kernel: per-workgroup slabs, ordered sum)
#include "grl_internal.h"

#include <math.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace grl {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

struct AttnArgs {
  const float* Q;      // [B, N, dk]
  const float* K;      // [B, N, dk]
  const float* H;      // [B, N, dv]
  const float* V;      // [B, N, dv] residual
  const float* gamma;  // [dv]
  float* out;          // [B, N, dv]
  float* onorm;        // [B, N, dv] or NULL: P H (normalised)
  float* rmax;         // [B, N] or NULL
  float* rsum;         // [B, N] or NULL
  const float* dO;     // [B, N, dv]  gamma * d_out
  const float* Drow;   // [B, N]      rowsum(dO * onorm)
  const float* smax;   // [B, N]      saved row max
  const float* ssum;   // [B, N]      saved row sum
  float* dQ;           // [B, N, dk]
  float* dK;           // [B, N, dk]
  float* dH;           // [B, N, dv]
  // x6 PRE staging: bf16 planes [3][B*N][W] split once per call (or NULL)
  const uint16_t* Kpl;  // W = DKP
  const uint16_t* Hpl;  // W = DV
  const uint16_t* Qpl;  // W = DKP
  const uint16_t* Opl;  // W = DV (dO)
  const uint16_t* Qpl16;  // bwd_kq: Q planes 16 wide
  // key / query split (small N): keys per split, and partial slabs (or NULL)
  int64_t kr;
  float* part;   // fwd: o [S][B*N][dv] + m, l [S][B*N]; bwd_q: dQ [S][B*N][dk]; bwd_kv: dH [S][B*N][dv]
  float* part2;  // bwd_kv: dK [S][B*N][dk]
  float* qslab;  // bwd_kq: dQ partials [B][ceil(N / 128)][N][16], one row block per key workgroup
  int64_t N;
  int dk, dv;
  // query rows computed: [q0, q1) of the N (forward and dQ: only these
  // outputs are written; dK / dH: only these queries contribute) -- a node-
  // range shard's own queries against every key (grl_node_attention_*_rows)
  int64_t q0, q1;
  // bwd_kq: first key of this launch, and key workgroups per launch (the
  // fused pass runs in key chunks whose dQ slabs fit the workspace; each
  // chunk's slabs are added onto dQ in order)
  int64_t k0, kq_chunk;
};

__device__ __forceinline__ int kappa(int s, int h) { return (s & 3) + 8 * (s >> 2) + 4 * h; }

// e^x for x <= 0 (softmax): one v_mul + v_exp_f32 (1 ulp) instead of expf's
// range-reduced sequence; exact at x = 0 (so alpha == 1 still detects an
// unchanged running max) and 0 at x = -inf
__device__ __forceinline__ float aexp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// The x6 kernels score in base 2: the lane's register operand of S (Q in the
// forward and dQ, K in dH / dK) is scaled by log2(e) before its split, so S
// arrives as log2(e) q.k and p = 2^(s - shift) is one v_sub + one v_exp
// (no per-score v_mul).  Saved row stats stay natural-log (rmax = max q.k,
// rsum): the backward forms lse2 = rmax log2(e) + log2(rsum) once per query
// and p = 2^(s - lse2), the normalisation folded into the exponent.
constexpr float ALOG2E = 1.44269504088896341f;
constexpr float ALN2 = 0.69314718055994531f;
__device__ __forceinline__ float aexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float alog2(float x) { return __builtin_amdgcn_logf(x); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.0f;
  return z;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// Rows [r0, r0+32) of a [N, width] matrix staged into an LDS tile[32][LD]
// (zero fill beyond N and beyond `width`, up to the padded width W).  fetch()
// issues every load of the tile into registers at once (float4 when the rows
// allow it) and store() writes them to LDS after the barrier, so the next
// block's loads are in flight while the current block is multiplied.
template <int W, int LD>
struct Stager {
  static constexpr int NF4 = 32 * W / 4;
  static constexpr int PER = (NF4 + 255) / 256;
  float4 reg[PER];

  __device__ __forceinline__ void fetch(const float* src, int64_t r0, int64_t N, int width, bool vec, int tid) {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int idx = tid + it * 256;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < NF4) {
        const int r = idx / (W / 4), c = (idx % (W / 4)) * 4;
        const int64_t row = r0 + r;
        if (row < N) {
          const float* sp = src + row * width + c;
          if (vec && c + 3 < width) {
            v = *reinterpret_cast<const float4*>(sp);
          } else {
            float* vp = reinterpret_cast<float*>(&v);
#pragma unroll
            for (int e = 0; e < 4; ++e) vp[e] = (c + e < width) ? sp[e] : 0.0f;
          }
        }
      }
      reg[it] = v;
    }
  }
  __device__ __forceinline__ void store(float* tile, int tid) const {
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int idx = tid + it * 256;
      if (idx < NF4) {
        const int r = idx / (W / 4), c = (idx % (W / 4)) * 4;
        *reinterpret_cast<float4*>(&tile[r * LD + c]) = reg[it];
      }
    }
  }
};

__device__ __forceinline__ bool vec_ok(const float* p, int width) {
  return p != nullptr && (width & 3) == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

template <int DKP, int NT>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  constexpr int KS = DKP / 2, DV = NT * 32, LDK = DKP + 4;
  __shared__ float Ks[32 * LDK];
  __shared__ float Hs[32 * DV];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Qb = a.Q + b * N * a.dk;
  const float* Kb = a.K + b * N * a.dk;
  const float* Hb = a.H + b * N * a.dv;
  const int64_t q = a.q0 + (int64_t)blockIdx.x * 128 + wave * 32 + l32;

  float qr[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d = h * KS + s;
    qr[s] = (q < a.q1 && d < a.dk) ? Qb[q * a.dk + d] : 0.0f;
  }
  f32x16 o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) o[t] = zero16();
  float m = -INFINITY, l = 0.0f;
  Stager<DKP, LDK> sk;
  Stager<DV, DV> sh;
  const bool vk = vec_ok(Kb, a.dk), vh = vec_ok(Hb, a.dv);
  sk.fetch(Kb, 0, N, a.dk, vk, tid);
  sh.fetch(Hb, 0, N, a.dv, vh, tid);

  for (int64_t k0 = 0; k0 < N; k0 += 32) {
    sk.store(Ks, tid);
    sh.store(Hs, tid);
    __syncthreads();
    if (k0 + 32 < N) {
      sk.fetch(Kb, k0 + 32, N, a.dk, vk, tid);
      sh.fetch(Hb, k0 + 32, N, a.dv, vh, tid);
    }
    f32x16 s = zero16();
#pragma unroll
    for (int st = 0; st < KS; ++st) s = MFMA(Ks[l32 * LDK + h * KS + st], qr[st], s);
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (k0 + kappa(r, h) >= N) s[r] = -INFINITY;
      mx = fmaxf(mx, s[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);
    const float alpha = aexp(m - mn);
    float ps = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = aexp(s[r] - mn);
      ps += s[r];
    }
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
#pragma unroll
      for (int st = 0; st < 16; ++st) o[t] = MFMA(Hs[kappa(st, h) * DV + t * 32 + l32], s[st], o[t]);
    }
    __syncthreads();
  }

  if (q < a.q1) {
    const float inv = 1.0f / l;
    const int64_t base = (b * N + q) * a.dv;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) {
          const float on = o[t][r] * inv;
          a.out[base + f] = a.gamma[f] * on + a.V[base + f];
          if (a.onorm) a.onorm[base + f] = on;
        }
      }
    if (h == 0 && a.rmax) {
      a.rmax[b * N + q] = m;
      a.rsum[b * N + q] = l;
    }
  }
}

// dQ: one wave per 32 queries, loop over key blocks.
template <int DKP, int NT>
__global__ __launch_bounds__(256) void attn_bwd_q_kernel(AttnArgs a) {
  constexpr int KS = DKP / 2, DV = NT * 32, HV = DV / 2, LDK = DKP + 4;
  __shared__ float Ks[32 * LDK];
  __shared__ float Hs[32 * DV];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Kb = a.K + b * N * a.dk;
  const float* Hb = a.H + b * N * a.dv;
  const int64_t q = a.q0 + (int64_t)blockIdx.x * 128 + wave * 32 + l32;
  const bool qv = q < a.q1;

  float qr[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d = h * KS + s;
    qr[s] = (qv && d < a.dk) ? a.Q[(b * N + q) * a.dk + d] : 0.0f;
  }
  float dor[HV];
#pragma unroll
  for (int s = 0; s < HV; ++s) {
    const int f = h * HV + s;
    dor[s] = (qv && f < a.dv) ? a.dO[(b * N + q) * a.dv + f] : 0.0f;
  }
  const float mq = qv ? a.smax[b * N + q] : 0.0f;
  const float il = qv ? 1.0f / a.ssum[b * N + q] : 0.0f;
  const float Dq = qv ? a.Drow[b * N + q] : 0.0f;
  constexpr int DT = (DKP + 31) / 32;  // 32-wide dQ tiles (dk up to 64)
  f32x16 dq[DT];
#pragma unroll
  for (int j = 0; j < DT; ++j) dq[j] = zero16();
  Stager<DKP, LDK> sk;
  Stager<DV, DV> sh;
  const bool vk = vec_ok(Kb, a.dk), vh = vec_ok(Hb, a.dv);
  sk.fetch(Kb, 0, N, a.dk, vk, tid);
  sh.fetch(Hb, 0, N, a.dv, vh, tid);

  for (int64_t k0 = 0; k0 < N; k0 += 32) {
    sk.store(Ks, tid);
    sh.store(Hs, tid);
    __syncthreads();
    if (k0 + 32 < N) {
      sk.fetch(Kb, k0 + 32, N, a.dk, vk, tid);
      sh.fetch(Hb, k0 + 32, N, a.dv, vh, tid);
    }
    f32x16 s = zero16();
#pragma unroll
    for (int st = 0; st < KS; ++st) s = MFMA(Ks[l32 * LDK + h * KS + st], qr[st], s);
    f32x16 dp = zero16();
#pragma unroll
    for (int st = 0; st < HV; ++st) dp = MFMA(Hs[l32 * DV + h * HV + st], dor[st], dp);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = (k0 + kappa(r, h) < N) ? aexp(s[r] - mq) * il : 0.0f;
      s[r] = p * (dp[r] - Dq);  // dS
    }
#pragma unroll
    for (int j = 0; j < DT; ++j)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const float kv = 32 * j + l32 < DKP ? Ks[kappa(st, h) * LDK + 32 * j + l32] : 0.0f;
        dq[j] = MFMA(kv, s[st], dq[j]);
      }
    __syncthreads();
  }
  if (qv) {
#pragma unroll
    for (int j = 0; j < DT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * j + kappa(r, h);
        if (d < a.dk) a.dQ[(b * N + q) * a.dk + d] = dq[j][r];
      }
  }
}

// dK, dH: one wave per 32 keys, loop over query blocks.
template <int DKP, int NT>
__global__ __launch_bounds__(256) void attn_bwd_kv_kernel(AttnArgs a) {
  constexpr int KS = DKP / 2, DV = NT * 32, HV = DV / 2, LDK = DKP + 4;
  __shared__ float Qs[32 * LDK];
  __shared__ float Os[32 * DV];
  __shared__ float Ms[32], Ls[32], Ds[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Qb = a.Q + b * N * a.dk;
  const float* dOb = a.dO + b * N * a.dv;
  const int64_t key = (int64_t)blockIdx.x * 128 + wave * 32 + l32;
  const bool kv = key < N;

  float kr[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int d = h * KS + s;
    kr[s] = (kv && d < a.dk) ? a.K[(b * N + key) * a.dk + d] : 0.0f;
  }
  float hr[HV];
#pragma unroll
  for (int s = 0; s < HV; ++s) {
    const int f = h * HV + s;
    hr[s] = (kv && f < a.dv) ? a.H[(b * N + key) * a.dv + f] : 0.0f;
  }
  f32x16 dh[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dh[t] = zero16();
  constexpr int DT = (DKP + 31) / 32;  // 32-wide dK tiles (dk up to 64)
  f32x16 dk[DT];
#pragma unroll
  for (int j = 0; j < DT; ++j) dk[j] = zero16();

  Stager<DKP, LDK> sq;
  Stager<DV, DV> so;
  const bool vq = vec_ok(Qb, a.dk), vo = vec_ok(dOb, a.dv);
  float pm = 0.0f, pl = 0.0f, pd = 0.0f;  // this thread's row statistics (tid < 32)
  auto fetch_stats = [&](int64_t q0) {
    if (tid < 32) {
      const int64_t qq = q0 + tid;
      const bool v = qq < a.q1;
      pm = v ? a.smax[b * N + qq] : 0.0f;
      pl = v ? 1.0f / a.ssum[b * N + qq] : 0.0f;  // 0 => P = 0 for padded queries
      pd = v ? a.Drow[b * N + qq] : 0.0f;
    }
  };
  sq.fetch(Qb, a.q0, N, a.dk, vq, tid);
  so.fetch(dOb, a.q0, N, a.dv, vo, tid);
  fetch_stats(a.q0);

  for (int64_t q0 = a.q0; q0 < a.q1; q0 += 32) {
    sq.store(Qs, tid);
    so.store(Os, tid);
    if (tid < 32) {
      Ms[tid] = pm;
      Ls[tid] = pl;
      Ds[tid] = pd;
    }
    __syncthreads();
    if (q0 + 32 < N) {
      sq.fetch(Qb, q0 + 32, N, a.dk, vq, tid);
      so.fetch(dOb, q0 + 32, N, a.dv, vo, tid);
      fetch_stats(q0 + 32);
    }
    // S[query][key]: lanes = keys, registers = queries kappa(r, h)
    f32x16 s = zero16();
#pragma unroll
    for (int st = 0; st < KS; ++st) s = MFMA(Qs[l32 * LDK + h * KS + st], kr[st], s);
    f32x16 dp = zero16();
#pragma unroll
    for (int st = 0; st < HV; ++st) dp = MFMA(Os[l32 * DV + h * HV + st], hr[st], dp);
    f32x16 ds;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = kappa(r, h);
      const float p = kv ? aexp(s[r] - Ms[qi]) * Ls[qi] : 0.0f;
      s[r] = p;
      ds[r] = p * (dp[r] - Ds[qi]);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int st = 0; st < 16; ++st) dh[t] = MFMA(Os[kappa(st, h) * DV + t * 32 + l32], s[st], dh[t]);
#pragma unroll
    for (int j = 0; j < DT; ++j)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const float qv = 32 * j + l32 < DKP ? Qs[kappa(st, h) * LDK + 32 * j + l32] : 0.0f;
        dk[j] = MFMA(qv, ds[st], dk[j]);
      }
    __syncthreads();
  }
  if (kv) {
    const int64_t rowv = (b * N + key) * a.dv, rowk = (b * N + key) * a.dk;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) a.dH[rowv + f] = dh[t][r];
      }
#pragma unroll
    for (int j = 0; j < DT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = 32 * j + kappa(r, h);
        if (d < a.dk) a.dK[rowk + d] = dk[j][r];
      }
  }
}

// ---------------------------------------------------------------------------
// Forward on the bf16 matrix cores by exact three-way splitting (the "x6"
// scheme of linear.hip): every fp32 operand value is
// v0 + v1 + v2 in bf16 exactly, and the six products with i + j <= 2 run on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation -- fp32-level accuracy at
// 6 x 32 MFMA cycles per 32x32x16 block instead of 8 x 64.  Same transposed
// products as attn_fwd_kernel (S^T = K Q^T, O^T += H^T P^T, one query per
// lane, keys in registers).  Q is split once into registers; each 32-key block
// of K and H is split while staged into LDS planes; P is split in registers.
// O^T's MFMA u (u = 0, 1) takes key slot 8h + j <-> key kappa(8u + j, h) --
// P registers 8u..8u+7 as the B operand -- and the matching H^T rows come
// out of ds_read_b64_tr_b16, whose 16-lane groups gather 4 rows (keys) x 16
// columns (features) from per-lane row addresses.  H plane rows keep column c
// at c ^ ((key & 3) << 5) so the four keys of a transposed read sit in
// different banks (DV >= 128).
typedef __bf16 abf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 abf16x2_t __attribute__((ext_vector_type(2)));
typedef float af32x2_t __attribute__((ext_vector_type(2)));
typedef short ai16x4_t __attribute__((ext_vector_type(4)));
typedef short ai16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t apack(float a, float b) {
  af32x2_t p = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(p, abf16x2_t));
}
__device__ __forceinline__ float alo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float ahi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// v (4 floats) -> three planes of 4 bf16 with v == p0 + p1 + p2 exactly
__device__ __forceinline__ void asplit3(float4 v, uint2& p0, uint2& p1, uint2& p2) {
  p0.x = apack(v.x, v.y);
  p0.y = apack(v.z, v.w);
  float4 r = make_float4(v.x - alo(p0.x), v.y - ahi(p0.x), v.z - alo(p0.y), v.w - ahi(p0.y));
  p1.x = apack(r.x, r.y);
  p1.y = apack(r.z, r.w);
  r = make_float4(r.x - alo(p1.x), r.y - ahi(p1.x), r.z - alo(p1.y), r.w - ahi(p1.y));
  p2.x = apack(r.x, r.y);
  p2.y = apack(r.z, r.w);
}

// 8 floats -> three bf16x8 planes
__device__ __forceinline__ void asplit8(float4 lo, float4 hi, abf16x8_t& a0, abf16x8_t& a1, abf16x8_t& a2) {
  uint2 l0, l1, l2, h0, h1, h2;
  asplit3(lo, l0, l1, l2);
  asplit3(hi, h0, h1, h2);
  a0 = __builtin_bit_cast(abf16x8_t, make_uint4(l0.x, l0.y, h0.x, h0.y));
  a1 = __builtin_bit_cast(abf16x8_t, make_uint4(l1.x, l1.y, h1.x, h1.y));
  a2 = __builtin_bit_cast(abf16x8_t, make_uint4(l2.x, l2.y, h2.x, h2.y));
}

#if defined(GRL_DIAG) && defined(GRL_ATTN_WI16)
// what-if (diagnostic builds only; timing, wrong results): every 32x32x16
// product as two v_mfma_f32_16x16x32_bf16 on the same operand registers into
// two quarters of the accumulator -- the same FLOPs and pipe cycles in the
// 16x16x32 shape, to price its clock against the 32x32x16 kernels
typedef float af32x4_t __attribute__((ext_vector_type(4)));
#define WI16(q0, q1, a, b)                                                   \
  do {                                                                      \
    q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, q0, 0, 0, 0);        \
    q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, q1, 0, 0, 0);        \
  } while (0)
#define MFMA6(acc, a0, a1, a2, b0, b1, b2)                                  \
  do {                                                                      \
    af32x4_t q0_ = {acc[0], acc[1], acc[2], acc[3]}, q1_ = {acc[4], acc[5], acc[6], acc[7]};       \
    af32x4_t q2_ = {acc[8], acc[9], acc[10], acc[11]}, q3_ = {acc[12], acc[13], acc[14], acc[15]}; \
    WI16(q0_, q1_, a2, b0);                                                 \
    WI16(q2_, q3_, a1, b1);                                                 \
    WI16(q0_, q1_, a0, b2);                                                 \
    WI16(q2_, q3_, a1, b0);                                                 \
    WI16(q0_, q1_, a0, b1);                                                 \
    WI16(q2_, q3_, a0, b0);                                                 \
    for (int r_ = 0; r_ < 4; ++r_) {                                        \
      acc[r_] = q0_[r_];                                                    \
      acc[4 + r_] = q1_[r_];                                                \
      acc[8 + r_] = q2_[r_];                                                \
      acc[12 + r_] = q3_[r_];                                               \
    }                                                                       \
  } while (0)
#else
#define MFMA6(acc, a0, a1, a2, b0, b1, b2)                                  \
  do {                                                                      \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc, 0, 0, 0);   \
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);   \
  } while (0)
#endif

template <int W>
__device__ __forceinline__ int hswz(int key, int col) {  // H plane element offset
  return key * W + (W >= 128 ? (col ^ ((key & 3) << 5)) : col);
}

__device__ __forceinline__ int swz128(int row, int col) {
  const int sw = ((row & 3) << 2) | ((row >> 2) & 3);
  return row * 128 + ((((col >> 3) ^ sw)) << 3) + (col & 7);
}

// LDS plane layouts of a 32-row block: PLAIN [32][LW], HSWZ (forward H:
// column c of row r at c ^ ((r & 3) << 5) when W >= 128), SWZ128 (backward
// 128-wide planes, image (b) of cdna_hip_programming.md T10)
enum PlaneLayout { PL_PLAIN = 0, PL_HSWZ = 1, PL_SWZ128 = 2 };

template <int W, int LW, int LAYOUT>
__device__ __forceinline__ int plane_off(int r, int c) {
  if (LAYOUT == PL_SWZ128) return swz128(r, c);
  if (LAYOUT == PL_HSWZ) return hswz<W>(r, c);
  return r * LW + c;
}

// One operand's 32-row blocks -> three bf16 LDS planes of LW-element rows,
// for the kernels' no-workspace path: fp32 rows are fetched (float4, zero
// fill) into registers and split at store.  fetch() is issued for the next
// block before the current one's MFMAs.  (With a workspace the operands are
// split once per call and staged by LDS-DMA instead: dma_block.)
template <int W, int LW, int LAYOUT>
struct XStage {
  static constexpr int PL = 32 * LW;  // LDS elements per plane
  Stager<W, W> f32;

  __device__ __forceinline__ void fetch(const float* src, int64_t r0, int64_t N, int width, bool vec, int tid) {
    f32.fetch(src, r0, N, width, vec, tid);
  }
  __device__ __forceinline__ void store(uint16_t* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < Stager<W, W>::PER; ++it) {
      const int idx = tid + it * 256;
      if (idx < Stager<W, W>::NF4) {
        const int r = idx / (W / 4), c = (idx % (W / 4)) * 4;
        uint2 p0, p1, p2;
        asplit3(f32.reg[it], p0, p1, p2);
        const int off = plane_off<W, LW, LAYOUT>(r, c);
        *reinterpret_cast<uint2*>(&lds[off]) = p0;
        *reinterpret_cast<uint2*>(&lds[PL + off]) = p1;
        *reinterpret_cast<uint2*>(&lds[2 * PL + off]) = p2;
      }
    }
  }
};

// planes[p][r][0..W) = bf16 part p of src[r][0..width) (zero beyond width):
// the once-per-call split of an attention operand for the PRE staging path
__global__ void attn_split_rows_kernel(const float* __restrict__ src, int64_t rows, int width, int W,
                                       uint16_t* __restrict__ planes) {
  const int64_t n4 = rows * (W / 4), ps = rows * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / (W / 4);
    const int c = (int)(i % (W / 4)) * 4;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = c + e < width ? src[r * width + c + e] : 0.0f;
    uint2 p0, p1, p2;
    asplit3(make_float4(v[0], v[1], v[2], v[3]), p0, p1, p2);
    *reinterpret_cast<uint2*>(planes + r * W + c) = p0;
    *reinterpret_cast<uint2*>(planes + ps + r * W + c) = p1;
    *reinterpret_cast<uint2*>(planes + 2 * ps + r * W + c) = p2;
  }
}

// global -> LDS DMA of one 16 B chunk per lane (lane l lands at lds_base + 16 l),
// issued from asm so that hipcc's waitcnt pass neither sees nor waits on it
__device__ __forceinline__ void adma16(const void* src, const void* lds_base) {
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

// PRE staging: one 32-row block of pre-split planes [3][rows][W] -> LDS
// [3][32][W] in LAYOUT by LDS-DMA (no VGPRs, no VALU).  The DMA lands
// lane-linear, so each lane fetches the source chunk whose swizzled position
// is its destination.  Rows past N re-read row N-1 (finite values whose
// scores / probabilities the kernels mask to zero).  Completion: the
// caller's vmcnt(0) + barrier at the top of the block that reads it.
template <int W, int LAYOUT, int NW = 4>
__device__ __forceinline__ void dma_block(const uint16_t* planes, int64_t ps, int64_t r0, int64_t N, uint16_t* lds,
                                          int wave, int lane) {
  constexpr int PL = 32 * W, NI = 3 * PL / 512;  // 1 KB chunks, dealt to the NW waves of the workgroup
  const int ln = lane;
#pragma unroll
  for (int j = 0; j < (NI + NW - 1) / NW; ++j) {
    const int i = wave + NW * j;
    if (i < NI) {
      const int e = i * 512 + ln * 8;
      const int pl = e / PL, rem = e % PL, r = rem / W, pos = rem % W;
      int c = pos;
      if (LAYOUT == PL_HSWZ && W >= 128) c = pos ^ ((r & 3) << 5);
      if (LAYOUT == PL_SWZ128) c = ((pos >> 3) ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 3;
      const int64_t row = min<int64_t>(r0 + r, N - 1);
      adma16(planes + pl * ps + row * W + c, lds + i * 512);
    }
  }
}

// dma_block with this lane's chunk addresses computed once: per block only a
// uniform row offset is added (the last, partial block takes dma_block's
// clamped path).  Costs 2 VGPRs per chunk slot (the forward has the room).
template <int W, int LAYOUT, int NW = 4>
struct DmaRows {
  static constexpr int PL = 32 * W, NI = 3 * PL / 512, NJ = (NI + NW - 1) / NW;
  const uint16_t* planes;
  const uint16_t* src[NJ];
  int64_t ps;
  __device__ __forceinline__ void init(const uint16_t* planes_, int64_t ps_, int wave, int lane) {
    planes = planes_;
    ps = ps_;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int i = wave + NW * j;
      const int e = (i < NI ? i : 0) * 512 + lane * 8;
      const int pl = e / PL, rem = e % PL, r = rem / W, pos = rem % W;
      int c = pos;
      if (LAYOUT == PL_HSWZ && W >= 128) c = pos ^ ((r & 3) << 5);
      if (LAYOUT == PL_SWZ128) c = ((pos >> 3) ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 3;
      src[j] = planes_ + pl * ps_ + (int64_t)r * W + c;
    }
  }
  __device__ __forceinline__ void issue(int64_t r0, int64_t N, uint16_t* lds, int wave, int lane) const {
    if (r0 + 32 <= N) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int i = wave + NW * j;
        if (i < NI) adma16(src[j] + r0 * W, lds + i * 512);
      }
    } else {
      dma_block<W, LAYOUT, NW>(planes, ps, r0, N, lds, wave, lane);
    }
  }
};

template <int DKP, int NT, bool PRE, bool SPLIT>
__global__ __launch_bounds__(256) void attn_fwd_x6_kernel(AttnArgs a) {
  constexpr int DV = NT * 32, KC = DKP / 16;
  constexpr int KPL = 32 * DKP, HPL = 32 * DV;  // bf16 per plane
  __shared__ __attribute__((aligned(16))) uint16_t Kp_s[(PRE ? 2 : 1) * 3 * KPL];  // PRE: 2 stages
  __shared__ __attribute__((aligned(16))) uint16_t Hp_s[(PRE ? 2 : 1) * 3 * HPL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Qb = a.Q + b * N * a.dk;
  const float* Kb = a.K + b * N * a.dk;
  const float* Hb = a.H + b * N * a.dv;
  const int64_t q = a.q0 + (int64_t)blockIdx.x * 128 + wave * 32 + l32;
  // key split blockIdx.z covers keys [k_lo, k_hi) (the whole range when unsplit)
  const int64_t k_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : 0, k_hi = SPLIT ? min<int64_t>(N, k_lo + a.kr) : N;

  // this lane's query, dims kc*16 + 8h + 0..7, split into three planes
  abf16x8_t qp[KC][3];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = kc * 16 + 8 * h + j;
      v[j] = (q < a.q1 && d < a.dk) ? Qb[q * a.dk + d] * ALOG2E : 0.0f;  // base-2 scores
    }
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), qp[kc][0], qp[kc][1],
            qp[kc][2]);
  }
  f32x16 o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) o[t] = zero16();
  float m = -INFINITY, l = 0.0f;
  XStage<DKP, DKP, PL_PLAIN> sk;
  XStage<DV, DV, PL_HSWZ> sh;
  const int64_t kps = (int64_t)gridDim.y * N * DKP, hps = (int64_t)gridDim.y * N * DV;
  const uint16_t* Kpb = a.Kpl + b * N * DKP;
  const uint16_t* Hpb = a.Hpl + b * N * DV;
  const bool vk = vec_ok(Kb, a.dk), vh = vec_ok(Hb, a.dv);
  DmaRows<DKP, PL_PLAIN> kd;
  DmaRows<DV, PL_HSWZ> hd;
  if constexpr (PRE) {
    kd.init(Kpb, kps, wave, lane);
    hd.init(Hpb, hps, wave, lane);
    kd.issue(k_lo, N, Kp_s, wave, lane);
    hd.issue(k_lo, N, Hp_s, wave, lane);
  } else {
    sk.fetch(Kb, k_lo, N, a.dk, vk, tid);
    sh.fetch(Hb, k_lo, N, a.dv, vh, tid);
  }
  // transposed-read coordinates: group row q' = (lane & 15) >> 2, columns 16 ((lane >> 4) & 1) + 4 (lane & 3)
  const int trq = (lane & 15) >> 2;
  const int trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  for (int64_t k0 = k_lo; k0 < k_hi; k0 += 32) {
    const int stg = PRE ? (int)(((k0 - k_lo) >> 5) & 1) : 0;
    uint16_t* Kp = Kp_s + stg * 3 * KPL;
    uint16_t* Hp = Hp_s + stg * 3 * HPL;
    if constexpr (PRE) {
      // this block's DMA landed (every wave's), and every wave is done with
      // the other stage (block k0 - 32): refill it with the next block
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (k0 + 32 < k_hi) {
        kd.issue(k0 + 32, N, Kp_s + (stg ^ 1) * 3 * KPL, wave, lane);
        hd.issue(k0 + 32, N, Hp_s + (stg ^ 1) * 3 * HPL, wave, lane);
      }
    } else {
      sk.store(Kp, tid);  // the staged K and H block -> bf16 planes
      sh.store(Hp, tid);
      __syncthreads();
      if (k0 + 32 < k_hi) {
        sk.fetch(Kb, k0 + 32, N, a.dk, vk, tid);
        sh.fetch(Hb, k0 + 32, N, a.dv, vh, tid);
      }
    }
    // S^T = K Q^T: A = K[key l32][kc*16 + 8h ..], B = Q
    f32x16 s = zero16();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int off = l32 * DKP + kc * 16 + 8 * h;
      const abf16x8_t k0p = *reinterpret_cast<const abf16x8_t*>(&Kp[off]);
      const abf16x8_t k1p = *reinterpret_cast<const abf16x8_t*>(&Kp[KPL + off]);
      const abf16x8_t k2p = *reinterpret_cast<const abf16x8_t*>(&Kp[2 * KPL + off]);
      MFMA6(s, k0p, k1p, k2p, qp[kc][0], qp[kc][1], qp[kc][2]);
    }
    if (k0 + 32 > k_hi) {  // the last, partial key block only (wave-uniform)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (k0 + kappa(r, h) >= k_hi) s[r] = -INFINITY;
    }
    float mx = fmaxf(s[0], s[1]);
#pragma unroll
    for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, s[r]), s[r + 1]);  // v_max3
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);
    const float alpha = aexp2(m - mn);
    float ps = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = aexp2(s[r] - mn);
      ps += s[r];
    }
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
    abf16x8_t pp[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u)
      asplit8(make_float4(s[8 * u], s[8 * u + 1], s[8 * u + 2], s[8 * u + 3]),
              make_float4(s[8 * u + 4], s[8 * u + 5], s[8 * u + 6], s[8 * u + 7]), pp[u][0], pp[u][1], pp[u][2]);
    // the running max of a wave's 32 queries rarely moves after the first
    // key blocks: alpha == 1 exactly then, and the 16 x NT rescale multiplies
    // are skipped wave-uniformly (x * 1 == x, so results are unchanged)
    const bool rescale = __any(alpha != 1.0f);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (rescale) {
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        abf16x8_t hp[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          typedef __attribute__((address_space(3))) ai16x4_t lds_v4;
          const int key0 = kappa(8 * u + trq, h), key1 = kappa(8 * u + 4 + trq, h);
          const uint16_t* p0 = &Hp[pl * HPL + hswz<DV>(key0, t * 32 + trc)];
          const uint16_t* p1 = &Hp[pl * HPL + hswz<DV>(key1, t * 32 + trc)];
          const ai16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p0);
          const ai16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p1);
          const ai16x8_t v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          hp[pl] = __builtin_bit_cast(abf16x8_t, v);
        }
        MFMA6(o[t], hp[0], hp[1], hp[2], pp[u][0], pp[u][1], pp[u][2]);
      }
    }
    if constexpr (!PRE) __syncthreads();
  }

  if (SPLIT && q < a.q1) {  // key split: unnormalised partials, combined by attn_fwd_combine_kernel
    const int64_t rows = (int64_t)gridDim.y * N, row = b * N + q, zs = blockIdx.z;
    float* po = a.part + zs * rows * a.dv + row * a.dv;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) po[f] = o[t][r];
      }
    if (h == 0) {
      float* pm = a.part + (int64_t)gridDim.z * rows * a.dv;
      pm[zs * rows + row] = m;
      pm[((int64_t)gridDim.z + zs) * rows + row] = l;
    }
  } else if (q < a.q1) {
    const float inv = 1.0f / l;
    const int64_t base = (b * N + q) * a.dv;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) {
          const float on = o[t][r] * inv;
          a.out[base + f] = a.gamma[f] * on + a.V[base + f];
          if (a.onorm) a.onorm[base + f] = on;
        }
      }
    if (h == 0 && a.rmax) {
      a.rmax[b * N + q] = m * ALN2;  // natural-log row max (the saved-stat contract)
      a.rsum[b * N + q] = l;
    }
  }
}

// ---------------------------------------------------------------------------
// The x6 forward software-pipelined within the wave (PRE staging only):
// iteration k runs block k's O^T += H^T P^T MFMAs with the softmax of block
// k+1 -- max, 2^(s - m), row sum, the split of P into planes -- in the same
// basic block, so the VALU issues in the MFMA gaps instead of between the
// blocks' MFMA phases (attn_fwd_x6_kernel: 61 % MFMA busy at N = 100k, the
// softmax on the critical path of every block).  Block k+1's scores come
// from its K planes, so K is staged three blocks deep (block k+2 in flight)
// and H two.  Same products, same order of every sum as attn_fwd_x6_kernel,
// hence the same bits.  The last block's partial-key mask is applied in its
// own instantiation of the iteration (MASK), outside the interleaved body.
#ifndef GRL_ATTN_HU2
#define GRL_ATTN_HU2 1
#endif
typedef __attribute__((address_space(3))) uint16_t lds_u16;
#ifndef GRL_ATTN_PIN_PN
#define GRL_ATTN_PIN_PN 1
#endif
#ifndef GRL_ATTN_B2
#define GRL_ATTN_B2 1
#endif
#ifndef GRL_ATTN_HPF
#define GRL_ATTN_HPF 1
#endif
template <int DKP, int NT, bool SPLIT, int NW = 4>
__global__ __launch_bounds__(64 * NW) void attn_fwd_x6p_kernel(AttnArgs a) {
  constexpr int DV = NT * 32, KC = DKP / 16;
  constexpr int KPL = 32 * DKP, HPL = 32 * DV;  // bf16 per plane
  constexpr int KST = 3 * KPL, HST = 3 * HPL;   // one stage: the three planes
  // B2 (GRL_ATTN_B2, 8-wave workgroups): one barrier per TWO key blocks --
  // four H and four K stages, the next pair's DMAs issued at the pair's
  // barrier (108 KB of LDS at dv = 128; the 8-wave form runs one workgroup
  // per CU anyway).  Else one barrier per block, H 2 / K 3 stages deep.
  constexpr bool B2 = GRL_ATTN_B2 && NW == 8 && NT <= 4;  // dv = 256: 4 H stages exceed the LDS
  __shared__ __attribute__((aligned(16))) uint16_t Kp_s[(B2 ? 4 : 3) * KST];
  __shared__ __attribute__((aligned(16))) uint16_t Hp_s[(B2 ? 4 : 2) * HST];
  auto hstage = [](int j) { return B2 ? (j & 3) : (j & 1); };
  auto kstage = [](int j) { return B2 ? (j & 3) : (j % 3); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Qb = a.Q + b * N * a.dk;
  const int64_t q = a.q0 + (int64_t)blockIdx.x * (32 * NW) + wave * 32 + l32;
  const int64_t k_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : 0, k_hi = SPLIT ? min<int64_t>(N, k_lo + a.kr) : N;
  const int nblk = (int)((k_hi - k_lo + 31) >> 5);
  const bool partial = ((k_hi - k_lo) & 31) != 0;

  abf16x8_t qp[KC][3];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = kc * 16 + 8 * h + j;
      v[j] = (q < a.q1 && d < a.dk) ? Qb[q * a.dk + d] * ALOG2E : 0.0f;  // base-2 scores
    }
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), qp[kc][0], qp[kc][1],
            qp[kc][2]);
  }
  f32x16 o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) o[t] = zero16();
  float m = -INFINITY, l = 0.0f;
  const int64_t kps = (int64_t)gridDim.y * N * DKP, hps = (int64_t)gridDim.y * N * DV;
  DmaRows<DKP, PL_PLAIN, NW> kd;
  DmaRows<DV, PL_HSWZ, NW> hd;
  kd.init(a.Kpl + b * N * DKP, kps, wave, lane);
  hd.init(a.Hpl + b * N * DV, hps, wave, lane);
  kd.issue(k_lo, N, Kp_s, wave, lane);
  hd.issue(k_lo, N, Hp_s, wave, lane);
  if (nblk > 1) kd.issue(k_lo + 32, N, Kp_s + KST, wave, lane);
  if (B2 && nblk > 1) hd.issue(k_lo + 32, N, Hp_s + HST, wave, lane);  // the first pair's H and
  if (B2 && nblk > 2) kd.issue(k_lo + 64, N, Kp_s + 2 * KST, wave, lane);  // K(2), before its barrier
  const int trq = (lane & 15) >> 2;
  const int trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  // S^T = K Q^T of the block staged at Kp (base 2)
  auto scores = [&](const uint16_t* Kp) {
    f32x16 sc = zero16();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int off = l32 * DKP + kc * 16 + 8 * h;
      const abf16x8_t k0p = *reinterpret_cast<const abf16x8_t*>(&Kp[off]);
      const abf16x8_t k1p = *reinterpret_cast<const abf16x8_t*>(&Kp[KPL + off]);
      const abf16x8_t k2p = *reinterpret_cast<const abf16x8_t*>(&Kp[2 * KPL + off]);
      MFMA6(sc, k0p, k1p, k2p, qp[kc][0], qp[kc][1], qp[kc][2]);
    }
    return sc;
  };
  // online softmax of one block: updates m, l; P -> planes; returns alpha
  auto softmax = [&](f32x16& sc, abf16x8_t (&pp)[2][3]) {
    float mx = fmaxf(sc[0], sc[1]);
#pragma unroll
    for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, sc[r]), sc[r + 1]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);
    const float alpha = aexp2(m - mn);
    float ps = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sc[r] = aexp2(sc[r] - mn);
      ps += sc[r];
    }
    ps += __shfl_xor(ps, 32);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      asplit8(make_float4(sc[8 * u], sc[8 * u + 1], sc[8 * u + 2], sc[8 * u + 3]),
              make_float4(sc[8 * u + 4], sc[8 * u + 5], sc[8 * u + 6], sc[8 * u + 7]), pp[u][0], pp[u][1],
              pp[u][2]);
    return alpha;
  };
  auto mask = [&](f32x16& sc, int64_t k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (k0 + kappa(r, h) >= k_hi) sc[r] = -INFINITY;
  };
  // O^T += H^T P^T of the block staged at Hp
  auto pv = [&](const uint16_t* Hp, const abf16x8_t (&pp)[2][3]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        abf16x8_t hp[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          typedef __attribute__((address_space(3))) ai16x4_t lds_v4;
          const int key0 = kappa(8 * u + trq, h), key1 = kappa(8 * u + 4 + trq, h);
          const uint16_t* p0 = &Hp[pl * HPL + hswz<DV>(key0, t * 32 + trc)];
          const uint16_t* p1 = &Hp[pl * HPL + hswz<DV>(key1, t * 32 + trc)];
          const ai16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p0);
          const ai16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p1);
          const ai16x8_t v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
          hp[pl] = __builtin_bit_cast(abf16x8_t, v);
        }
        MFMA6(o[t], hp[0], hp[1], hp[2], pp[u][0], pp[u][1], pp[u][2]);
      }
  };
  auto rescale = [&](float alpha) {
    if (__any(alpha != 1.0f)) {  // wave-uniform; x * 1 == x, so skipping is exact
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
    }
  };

  // prologue: block 0's scores and softmax (o is zero: no rescale)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  abf16x8_t pp[2][3];
  {
    f32x16 sc = scores(Kp_s);
    if (nblk == 1 && partial) mask(sc, k_lo);
    softmax(sc, pp);
  }
  float alpha = 1.0f;
  // iteration it: block it's P.H with block it+1's softmax in the same body
  // hs: the H stage (it & 1) as a constant (GRL_ATTN_HU2 unrolls the loop by
  // two): the 8 NT transposed H reads then take it as an immediate offset
  // instead of an address add each; -1 = the stage at run time
  auto iteration = [&](int it, auto masked, auto hs) {
    constexpr bool MASK = decltype(masked)::value;
    constexpr int HS = decltype(hs)::value;
    const int64_t k0 = k_lo + 32 * (int64_t)it;
    if constexpr (B2) {
      // even it: blocks it, it+1's H and K(it+1), K(it+2) landed; every wave is
      // done with blocks it-2, it-1, whose stages the next pair's DMAs take
      if ((HS >= 0 ? HS : it) % 2 == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (it + 2 < nblk) hd.issue(k0 + 64, N, Hp_s + hstage(it + 2) * HST, wave, lane);
        if (it + 3 < nblk) hd.issue(k0 + 96, N, Hp_s + hstage(it + 3) * HST, wave, lane);
        if (it + 3 < nblk) kd.issue(k0 + 96, N, Kp_s + kstage(it + 3) * KST, wave, lane);
        if (it + 4 < nblk) kd.issue(k0 + 128, N, Kp_s + kstage(it + 4) * KST, wave, lane);
      }
    } else {
      // block it's H and block it+1's K landed; every wave is done with the
      // stages the next DMAs overwrite (H of block it-1, K of block it-1)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (it + 1 < nblk) hd.issue(k0 + 32, N, Hp_s + hstage(it + 1) * HST, wave, lane);
      if (it + 2 < nblk) kd.issue(k0 + 64, N, Kp_s + kstage(it + 2) * KST, wave, lane);
    }
    rescale(alpha);
    f32x16 sc = scores(Kp_s + (B2 && HS >= 0 ? (HS + 1) & 3 : kstage(it + 1)) * KST);
    if constexpr (MASK) mask(sc, k0 + 32);
    abf16x8_t pn[2][3];
    // block it's P.H in 2 NT groups of 6 MFMAs; block it+1's softmax cut into
    // 7 pieces placed after groups 1 .. 2 NT - 1 (group 0 covers the score
    // MFMAs' latency), each group fenced so its VALU fills that group's gaps
    const lds_u16* Hp = (const lds_u16*)Hp_s + (HS < 0 ? hstage(it) : HS) * HST;
    float mn = 0.0f, an = 1.0f, ps = 0.0f;
    auto piece = [&](int pc) {
      if (pc == 0) {
        float mx = fmaxf(sc[0], sc[1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) mx = fmaxf(fmaxf(mx, sc[r]), sc[r + 1]);
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        mn = fmaxf(m, mx);
        an = aexp2(m - mn);
      } else if (pc <= 2) {
#pragma unroll
        for (int r = 8 * (pc - 1); r < 8 * pc; ++r) {
          sc[r] = aexp2(sc[r] - mn);
          ps += sc[r];
        }
        if (pc == 2) {
          ps += __shfl_xor(ps, 32);
          l = l * an + ps;
          m = mn;
        }
      } else {
        const int u = (pc - 3) >> 1, half = (pc - 3) & 1;
        if (half == 0) {
          uint2 l0, l1, l2;
          asplit3(make_float4(sc[8 * u], sc[8 * u + 1], sc[8 * u + 2], sc[8 * u + 3]), l0, l1, l2);
          pn[u][0] = __builtin_bit_cast(abf16x8_t, make_uint4(l0.x, l0.y, 0u, 0u));
          pn[u][1] = __builtin_bit_cast(abf16x8_t, make_uint4(l1.x, l1.y, 0u, 0u));
          pn[u][2] = __builtin_bit_cast(abf16x8_t, make_uint4(l2.x, l2.y, 0u, 0u));
        } else {
          uint2 h0, h1, h2;
          asplit3(make_float4(sc[8 * u + 4], sc[8 * u + 5], sc[8 * u + 6], sc[8 * u + 7]), h0, h1, h2);
          uint4 w0 = __builtin_bit_cast(uint4, pn[u][0]), w1 = __builtin_bit_cast(uint4, pn[u][1]),
                w2 = __builtin_bit_cast(uint4, pn[u][2]);
          pn[u][0] = __builtin_bit_cast(abf16x8_t, make_uint4(w0.x, w0.y, h0.x, h0.y));
          pn[u][1] = __builtin_bit_cast(abf16x8_t, make_uint4(w1.x, w1.y, h1.x, h1.y));
          pn[u][2] = __builtin_bit_cast(abf16x8_t, make_uint4(w2.x, w2.y, h2.x, h2.y));
        }
      }
    };
    // group g's H fragments (three planes, transposed reads)
    auto load_h = [&](int g, abf16x8_t (&hp)[3]) {
      const int t = g >> 1, u = g & 1;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        typedef __attribute__((address_space(3))) ai16x4_t lds_v4;
        const int key0 = kappa(8 * u + trq, h), key1 = kappa(8 * u + 4 + trq, h);
        const lds_u16* p0 = Hp + pl * HPL + hswz<DV>(key0, t * 32 + trc);
        const lds_u16* p1 = Hp + pl * HPL + hswz<DV>(key1, t * 32 + trc);
        const ai16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p0);
        const ai16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p1);
        const ai16x8_t v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        hp[pl] = __builtin_bit_cast(abf16x8_t, v);
      }
    };
    // HPF: the next group's fragments are read one group ahead (two register
    // sets): behind the fence each group's reads would otherwise expose the LDS
    // latency (where the registers allow: 12 more VGPRs)
    constexpr bool HPF = GRL_ATTN_HPF && NT <= 4 && (DKP <= 16 || NW == 4);
    abf16x8_t hq[HPF ? 2 : 1][3];
    if constexpr (HPF) load_h(0, hq[0]);
    (void)hq;
#pragma unroll
    for (int g = 0; g < 2 * NT; ++g) {
      const int t = g >> 1, u = g & 1;
      if constexpr (HPF) {
        if (g + 1 < 2 * NT) load_h(g + 1, hq[(g + 1) & 1]);
        MFMA6(o[t], hq[g & 1][0], hq[g & 1][1], hq[g & 1][2], pp[u][0], pp[u][1], pp[u][2]);
      } else {
        abf16x8_t hp[3];
        load_h(g, hp);
        MFMA6(o[t], hp[0], hp[1], hp[2], pp[u][0], pp[u][1], pp[u][2]);
      }
      // pieces assigned to this group: piece pc runs after group 1 + pc * (2 NT - 1) / 7
#pragma unroll
      for (int pc = 0; pc < 7; ++pc)
        if (g >= 1 && 1 + pc * (2 * NT - 1) / 7 == g) piece(pc);
      __builtin_amdgcn_sched_barrier(0);
    }
    alpha = an;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        // keep block it+1's split in this body: unrolled, LLVM would sink it
        // into the next body (where its MFMAs use it), undoing the interleave
        if constexpr (GRL_ATTN_PIN_PN && NT <= 4) asm volatile("" : "+v"(pn[u][pl]));
        pp[u][pl] = pn[u][pl];
      }
  };
  using HRun = std::integral_constant<int, -1>;
  int it = 0;
#if GRL_ATTN_HU2
  // (dv = 256, NT = 8: the unrolled bodies spill -- that form keeps the rolled loop)
  if constexpr (NT > 4) {
  } else if constexpr (B2) {
    for (; it + 5 < nblk; it += 4) {  // it % 4 == 0: H stages 0..3
      iteration(it, std::false_type{}, std::integral_constant<int, 0>{});
      iteration(it + 1, std::false_type{}, std::integral_constant<int, 1>{});
      iteration(it + 2, std::false_type{}, std::integral_constant<int, 2>{});
      iteration(it + 3, std::false_type{}, std::integral_constant<int, 3>{});
    }
  } else {
    for (; it + 3 < nblk; it += 2) {  // it even: H stages 0, 1
      iteration(it, std::false_type{}, std::integral_constant<int, 0>{});
      iteration(it + 1, std::false_type{}, std::integral_constant<int, 1>{});
    }
  }
#endif
  for (; it + 2 < nblk; ++it) iteration(it, std::false_type{}, HRun{});
  if (it + 1 < nblk) {
    if (partial)
      iteration(it, std::true_type{}, HRun{});
    else
      iteration(it, std::false_type{}, HRun{});
    ++it;
  }
  // the last block: its P.H only
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  rescale(alpha);
  pv(Hp_s + hstage(it) * HST, pp);

  if (SPLIT && q < a.q1) {  // key split: unnormalised partials, combined by attn_fwd_combine_kernel
    const int64_t rows = (int64_t)gridDim.y * N, row = b * N + q, zs = blockIdx.z;
    float* po = a.part + zs * rows * a.dv + row * a.dv;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) po[f] = o[t][r];
      }
    if (h == 0) {
      float* pm = a.part + (int64_t)gridDim.z * rows * a.dv;
      pm[zs * rows + row] = m;
      pm[((int64_t)gridDim.z + zs) * rows + row] = l;
    }
  } else if (q < a.q1) {
    const float inv = 1.0f / l;
    const int64_t base = (b * N + q) * a.dv;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int f = t * 32 + kappa(r, h);
        if (f < a.dv) {
          const float on = o[t][r] * inv;
          a.out[base + f] = a.gamma[f] * on + a.V[base + f];
          if (a.onorm) a.onorm[base + f] = on;
        }
      }
    if (h == 0 && a.rmax) {
      a.rmax[b * N + q] = m * ALN2;  // natural-log row max (the saved-stat contract)
      a.rsum[b * N + q] = l;
    }
  }
}

// ---------------------------------------------------------------------------
// Backward on the bf16 matrix cores (x6), for dv in (96, 128] (NT = 4: the
// model's 128-wide values).  Three kernels instead of two: the key-stationary
// work is split into dH (needs P only) and dK (needs dP, so the lane's H row
// in registers) so that neither holds both a 64-register dH accumulator and
// the 96 registers of H's planes.  Each recomputes S (6 MFMAs per block).
// The 128-column planes (H, dO) use the guide's 256-B-row image (b)
// (cdna_hip_programming.md T10): 16-B chunk ch of row r at
// ch ^ (((r & 3) << 2) | ((r >> 2) & 3)), conflict-free for both the
// ds_read_b128 row reads and the ds_read_b64_tr_b16 reads of 4 consecutive
// rows.  The 32-column planes (K, Q; dk padded with zeros) are read
// transposed over 4 consecutive rows of 64 B: conflict-free as they lie.
// tr8 on LDS-space pointers: constant offsets fold into the reads' immediates
__device__ __forceinline__ abf16x8_t tr8s(const lds_u16* p0, const lds_u16* p1) {
  typedef __attribute__((address_space(3))) ai16x4_t lds_v4;
  const ai16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p0);
  const ai16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)p1);
  const ai16x8_t v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(abf16x8_t, v);
}

__device__ __forceinline__ abf16x8_t tr8(const uint16_t* p0, const uint16_t* p1) {
  typedef __attribute__((address_space(3))) ai16x4_t lds_v4;
  const ai16x4_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p0);
  const ai16x4_t x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(uintptr_t)(uint32_t)(uintptr_t)p1);
  const ai16x8_t v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(abf16x8_t, v);
}

// lane's own 8-value slices v[c*16 + 8h + j] of a row, split into planes
template <int NC>
__device__ __forceinline__ void row_planes(const float* row, bool valid, int width, int h, abf16x8_t (&pl)[NC][3],
                                           float scale = 1.0f) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = c * 16 + 8 * h + j;
      v[j] = (valid && d < width) ? row[d] * scale : 0.0f;
    }
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), pl[c][0], pl[c][1], pl[c][2]);
  }
}

// 16 fp32 registers (keys / queries kappa(r, h)) -> the two B operands u = 0, 1
__device__ __forceinline__ void reg_planes(const f32x16& x, abf16x8_t (&pl)[2][3]) {
#pragma unroll
  for (int u = 0; u < 2; ++u)
    asplit8(make_float4(x[8 * u], x[8 * u + 1], x[8 * u + 2], x[8 * u + 3]),
            make_float4(x[8 * u + 4], x[8 * u + 5], x[8 * u + 6], x[8 * u + 7]), pl[u][0], pl[u][1], pl[u][2]);
}

// query-stationary: dQ^T += K^T dS^T
template <int DKP, bool PRE, bool SPLIT>
__global__ __launch_bounds__(256, 2) void attn_bwd_q_x6_kernel(AttnArgs a) {
  constexpr int KC = DKP / 16, FC = 8;  // 128 value columns = 8 chunks of 16
  __shared__ __attribute__((aligned(16))) uint16_t Kp_s[(PRE ? 2 : 1) * 3 * 32 * 32];  // PRE: 2 stages
  __shared__ __attribute__((aligned(16))) uint16_t Hp_s[(PRE ? 2 : 1) * 3 * 32 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Kb = a.K + b * N * a.dk;
  const float* Hb = a.H + b * N * a.dv;
  const int64_t q = a.q0 + (int64_t)blockIdx.x * 128 + wave * 32 + l32;
  const bool qv = q < a.q1;
  const int64_t k_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : 0, k_hi = SPLIT ? min<int64_t>(N, k_lo + a.kr) : N;
  abf16x8_t qp[KC][3], dop[FC][3];
  row_planes<KC>(a.Q + (b * N + q) * a.dk, qv, a.dk, h, qp, ALOG2E);  // base-2 scores
  row_planes<FC>(a.dO + (b * N + q) * a.dv, qv, a.dv, h, dop);
  // p = 2^(s - lse2); a padded query gets lse2 = +inf, so p = 0
  const float lse2 = qv ? fmaf(a.smax[b * N + q], ALOG2E, alog2(a.ssum[b * N + q])) : INFINITY;
  const float Dq = qv ? a.Drow[b * N + q] : 0.0f;
  f32x16 dq = zero16();
  if (!PRE && DKP < 32)  // zero pad columns of the K planes, never written by the staging
    for (int i = tid; i < 3 * 32 * (32 - DKP); i += 256) {
      const int pl = i / (32 * (32 - DKP)), rc = i % (32 * (32 - DKP));
      Kp_s[pl * 1024 + (rc / (32 - DKP)) * 32 + DKP + rc % (32 - DKP)] = 0;
    }
  XStage<DKP, 32, PL_PLAIN> sk;
  XStage<128, 128, PL_SWZ128> sh;
  // PRE planes: K split 32 wide (zero columns >= dk), H 128 wide
  const int64_t kps = (int64_t)gridDim.y * N * 32, hps = (int64_t)gridDim.y * N * 128;
  const uint16_t* Kpb = a.Kpl + b * N * 32;
  const uint16_t* Hpb = a.Hpl + b * N * 128;
  const bool vk = vec_ok(Kb, a.dk), vh = vec_ok(Hb, a.dv);
  if constexpr (PRE) {
    dma_block<32, PL_PLAIN>(Kpb, kps, k_lo, N, Kp_s, wave, lane);
    dma_block<128, PL_SWZ128>(Hpb, hps, k_lo, N, Hp_s, wave, lane);
  } else {
    sk.fetch(Kb, k_lo, N, a.dk, vk, tid);
    sh.fetch(Hb, k_lo, N, a.dv, vh, tid);
  }
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  for (int64_t k0 = k_lo; k0 < k_hi; k0 += 32) {
    const int stg = PRE ? (int)(((k0 - k_lo) >> 5) & 1) : 0;
    uint16_t* Kp = Kp_s + stg * 3 * 1024;
    uint16_t* Hp = Hp_s + stg * 3 * 4096;
    if constexpr (PRE) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (k0 + 32 < k_hi) {
        dma_block<32, PL_PLAIN>(Kpb, kps, k0 + 32, N, Kp_s + (stg ^ 1) * 3 * 1024, wave, lane);
        dma_block<128, PL_SWZ128>(Hpb, hps, k0 + 32, N, Hp_s + (stg ^ 1) * 3 * 4096, wave, lane);
      }
    } else {
      sk.store(Kp, tid);
      sh.store(Hp, tid);
      __syncthreads();
      if (k0 + 32 < k_hi) {
        sk.fetch(Kb, k0 + 32, N, a.dk, vk, tid);
        sh.fetch(Hb, k0 + 32, N, a.dv, vh, tid);
      }
    }
    const int l32o = l32, trqo = trq, trco = trc;
    f32x16 s = zero16();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int off = l32o * 32 + kc * 16 + 8 * h;
      const abf16x8_t k0p = *reinterpret_cast<const abf16x8_t*>(&Kp[off]);
      const abf16x8_t k1p = *reinterpret_cast<const abf16x8_t*>(&Kp[1024 + off]);
      const abf16x8_t k2p = *reinterpret_cast<const abf16x8_t*>(&Kp[2048 + off]);
      MFMA6(s, k0p, k1p, k2p, qp[kc][0], qp[kc][1], qp[kc][2]);
    }
    f32x16 dp = zero16();  // dP^T[key][query] = sum_f H[key][f] dO[query][f]
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) {
      const int off = swz128(l32o, fc * 16 + 8 * h);
      const abf16x8_t h0 = *reinterpret_cast<const abf16x8_t*>(&Hp[off]);
      const abf16x8_t h1 = *reinterpret_cast<const abf16x8_t*>(&Hp[4096 + off]);
      const abf16x8_t h2 = *reinterpret_cast<const abf16x8_t*>(&Hp[8192 + off]);
      MFMA6(dp, h0, h1, h2, dop[fc][0], dop[fc][1], dop[fc][2]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = aexp2(s[r] - lse2) * (dp[r] - Dq);  // dS^T = P (dP - D)
    if (k0 + 32 > k_hi) {  // the last, partial key block only (wave-uniform)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (k0 + kappa(r, h) >= k_hi) s[r] = 0.0f;
    }
    abf16x8_t dsp[2][3];
    reg_planes(s, dsp);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r0 = kappa(8 * u + trqo, h), r1 = kappa(8 * u + 4 + trqo, h);
      abf16x8_t kt[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) kt[pl] = tr8(&Kp[pl * 1024 + r0 * 32 + trco], &Kp[pl * 1024 + r1 * 32 + trco]);
      MFMA6(dq, kt[0], kt[1], kt[2], dsp[u][0], dsp[u][1], dsp[u][2]);
    }
    if constexpr (!PRE) __syncthreads();
  }
  if (qv) {  // key split: partial dQ into slab blockIdx.z (summed in split order afterwards)
    float* dst = SPLIT ? a.part + (int64_t)blockIdx.z * gridDim.y * N * a.dk : a.dQ;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = kappa(r, h);
      if (d < a.dk) dst[(b * N + q) * a.dk + d] = dq[r];
    }
  }
}

// key-stationary.  WANT_H: dH^T += dO^T P;  else dK^T += Q^T dS (needs dP)
// NW = 8 (PRE only): 256 keys per workgroup, one per CU -- the query block's
// Q / dO stage serves twice the keys (half the LDS-DMA per key)
template <int DKP, bool WANT_H, bool PRE, bool SPLIT, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_kv_x6_kernel(AttnArgs a) {
  static_assert(NW == 4 || (NW == 8 && PRE), "8-wave workgroups stage by LDS-DMA only");
  constexpr int KC = DKP / 16, FC = 8;
  __shared__ __attribute__((aligned(16))) uint16_t Qp_s[(PRE ? 2 : 1) * 3 * 32 * 32];  // PRE: 2 stages
  __shared__ __attribute__((aligned(16))) uint16_t Op_s[(PRE ? 2 : 1) * 3 * 32 * 128];
  __shared__ float Ms_s[(PRE ? 2 : 1) * 32], Ds_s[(PRE ? 2 : 1) * 32];  // lse2, D per query
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const float* Qb = a.Q + b * N * a.dk;
  const float* dOb = a.dO + b * N * a.dv;
  const int64_t key = (int64_t)blockIdx.x * (32 * NW) + wave * 32 + l32;
  const bool kv = key < N;
  const int64_t q_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : a.q0, q_hi = SPLIT ? min<int64_t>(N, q_lo + a.kr) : a.q1;
  abf16x8_t kp[KC][3];
  row_planes<KC>(a.K + (b * N + key) * a.dk, kv, a.dk, h, kp, ALOG2E);  // base-2 scores
  abf16x8_t hp[WANT_H ? 1 : FC][3];
  if (!WANT_H) row_planes<WANT_H ? 1 : FC>(a.H + (b * N + key) * a.dv, kv, a.dv, h, hp);
  f32x16 acc[WANT_H ? 4 : 1];
#pragma unroll
  for (int t = 0; t < (WANT_H ? 4 : 1); ++t) acc[t] = zero16();
  if (!PRE && DKP < 32)
    for (int i = tid; i < 3 * 32 * (32 - DKP); i += 256) {
      const int pl = i / (32 * (32 - DKP)), rc = i % (32 * (32 - DKP));
      Qp_s[pl * 1024 + (rc / (32 - DKP)) * 32 + DKP + rc % (32 - DKP)] = 0;
    }
  XStage<DKP, 32, PL_PLAIN> sq;
  XStage<128, 128, PL_SWZ128> so;
  const int64_t qps = (int64_t)gridDim.y * N * 32, ops = (int64_t)gridDim.y * N * 128;
  const uint16_t* Qpb = a.Qpl + b * N * 32;
  const uint16_t* Opb = a.Opl + b * N * 128;
  const bool vq = vec_ok(Qb, a.dk), vo = vec_ok(dOb, a.dv);
  float pm = 0.0f, pd = 0.0f;
  auto fetch_stats = [&](int64_t q0) {
    if (tid < 32) {
      const int64_t qq = q0 + tid;
      const bool v = qq < q_hi;
      // lse2 = +inf => P = 0 for padded queries
      pm = v ? fmaf(a.smax[b * N + qq], ALOG2E, alog2(a.ssum[b * N + qq])) : INFINITY;
      pd = v ? a.Drow[b * N + qq] : 0.0f;
    }
  };
  // dH (WANT_H) has the VGPR room for precomputed DMA addresses; dK does not
  DmaRows<32, PL_PLAIN, NW> qd;
  DmaRows<128, PL_SWZ128, NW> od;
  if constexpr (PRE && WANT_H) {
    qd.init(Qpb, qps, wave, lane);
    od.init(Opb, ops, wave, lane);
    qd.issue(q_lo, N, Qp_s, wave, lane);
    od.issue(q_lo, N, Op_s, wave, lane);
  } else if constexpr (PRE) {
    dma_block<32, PL_PLAIN, NW>(Qpb, qps, q_lo, N, Qp_s, wave, lane);
    dma_block<128, PL_SWZ128, NW>(Opb, ops, q_lo, N, Op_s, wave, lane);
  } else {
    sq.fetch(Qb, q_lo, N, a.dk, vq, tid);
    so.fetch(dOb, q_lo, N, a.dv, vo, tid);
  }
  fetch_stats(q_lo);
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  // one query block; stc: its stage as a constant (the PRE dH loop unrolled
  // by two under GRL_ATTN_HU2: transposed reads at immediate LDS offsets), -1 = at run time
  auto block = [&](int64_t q0, auto stc) {
    constexpr int SC = decltype(stc)::value;
    const int stg = SC >= 0 ? SC : (PRE ? (int)(((q0 - q_lo) >> 5) & 1) : 0);
    uint16_t* Qp = Qp_s + stg * 3 * 1024;
    uint16_t* Op = Op_s + stg * 3 * 4096;
    const lds_u16* Qp3 = (const lds_u16*)Qp_s + stg * 3 * 1024;
    const lds_u16* Op3 = (const lds_u16*)Op_s + stg * 3 * 4096;
    float* Ms = Ms_s + stg * 32;
    float* Ds = Ds_s + stg * 32;
    if (!PRE) {
      sq.store(Qp, tid);
      so.store(Op, tid);
    }
    if (tid < 32) {
      Ms[tid] = pm;
      Ds[tid] = pd;
    }
    if constexpr (PRE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (q0 + 32 < q_hi) {
      if constexpr (PRE && WANT_H) {
        qd.issue(q0 + 32, N, Qp_s + (stg ^ 1) * 3 * 1024, wave, lane);
        od.issue(q0 + 32, N, Op_s + (stg ^ 1) * 3 * 4096, wave, lane);
      } else if constexpr (PRE) {
        dma_block<32, PL_PLAIN, NW>(Qpb, qps, q0 + 32, N, Qp_s + (stg ^ 1) * 3 * 1024, wave, lane);
        dma_block<128, PL_SWZ128, NW>(Opb, ops, q0 + 32, N, Op_s + (stg ^ 1) * 3 * 4096, wave, lane);
      } else {
        sq.fetch(Qb, q0 + 32, N, a.dk, vq, tid);
        so.fetch(dOb, q0 + 32, N, a.dv, vo, tid);
      }
      fetch_stats(q0 + 32);
    }
    // S[query][key]: lanes = keys, registers = queries kappa(r, h)
    f32x16 s = zero16();
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int off = l32 * 32 + kc * 16 + 8 * h;
      const abf16x8_t q0p = *reinterpret_cast<const abf16x8_t*>(&Qp[off]);
      const abf16x8_t q1p = *reinterpret_cast<const abf16x8_t*>(&Qp[1024 + off]);
      const abf16x8_t q2p = *reinterpret_cast<const abf16x8_t*>(&Qp[2048 + off]);
      MFMA6(s, q0p, q1p, q2p, kp[kc][0], kp[kc][1], kp[kc][2]);
    }
    if (WANT_H) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = kappa(r, h);
        s[r] = aexp2(s[r] - Ms[qi]);  // P (a padded key's column is never stored)
      }
      abf16x8_t pp[2][3];
      reg_planes(s, pp);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int r0 = kappa(8 * u + trq, h), r1 = kappa(8 * u + 4 + trq, h);
          abf16x8_t ot[3];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            ot[pl] = tr8s(Op3 + pl * 4096 + swz128(r0, t * 32 + trc), Op3 + pl * 4096 + swz128(r1, t * 32 + trc));
          MFMA6(acc[t], ot[0], ot[1], ot[2], pp[u][0], pp[u][1], pp[u][2]);
        }
    } else {
      f32x16 dp = zero16();  // dP[query][key] = sum_f dO[query][f] H[key][f]
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const int off = swz128(l32, fc * 16 + 8 * h);
        const abf16x8_t o0 = *reinterpret_cast<const abf16x8_t*>(&Op[off]);
        const abf16x8_t o1 = *reinterpret_cast<const abf16x8_t*>(&Op[4096 + off]);
        const abf16x8_t o2 = *reinterpret_cast<const abf16x8_t*>(&Op[8192 + off]);
        MFMA6(dp, o0, o1, o2, hp[fc][0], hp[fc][1], hp[fc][2]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = kappa(r, h);
        s[r] = aexp2(s[r] - Ms[qi]) * (dp[r] - Ds[qi]);  // dS (a padded key's column is never stored)
      }
      abf16x8_t dsp[2][3];
      reg_planes(s, dsp);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r0 = kappa(8 * u + trq, h), r1 = kappa(8 * u + 4 + trq, h);
        abf16x8_t qt[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) qt[pl] = tr8s(Qp3 + pl * 1024 + r0 * 32 + trc, Qp3 + pl * 1024 + r1 * 32 + trc);
        MFMA6(acc[0], qt[0], qt[1], qt[2], dsp[u][0], dsp[u][1], dsp[u][2]);
      }
    }
    if constexpr (!PRE) __syncthreads();
    };
#if GRL_ATTN_HU2
  if constexpr (PRE && WANT_H) {  // (the dK form has no VGPRs left for the unrolled pair)
    int64_t q0 = q_lo;
    for (; q0 + 32 < q_hi; q0 += 64) {
      block(q0, std::integral_constant<int, 0>{});
      block(q0 + 32, std::integral_constant<int, 1>{});
    }
    if (q0 < q_hi) block(q0, std::integral_constant<int, 0>{});
  } else
#endif
  {
    for (int64_t q0 = q_lo; q0 < q_hi; q0 += 32) block(q0, std::integral_constant<int, -1>{});
  }
  if (kv) {  // query split: partial dH / dK into slab blockIdx.z (summed in split order afterwards)
    const int64_t rows = (int64_t)gridDim.y * N;
    if (WANT_H) {
      float* dst = SPLIT ? a.part + (int64_t)blockIdx.z * rows * a.dv : a.dH;
      const int64_t rowv = (b * N + key) * a.dv;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int f = t * 32 + kappa(r, h);
          if (f < a.dv) dst[rowv + f] = acc[t][r];
        }
    } else {
      float* dst = SPLIT ? a.part2 + (int64_t)blockIdx.z * rows * a.dk : a.dK;
      const int64_t rowk = (b * N + key) * a.dk;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = kappa(r, h);
        if (d < a.dk) dst[rowk + d] = acc[0][r];
      }
    }
  }
}


// ---------------------------------------------------------------------------
// dH on v_mfma_f32_16x16x32_bf16 (dk <= 16, PRE staging, 8 waves of 32 keys):
// the work of attn_bwd_kv_x6_kernel<16, true, true, *, 8> in 16 x 16 tiles.
//  * S = Q K^T, 4 tiles (2 query x 2 key) of 3 MFMAs: the six x6 products of
//    the dk = 16 contraction paired along K = 32 -- lanes 0..31 carry the
//    first product's 16 k, lanes 32..63 the second's: [Q_hi | Q_hi] [K_hi |
//    K_mid], [Q_mid | Q_lo] [K_hi | K_hi], [Q_mid | Q_hi] [K_mid | K_lo].
//    The keys' planes (B) are split once into registers; the query rows (A)
//    come from the staged Q planes, row c of query tile t being query
//    8 (c >> 2) + 4 t + (c & 3), so that the tile rows a lane group g holds
//    after the MFMA are queries 8 g .. 8 g + 7 -- its K slice of the P.dO
//    product, in natural order;
//  * P = 2^(s - lse2) (8 distinct queries per lane), split into planes, is
//    the B operand of dH^T += dO^T P as it lies; dO^T's fragments are two
//    ds_read_b64_tr_b16 per plane (rows 8 g .. 8 g + 3 and 8 g + 4 ..
//    8 g + 7: the two 16-lane groups of a half read blocks 8 rows apart, the
//    conflict-free case of the swizzled 256-B rows);
//  * 16 f32x4 accumulators (8 feature x 2 key tiles), x6 product order.
// The same products as the 32x32x16 kernel with the two plane products of
// S summed inside one MFMA: results equal within fp32 rounding (tested vs
// float64).  Staging, stats and the query split are the 32x32x16 kernel's.
typedef float af32x4_t __attribute__((ext_vector_type(4)));
#define MFMA16(acc, a, b) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (acc), 0, 0, 0)
template <bool SPLIT>
__global__ __launch_bounds__(512, 1) void attn_bwd_h16_kernel(AttnArgs a) {
  constexpr int NW = 8, FT = 8;  // 128 value columns = 8 tiles of 16
  __shared__ __attribute__((aligned(16))) uint16_t Qp_s[2 * 3 * 32 * 32];
  __shared__ __attribute__((aligned(16))) uint16_t Op_s[2 * 3 * 32 * 128];
  __shared__ __attribute__((aligned(16))) float Ms_s[2 * 32];  // lse2 per query
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int64_t N = a.N, b = blockIdx.y;
  const int64_t key0 = (int64_t)blockIdx.x * (32 * NW) + wave * 32;  // this wave's 32 keys
  const int64_t q_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : a.q0, q_hi = SPLIT ? min<int64_t>(N, q_lo + a.kr) : a.q1;
  // B operands of S: key 16 kt + c16, k = 8 (g & 1) .. + 7, plane by MFMA m and lane half
  abf16x8_t kb[2][3];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int64_t key = key0 + 16 * kt + c16;
    const bool kv = key < N;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * (g & 1) + j;
      v[j] = (kv && d < a.dk) ? a.K[(b * N + key) * a.dk + d] * ALOG2E : 0.0f;  // base-2 scores
    }
    abf16x8_t p0, p1, p2;
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), p0, p1, p2);
    kb[kt][0] = g < 2 ? p0 : p1;  // [K_hi | K_mid]
    kb[kt][1] = p0;               // [K_hi | K_hi]
    kb[kt][2] = g < 2 ? p1 : p2;  // [K_mid | K_lo]
  }
  af32x4_t acc[FT][2];
#pragma unroll
  for (int ft = 0; ft < FT; ++ft)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) acc[ft][kt] = af32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t qps = (int64_t)gridDim.y * N * 32, ops = (int64_t)gridDim.y * N * 128;
  DmaRows<32, PL_PLAIN, NW> qd;
  DmaRows<128, PL_SWZ128, NW> od;
  qd.init(a.Qpl + b * N * 32, qps, wave, lane);
  od.init(a.Opl + b * N * 128, ops, wave, lane);
  qd.issue(q_lo, N, Qp_s, wave, lane);
  od.issue(q_lo, N, Op_s, wave, lane);
  float pm = 0.0f;
  auto fetch_stats = [&](int64_t q0) {
    if (tid < 32) {
      const int64_t qq = q0 + tid;
      // lse2 = +inf => P = 0 for padded queries
      pm = qq < q_hi ? fmaf(a.smax[b * N + qq], ALOG2E, alog2(a.ssum[b * N + qq])) : INFINITY;
    }
  };
  fetch_stats(q_lo);
  // A-operand planes of S per MFMA m for this lane's half: [hi | hi], [mid | lo], [mid | hi]
  const int qa0 = 0, qa1 = g < 2 ? 1 : 2, qa2 = g < 2 ? 1 : 0;
  const int qrow0 = 8 * (c16 >> 2) + (c16 & 3);  // query tile 0's row; tile 1: + 4
  const int qcol = 8 * (g & 1);
  const int q4 = c16 >> 2, p4 = c16 & 3;  // transposed reads: row q4 of a 4-row block, 8-B piece p4

  auto block = [&](int64_t q0, auto stc) {
    constexpr int SC = decltype(stc)::value;
    const int stg = SC >= 0 ? SC : (int)(((q0 - q_lo) >> 5) & 1);
    const lds_u16* Op3 = (const lds_u16*)Op_s + stg * 3 * 4096;
    float* Ms = Ms_s + stg * 32;
    if (tid < 32) Ms[tid] = pm;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (q0 + 32 < q_hi) {
      qd.issue(q0 + 32, N, Qp_s + (stg ^ 1) * 3 * 1024, wave, lane);
      od.issue(q0 + 32, N, Op_s + (stg ^ 1) * 3 * 4096, wave, lane);
      fetch_stats(q0 + 32);
    }
    // S tiles [qt][kt]: rows (queries 8 g + 4 qt + i) in registers, keys 16 kt + c16 on lanes
    af32x4_t st[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const uint16_t* qr = Qp_s + stg * 3 * 1024 + (qrow0 + 4 * qt) * 32 + qcol;
      abf16x8_t qa[3];
      qa[0] = *reinterpret_cast<const abf16x8_t*>(qr + qa0 * 1024);
      qa[1] = *reinterpret_cast<const abf16x8_t*>(qr + qa1 * 1024);
      qa[2] = *reinterpret_cast<const abf16x8_t*>(qr + qa2 * 1024);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        af32x4_t sacc = {0.0f, 0.0f, 0.0f, 0.0f};  // small products first, hi.hi last: one rounding at |s|
        MFMA16(sacc, qa[2], kb[kt][2]);
        MFMA16(sacc, qa[1], kb[kt][1]);
        MFMA16(sacc, qa[0], kb[kt][0]);
        st[qt][kt] = sacc;
      }
    }
    // P = 2^(s - lse2) for queries 8 g .. 8 g + 7 (a padded key's column is never stored)
    const float4 m0 = *reinterpret_cast<const float4*>(Ms + 8 * g);
    const float4 m1 = *reinterpret_cast<const float4*>(Ms + 8 * g + 4);
    abf16x8_t pb[2][3];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const float4 lo = make_float4(aexp2(st[0][kt][0] - m0.x), aexp2(st[0][kt][1] - m0.y),
                                    aexp2(st[0][kt][2] - m0.z), aexp2(st[0][kt][3] - m0.w));
      const float4 hi = make_float4(aexp2(st[1][kt][0] - m1.x), aexp2(st[1][kt][1] - m1.y),
                                    aexp2(st[1][kt][2] - m1.z), aexp2(st[1][kt][3] - m1.w));
      asplit8(lo, hi, pb[kt][0], pb[kt][1], pb[kt][2]);
    }
    // dH^T[feature][key] += dO^T[feature][query] P[query][key]
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      abf16x8_t oa[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        oa[pl] = tr8s(Op3 + pl * 4096 + swz128(8 * g + q4, 16 * ft + 4 * p4),
                      Op3 + pl * 4096 + swz128(8 * g + 4 + q4, 16 * ft + 4 * p4));
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {  // gemm_x6_kernel's product order
        MFMA16(acc[ft][kt], oa[2], pb[kt][0]);
        MFMA16(acc[ft][kt], oa[1], pb[kt][1]);
        MFMA16(acc[ft][kt], oa[0], pb[kt][2]);
        MFMA16(acc[ft][kt], oa[1], pb[kt][0]);
        MFMA16(acc[ft][kt], oa[0], pb[kt][1]);
        MFMA16(acc[ft][kt], oa[0], pb[kt][0]);
      }
    }
  };
  int64_t q0 = q_lo;
  for (; q0 + 32 < q_hi; q0 += 64) {
    block(q0, std::integral_constant<int, 0>{});
    block(q0 + 32, std::integral_constant<int, 1>{});
  }
  if (q0 < q_hi) block(q0, std::integral_constant<int, 0>{});
  // query split: partial dH into slab blockIdx.z (summed in split order afterwards)
  const int64_t rows = (int64_t)gridDim.y * N;
  float* dst = SPLIT ? a.part + (int64_t)blockIdx.z * rows * a.dv : a.dH;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int64_t key = key0 + 16 * kt + c16;
    if (key >= N) continue;
    float* row = dst + (b * N + key) * a.dv;
#pragma unroll
    for (int ft = 0; ft < FT; ++ft) {
      const int f = 16 * ft + 4 * g;
      if (f + 3 < a.dv) {
        *reinterpret_cast<float4*>(row + f) = make_float4(acc[ft][kt][0], acc[ft][kt][1], acc[ft][kt][2], acc[ft][kt][3]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (f + i < a.dv) row[f + i] = acc[ft][kt][i];
      }
    }
  }
}
#undef MFMA16

// Key-stationary dK with dQ folded in (dk <= 16, PRE staging): what the
// query-stationary attn_bwd_q_x6_kernel computes, without recomputing S and
// dP = dO H^T for it -- 66 MFMAs per 32 x 32 block pair there, 18 more here.
// 8 waves (256 keys) per workgroup, one workgroup per CU: the query block's
// Q / dO stage is shared by twice the keys, and the LDS holds the partials
// of two blocks.  Per query block, after the dK kernel's work:
//  - dS (keys on lanes, queries in registers) is transposed EXACTLY by MFMAs
//    against a 0/1 permutation operand: D[key][q] = sum over the 3 planes of
//    dS's split, one nonzero product per element and plane, and hi + mid + lo
//    is exact in fp32; so D's registers hold keys and its lanes queries;
//  - dQ_blk[q][d] = D^T K over the wave's 32 keys: A = D's planes, B = the
//    wave's K rows (natural scale, planes in LDS, read transposed like Q^T
//    for dK; lanes 16..31 read columns 0..15 again, their outputs dropped);
//  - every wave parks its partial in the block's LDS slot (block parity);
//    after the NEXT block's barrier wave w adds queries [4w, 4w + 4) of the
//    eight in wave order and writes them to this workgroup's slab,
//    qslab[b][blockIdx.x][d][npad] -- no barrier of its own (the slot is
//    rewritten two blocks later, behind another barrier).
// attn_qslab_sum_kernel then adds the slabs in workgroup order: dQ is
// deterministic.  The scores are natural-scale here (K is shared with dQ)
// and p = 2^(fma(s, log2 e, -lse2)): the same instruction count as the
// base-2 kernels' v_sub.  Q comes as 16-wide planes.
#ifndef GRL_ATTN_TPLANES
#define GRL_ATTN_TPLANES 1
#endif
constexpr int KQ_WAVES = 8, KQ_KEYS = 32 * KQ_WAVES;
template <bool SPLIT>
__global__ __launch_bounds__(64 * KQ_WAVES, 1) void attn_bwd_kq_x6_kernel(AttnArgs a) {
  constexpr int FC = 8, NW = KQ_WAVES, KW = KQ_KEYS;
  constexpr int RP = 36;  // partial row pitch in floats: d-major rows, conflict-free reads of 4 queries x 16 d
  constexpr int RSLOT = NW * 16 * RP;
  __shared__ __attribute__((aligned(16))) uint16_t Qp_s[2 * 3 * 32 * 16];  // 2 stages, 16-wide planes
  __shared__ __attribute__((aligned(16))) uint16_t Op_s[2 * 3 * 32 * 128];
  __shared__ __attribute__((aligned(16))) uint16_t Kt_s[3 * KW * 16];  // this workgroup's K rows, planes [key][16]
  __shared__ __attribute__((aligned(16))) float Red_s[2 * RSLOT];      // 2 slots x the waves' partials [w][d][RP]
  __shared__ float Ms_s[2 * 32], Ds_s[2 * 32];                         // lse2, D per query
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int64_t N = a.N, b = blockIdx.y;
  const int64_t key = a.k0 + (int64_t)blockIdx.x * KW + wave * 32 + l32;
  const bool kv = key < N;
  const int64_t q_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : a.q0, q_hi = SPLIT ? min<int64_t>(N, q_lo + a.kr) : a.q1;
  abf16x8_t hp[FC][3];
  row_planes<FC>(a.H + (b * N + key) * a.dv, kv, a.dv, h, hp);
  {  // K rows, natural scale (the scores' B operand, and dQ's; zero for padded keys)
    abf16x8_t kt[1][3];
    row_planes<1>(a.K + (b * N + key) * a.dk, kv, a.dk, h, kt);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      *reinterpret_cast<abf16x8_t*>(&Kt_s[pl * KW * 16 + (wave * 32 + l32) * 16 + 8 * h]) = kt[0][pl];
  }
  // permutation operand of MFMA u: B[k = 8h + j][n] = 1 iff query kappa(8u + j, h) == n (n = l32),
  // i.e. u == n >> 4 and, in half h == (n >> 2) & 1, slot j == 4 ((n >> 3) & 1) + (n & 3)
  const int perm_u = l32 >> 4;
  ai16x8_t onehot;
  {
    const int jj = 4 * ((l32 >> 3) & 1) + (l32 & 3);
    const bool mine = h == ((l32 >> 2) & 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) onehot[j] = (mine && j == jj) ? (short)0x3F80 : (short)0;
  }
  f32x16 acc = zero16();
  const int64_t qps = (int64_t)gridDim.y * N * 16, ops = (int64_t)gridDim.y * N * 128;
  const uint16_t* Qpb = a.Qpl16 + b * N * 16;
  const uint16_t* Opb = a.Opl + b * N * 128;
  const int64_t npad = (N + 31) & ~(int64_t)31;  // slab rows padded to whole query blocks
  float* slab = a.qslab + ((int64_t)b * gridDim.x + blockIdx.x) * 16 * npad;  // [d][npad]
  float pm = 0.0f, pd = 0.0f;
  auto fetch_stats = [&](int64_t q0) {
    if (tid < 32) {
      const int64_t qq = q0 + tid;
      const bool v = qq < q_hi;
      pm = v ? fmaf(a.smax[b * N + qq], ALOG2E, alog2(a.ssum[b * N + qq])) : INFINITY;  // P = 0 when padded
      pd = v ? a.Drow[b * N + qq] : 0.0f;
    }
  };
  // block qb's eight partials (its slot, visible behind a barrier): wave w adds queries
  // [4w, 4w + 4) x 16 d in wave order.  Split ranges are whole query blocks, so a block
  // never reaches into another split's rows; past N it writes the padding (zeros: P = 0).
  auto reduce = [&](int64_t qb) {
    const float* src = Red_s + (int)(((qb - q_lo) >> 5) & 1) * RSLOT;
    const int q = 4 * wave + (lane >> 4), d = lane & 15;
    float x = src[d * RP + q];
#pragma unroll
    for (int w = 1; w < NW; ++w) x += src[w * 16 * RP + d * RP + q];
    slab[d * npad + qb + q] = x;
  };
  dma_block<16, PL_PLAIN, NW>(Qpb, qps, q_lo, N, Qp_s, wave, lane);
  dma_block<128, PL_SWZ128, NW>(Opb, ops, q_lo, N, Op_s, wave, lane);
  fetch_stats(q_lo);
  const int trq = (lane & 15) >> 2, trc = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);

  for (int64_t q0 = q_lo; q0 < q_hi; q0 += 32) {
    const int stg = (int)(((q0 - q_lo) >> 5) & 1);
    uint16_t* Qp = Qp_s + stg * 3 * 512;
    uint16_t* Op = Op_s + stg * 3 * 4096;
    float* Ms = Ms_s + stg * 32;
    float* Ds = Ds_s + stg * 32;
    if (tid < 32) {
      Ms[tid] = pm;
      Ds[tid] = pd;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (q0 + 32 < q_hi) {
      dma_block<16, PL_PLAIN, NW>(Qpb, qps, q0 + 32, N, Qp_s + (stg ^ 1) * 3 * 512, wave, lane);
      dma_block<128, PL_SWZ128, NW>(Opb, ops, q0 + 32, N, Op_s + (stg ^ 1) * 3 * 4096, wave, lane);
      fetch_stats(q0 + 32);
    }
    if (q0 > q_lo) reduce(q0 - 32);
    // S[query][key]: lanes = keys, registers = queries kappa(r, h)
    f32x16 s = zero16();  // natural-scale scores q.k (base 2 applied in the exponent's fma)
    {
      const int off = l32 * 16 + 8 * h, koff = (wave * 32 + l32) * 16 + 8 * h;
      const abf16x8_t q0p = *reinterpret_cast<const abf16x8_t*>(&Qp[off]);
      const abf16x8_t q1p = *reinterpret_cast<const abf16x8_t*>(&Qp[512 + off]);
      const abf16x8_t q2p = *reinterpret_cast<const abf16x8_t*>(&Qp[1024 + off]);
      const abf16x8_t k0p = *reinterpret_cast<const abf16x8_t*>(&Kt_s[koff]);
      const abf16x8_t k1p = *reinterpret_cast<const abf16x8_t*>(&Kt_s[KW * 16 + koff]);
      const abf16x8_t k2p = *reinterpret_cast<const abf16x8_t*>(&Kt_s[2 * KW * 16 + koff]);
      MFMA6(s, q0p, q1p, q2p, k0p, k1p, k2p);
    }
    f32x16 dp = zero16();  // dP[query][key] = sum_f dO[query][f] H[key][f]
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) {
      const int off = swz128(l32, fc * 16 + 8 * h);
      const abf16x8_t o0 = *reinterpret_cast<const abf16x8_t*>(&Op[off]);
      const abf16x8_t o1 = *reinterpret_cast<const abf16x8_t*>(&Op[4096 + off]);
      const abf16x8_t o2 = *reinterpret_cast<const abf16x8_t*>(&Op[8192 + off]);
      MFMA6(dp, o0, o1, o2, hp[fc][0], hp[fc][1], hp[fc][2]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = kappa(r, h);
      s[r] = aexp2(fmaf(s[r], ALOG2E, -Ms[qi])) * (dp[r] - Ds[qi]);  // dS
    }
    abf16x8_t dsp[2][3];
    reg_planes(s, dsp);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r0 = kappa(8 * u + trq, h), r1 = kappa(8 * u + 4 + trq, h);
      abf16x8_t qt[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        qt[pl] = tr8(&Qp[pl * 512 + r0 * 16 + (trc & 15)], &Qp[pl * 512 + r1 * 16 + (trc & 15)]);
      MFMA6(acc, qt[0], qt[1], qt[2], dsp[u][0], dsp[u][1], dsp[u][2]);  // dK^T += Q^T dS
    }
    // dS transposed (lanes = queries, registers = keys kappa(r, h)) PLANE BY PLANE:
    // each transposed element is one plane value times 1 plus zeros, so it is
    // that bf16 value exactly and packs back without a split: dQ's A operand
    // is dS's own three planes (the ones dK used).  The previous form summed
    // the planes in fp32 and split the sum again -- 48 more VALU per block,
    // and not always the same planes (a re-split of hi + mid + lo can round
    // differently), so dQ's last bits differ between the two forms
#if GRL_ATTN_TPLANES
    abf16x8_t dtp[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      f32x16 dt = zero16();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        ai16x8_t pv;
#pragma unroll
        for (int j = 0; j < 8; ++j) pv[j] = u == perm_u ? onehot[j] : (short)0;
        dt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dsp[u][pl], __builtin_bit_cast(abf16x8_t, pv), dt, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
        dtp[u][pl] = __builtin_bit_cast(abf16x8_t, make_uint4(apack(dt[8 * u], dt[8 * u + 1]),
                                                              apack(dt[8 * u + 2], dt[8 * u + 3]),
                                                              apack(dt[8 * u + 4], dt[8 * u + 5]),
                                                              apack(dt[8 * u + 6], dt[8 * u + 7])));
    }
#else
    f32x16 dt = zero16();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ai16x8_t pv;
#pragma unroll
      for (int j = 0; j < 8; ++j) pv[j] = u == perm_u ? onehot[j] : (short)0;
      const abf16x8_t perm = __builtin_bit_cast(abf16x8_t, pv);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) dt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dsp[u][pl], perm, dt, 0, 0, 0);
    }
    abf16x8_t dtp[2][3];
    reg_planes(dt, dtp);
#endif
    f32x16 dq = zero16();  // dQ_blk[query][d] over this wave's 32 keys (columns d >= 16 discarded)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r0 = wave * 32 + kappa(8 * u + trq, h), r1 = wave * 32 + kappa(8 * u + 4 + trq, h);
      abf16x8_t kt[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        kt[pl] = tr8(&Kt_s[pl * KW * 16 + r0 * 16 + (trc & 15)], &Kt_s[pl * KW * 16 + r1 * 16 + (trc & 15)]);
      MFMA6(dq, dtp[u][0], dtp[u][1], dtp[u][2], kt[0], kt[1], kt[2]);
    }
    // dq: lanes = d (valid l32 < 16), registers r = query kappa(r, h); registers 4g..4g+3 are
    // the 4 consecutive queries 8g + 4h + 0..3 -> this block's slot, row d of wave's partial
    if (l32 < 16) {
      float* dst = Red_s + stg * RSLOT + wave * 16 * RP + l32 * RP + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + 8 * g) = make_float4(dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]);
    }
  }
  __syncthreads();
  if (q_hi > q_lo) reduce(q_lo + ((q_hi - q_lo - 1) >> 5 << 5));  // the last block's partials
  if (kv) {  // query split: partial dK into slab blockIdx.z (summed in split order afterwards)
    const int64_t rows = (int64_t)gridDim.y * N;
    float* dst = SPLIT ? a.part2 + (int64_t)blockIdx.z * rows * a.dk : a.dK;
    const int64_t rowk = (b * N + key) * a.dk;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = kappa(r, h);
      if (d < a.dk) dst[rowk + d] = acc[r];
    }
  }
}

// ---------------------------------------------------------------------------
// The fused dK / dQ pass on v_mfma_f32_16x16x32_bf16 (dk <= 16, PRE staging,
// 8 waves of 32 keys, one workgroup per CU): attn_bwd_kq_x6_kernel's work in
// 16 x 16 tiles.  Per query block of 32:
//  * S = Q K^T as in attn_bwd_h16_kernel (the six x6 products of the dk = 16
//    contraction paired along K = 32; K at natural scale, as dQ needs it, so
//    P = 2^(fma(s, log2 e, -lse2))) and dP = dO H^T (4 feature chunks of 32,
//    6 products each) in the same 2 x 2 tiles: lane group g holds queries
//    8 g .. 8 g + 7 of both, keys on lanes;
//  * dS = P (dP - D), split into planes, is the B operand of
//    dK^T[d][key] += Q^T dS as it lies (Q^T: transposed reads of the staged
//    16-wide planes); the 32x32x16 kernel's dK and dQ tiles were half
//    padding (dk = 16 of 32 rows), these have none;
//  * dS transposed through the wave's LDS slots: each plane's registers are
//    written as [key][q] rows and read back by ds_read_b64_tr_b16 with
//    queries on lanes and keys 8 g .. 8 g + 7 in registers -- dQ's A
//    operand, with K's planes (split once, registers) as B (an exact
//    selection-MFMA transposition, 12 more MFMAs and 12 packs per block,
//    measured 0.3-1.4 % slower end to end);
//  * dQ partials go through the LDS slots and per-workgroup slabs exactly as
//    in attn_bwd_kq_x6_kernel, so attn_qslab_sum_kernel is unchanged.
// Per block and wave 132 MFMAs of 16x16x32 = 66 of 32x32x16 (84 there).
// The same products in the same order per output; the pairing of S's
// products inside one MFMA changes rounding only (tested vs float64).
#define MFMA16(acc, a, b) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (acc), 0, 0, 0)
#define X6_16(acc, A, B)    \
  do {                      \
    MFMA16(acc, A[2], B[0]); \
    MFMA16(acc, A[1], B[1]); \
    MFMA16(acc, A[0], B[2]); \
    MFMA16(acc, A[1], B[0]); \
    MFMA16(acc, A[0], B[1]); \
    MFMA16(acc, A[0], B[0]); \
  } while (0)
template <bool SPLIT>
__global__ __launch_bounds__(64 * KQ_WAVES, 1) void attn_bwd_kq16_kernel(AttnArgs a) {
  constexpr int FC = 4, NW = KQ_WAVES, KW = KQ_KEYS;  // 128 value columns = 4 chunks of 32
  constexpr int RP = 36;                              // partial row pitch (floats), as attn_bwd_kq_x6_kernel
  constexpr int RSLOT = NW * 16 * RP;
  __shared__ __attribute__((aligned(16))) uint16_t Qp_s[2 * 3 * 32 * 16];  // 2 stages, 16-wide planes
  __shared__ __attribute__((aligned(16))) uint16_t Op_s[2 * 3 * 32 * 128];
  __shared__ __attribute__((aligned(16))) uint16_t Kt_s[3 * KW * 16];  // the workgroup's K rows, planes [key][16]
  __shared__ __attribute__((aligned(16))) float Red_s[2 * RSLOT];  // 2 slots x the waves' partials [w][d][RP]
  __shared__ __attribute__((aligned(16))) float Ms_s[2 * 32], Ds_s[2 * 32];  // lse2, D per query
  __shared__ __attribute__((aligned(16))) uint16_t Dt_s[NW * 2 * 1024];  // each wave's two 32 x 32 bf16 dS slots
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g = lane >> 4;
  const int64_t N = a.N, b = blockIdx.y;
  const int64_t key0 = a.k0 + (int64_t)blockIdx.x * KW + wave * 32;  // this wave's 32 keys
  const int64_t q_lo = SPLIT ? (int64_t)blockIdx.z * a.kr : a.q0, q_hi = SPLIT ? min<int64_t>(N, q_lo + a.kr) : a.q1;
  // this wave's K rows, natural scale, as planes [key][16] in LDS (S's B operand; zero for padded
  // keys), and dP's B operand H[key 16 kt + c16][32 fc + 8 g + j] in registers
  {
    const int64_t key = key0 + (lane >> 1);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = 8 * (lane & 1) + j;
      v[j] = (key < N && d < a.dk) ? a.K[(b * N + key) * a.dk + d] : 0.0f;
    }
    abf16x8_t p[3];
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), p[0], p[1], p[2]);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      *reinterpret_cast<abf16x8_t*>(&Kt_s[pl * KW * 16 + (wave * 32 + (lane >> 1)) * 16 + 8 * (lane & 1)]) = p[pl];
  }
  abf16x8_t hb[2][FC][3];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int64_t key = key0 + 16 * kt + c16;
    const bool kv = key < N;
    float v[8];
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 32 * fc + 8 * g + j;
        v[j] = (kv && f < a.dv) ? a.H[(b * N + key) * a.dv + f] : 0.0f;
      }
      asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), hb[kt][fc][0], hb[kt][fc][1],
              hb[kt][fc][2]);
    }
  }
  // B operand of dQ: K[key 8 g + j][d c16], the key order of the transposed dS
  abf16x8_t kq[3];
  {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t key = key0 + 8 * g + j;
      v[j] = (key < N && c16 < a.dk) ? a.K[(b * N + key) * a.dk + c16] : 0.0f;
    }
    asplit8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), kq[0], kq[1], kq[2]);
  }
  af32x4_t acck[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
  const int64_t qps = (int64_t)gridDim.y * N * 16, ops = (int64_t)gridDim.y * N * 128;
  const uint16_t* Qpb = a.Qpl16 + b * N * 16;
  const uint16_t* Opb = a.Opl + b * N * 128;
  const int64_t npad = (N + 31) & ~(int64_t)31;  // slab rows padded to whole query blocks
  float* slab = a.qslab + ((int64_t)b * gridDim.x + blockIdx.x) * 16 * npad;  // [d][npad]
  float pm = 0.0f, pd = 0.0f;
  auto fetch_stats = [&](int64_t q0) {
    if (tid < 32) {
      const int64_t qq = q0 + tid;
      const bool v = qq < q_hi;
      pm = v ? fmaf(a.smax[b * N + qq], ALOG2E, alog2(a.ssum[b * N + qq])) : INFINITY;  // P = 0 when padded
      pd = v ? a.Drow[b * N + qq] : 0.0f;
    }
  };
  auto reduce = [&](int64_t qb) {  // as attn_bwd_kq_x6_kernel: wave w adds queries [4w, 4w + 4) x 16 d
    const float* src = Red_s + (int)(((qb - q_lo) >> 5) & 1) * RSLOT;
    const int q = 4 * wave + (lane >> 4), d = lane & 15;
    float x = src[d * RP + q];
#pragma unroll
    for (int w = 1; w < NW; ++w) x += src[w * 16 * RP + d * RP + q];
    slab[d * npad + qb + q] = x;
  };
  dma_block<16, PL_PLAIN, NW>(Qpb, qps, q_lo, N, Qp_s, wave, lane);
  dma_block<128, PL_SWZ128, NW>(Opb, ops, q_lo, N, Op_s, wave, lane);
  fetch_stats(q_lo);
  const int qa1 = g < 2 ? 1 : 2, qa2 = g < 2 ? 1 : 0;  // S's A planes per MFMA: [hi|hi], [mid|lo], [mid|hi]
  const int kb0 = g < 2 ? 0 : 1, kb2 = g < 2 ? 1 : 2;  // and B planes: [hi|mid], [hi|hi], [mid|lo]
  const int qrow0 = 8 * (c16 >> 2) + (c16 & 3);        // query tile 0's row c16; tile 1: + 4
  const int q4 = c16 >> 2, p4 = c16 & 3;               // transposed reads: row q4 of a 4-row block, piece p4

  for (int64_t q0 = q_lo; q0 < q_hi; q0 += 32) {
    const int stg = (int)(((q0 - q_lo) >> 5) & 1);
    const uint16_t* Qp = Qp_s + stg * 3 * 512;
    const lds_u16* Qt = (const lds_u16*)Qp_s + stg * 3 * 512;
    const uint16_t* Op = Op_s + stg * 3 * 4096;
    float* Ms = Ms_s + stg * 32;
    float* Ds = Ds_s + stg * 32;
    if (tid < 32) {
      Ms[tid] = pm;
      Ds[tid] = pd;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (q0 + 32 < q_hi) {
      dma_block<16, PL_PLAIN, NW>(Qpb, qps, q0 + 32, N, Qp_s + (stg ^ 1) * 3 * 512, wave, lane);
      dma_block<128, PL_SWZ128, NW>(Opb, ops, q0 + 32, N, Op_s + (stg ^ 1) * 3 * 4096, wave, lane);
      fetch_stats(q0 + 32);
    }
    if (q0 > q_lo) reduce(q0 - 32);
    // S and dP tiles [qt][kt]: rows (queries 8 g + 4 qt + i) in registers, keys 16 kt + c16 on lanes
    af32x4_t st[2][2], dp[2][2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const uint16_t* qr = Qp + (qrow0 + 4 * qt) * 16 + 8 * (g & 1);
      abf16x8_t qa[3];
      qa[0] = *reinterpret_cast<const abf16x8_t*>(qr);
      qa[1] = *reinterpret_cast<const abf16x8_t*>(qr + qa1 * 512);
      qa[2] = *reinterpret_cast<const abf16x8_t*>(qr + qa2 * 512);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const uint16_t* kr = Kt_s + (wave * 32 + 16 * kt + c16) * 16 + 8 * (g & 1);
        af32x4_t s = {0.0f, 0.0f, 0.0f, 0.0f};  // small products first, hi.hi last: one rounding at |s|
        MFMA16(s, qa[2], *reinterpret_cast<const abf16x8_t*>(kr + kb2 * KW * 16));
        MFMA16(s, qa[1], *reinterpret_cast<const abf16x8_t*>(kr));
        MFMA16(s, qa[0], *reinterpret_cast<const abf16x8_t*>(kr + kb0 * KW * 16));
        st[qt][kt] = s;
        dp[qt][kt] = af32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
      }
    }
#pragma unroll
    for (int fc = 0; fc < FC; ++fc)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int off = swz128(qrow0 + 4 * qt, 32 * fc + 8 * g);  // conflict-free in the b128 lane groups
        abf16x8_t oa[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) oa[pl] = *reinterpret_cast<const abf16x8_t*>(&Op[pl * 4096 + off]);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) X6_16(dp[qt][kt], oa, hb[kt][fc]);
      }
    // dS = P (dP - D) for queries 8 g .. 8 g + 7, split into planes: dS[q][key] as B (k = q)
    const float4 m0 = *reinterpret_cast<const float4*>(Ms + 8 * g), m1 = *reinterpret_cast<const float4*>(Ms + 8 * g + 4);
    const float4 e0 = *reinterpret_cast<const float4*>(Ds + 8 * g), e1 = *reinterpret_cast<const float4*>(Ds + 8 * g + 4);
    abf16x8_t dsp[2][3];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const float4 lo = make_float4(aexp2(fmaf(st[0][kt][0], ALOG2E, -m0.x)) * (dp[0][kt][0] - e0.x),
                                    aexp2(fmaf(st[0][kt][1], ALOG2E, -m0.y)) * (dp[0][kt][1] - e0.y),
                                    aexp2(fmaf(st[0][kt][2], ALOG2E, -m0.z)) * (dp[0][kt][2] - e0.z),
                                    aexp2(fmaf(st[0][kt][3], ALOG2E, -m0.w)) * (dp[0][kt][3] - e0.w));
      const float4 hi = make_float4(aexp2(fmaf(st[1][kt][0], ALOG2E, -m1.x)) * (dp[1][kt][0] - e1.x),
                                    aexp2(fmaf(st[1][kt][1], ALOG2E, -m1.y)) * (dp[1][kt][1] - e1.y),
                                    aexp2(fmaf(st[1][kt][2], ALOG2E, -m1.z)) * (dp[1][kt][2] - e1.z),
                                    aexp2(fmaf(st[1][kt][3], ALOG2E, -m1.w)) * (dp[1][kt][3] - e1.w));
      asplit8(lo, hi, dsp[kt][0], dsp[kt][1], dsp[kt][2]);
    }
    {  // dK^T[d][key] += Q^T[d][q] dS[q][key]; Q^T rows 8 g .. 8 g + 7 by transposed reads
      abf16x8_t qT[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        qT[pl] = tr8s(Qt + pl * 512 + (8 * g + q4) * 16 + 4 * p4, Qt + pl * 512 + (8 * g + 4 + q4) * 16 + 4 * p4);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) X6_16(acck[kt], qT, dsp[kt]);
    }
    abf16x8_t dt[2][3];
    {
      // dS^T through this wave's LDS slots: plane pl's [key][q] rows (16-B chunk c of row k at
      // c ^ ((k >> 2) & 3): conflict-free row writes and transposed reads), read back by
      // ds_read_b64_tr_b16 as tile nt = dS[q 16 nt + c16][keys 8 g .. 8 g + 7]; plane 2 reuses slot 0
      // (a wave's LDS instructions execute in order, so its reads of plane 0 precede the rewrite)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        uint16_t* slot = Dt_s + (wave * 2 + (pl & 1)) * 1024;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int k = 16 * kt + c16;
          *reinterpret_cast<abf16x8_t*>(slot + k * 32 + ((g ^ ((k >> 2) & 3)) << 3)) = dsp[kt][pl];
        }
        const lds_u16* sl = (const lds_u16*)Dt_s + (wave * 2 + (pl & 1)) * 1024;
        const int k0 = 8 * g + q4, k1 = 8 * g + 4 + q4;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int ch = 2 * nt + (p4 >> 1), w = 4 * (p4 & 1);
          dt[nt][pl] = tr8s(sl + k0 * 32 + ((ch ^ ((k0 >> 2) & 3)) << 3) + w,
                            sl + k1 * 32 + ((ch ^ ((k1 >> 2) & 3)) << 3) + w);
        }
      }
    }
    // dQ_blk[q 16 nt + 4 g + i][d c16] over this wave's 32 keys -> this block's slot, row d of the wave's partial
    float* dst = Red_s + stg * RSLOT + wave * 16 * RP + c16 * RP + 4 * g;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      af32x4_t dq = {0.0f, 0.0f, 0.0f, 0.0f};
      X6_16(dq, dt[nt], kq);
      *reinterpret_cast<float4*>(dst + 16 * nt) = make_float4(dq[0], dq[1], dq[2], dq[3]);
    }
  }
  __syncthreads();
  if (q_hi > q_lo) reduce(q_lo + ((q_hi - q_lo - 1) >> 5 << 5));  // the last block's partials
  // dK[key 16 kt + c16][d 4 g + i]; query split: partial dK into slab blockIdx.z
  const int64_t rows = (int64_t)gridDim.y * N;
  float* dkd = SPLIT ? a.part2 + (int64_t)blockIdx.z * rows * a.dk : a.dK;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int64_t key = key0 + 16 * kt + c16;
    if (key >= N) continue;
    float* row = dkd + (b * N + key) * a.dk;
    if (a.dk == 16) {
      *reinterpret_cast<float4*>(row + 4 * g) = make_float4(acck[kt][0], acck[kt][1], acck[kt][2], acck[kt][3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < a.dk) row[4 * g + i] = acck[kt][i];
    }
  }
}
#undef X6_16
#undef MFMA16

// dQ[b][q][d] = sum over key workgroups x of qslab[b][x][q][d], in x order;
// accumulate: start from dQ (a later key chunk: the same chain of fp32 adds
// as one pass over every chunk's slabs)
__global__ void attn_qslab_sum_kernel(const float* __restrict__ qslab, int64_t B, int64_t X, int64_t N, int dk,
                                      float* __restrict__ dQ, int accumulate) {
  const int64_t n_all = B * N * dk;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x) {
    // i = (b * dk + d) * N + q: consecutive threads read consecutive q of one slab row
    const int64_t bd = i / N, q = i - bd * N, b = bd / dk;
    const int d = (int)(bd - b * dk);
    const int64_t npad = (N + 31) & ~(int64_t)31, xs = 16 * npad;  // slab [b][x][d][npad]
    const float* p = qslab + b * X * xs + (int64_t)d * npad + q;
    float acc = accumulate ? dQ[(b * N + q) * dk + d] : 0.0f;
    int64_t x = 0;
    for (; x + 4 <= X; x += 4) {
      const float v0 = p[(x + 0) * xs], v1 = p[(x + 1) * xs], v2 = p[(x + 2) * xs], v3 = p[(x + 3) * xs];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; x < X; ++x) acc += p[x * xs];
    dQ[(b * N + q) * dk + d] = acc;
  }
}

// Key split of the forward: out / o_norm / row_max / row_sum from the S
// partial (o, m, l) in split order (deterministic), m_s in base 2:
//   M = max_s m_s,  L = sum_s l_s 2^(m_s - M),  O = sum_s o_s 2^(m_s - M) / L
__global__ void attn_fwd_combine_kernel(AttnArgs a, int64_t rows, int S) {
  const int64_t n_all = rows * a.dv;
  const float* pm = a.part + (int64_t)S * rows * a.dv;
  const float* pl = pm + (int64_t)S * rows;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / a.dv;
    const int f = (int)(i - row * a.dv);
    const int64_t q = row % a.N;
    if (q < a.q0 || q >= a.q1) continue;  // a query range (grl_node_attention_fwd_rows): its rows only
    float M = -INFINITY;
    for (int s = 0; s < S; ++s) M = fmaxf(M, pm[s * rows + row]);
    float L = 0.0f, O = 0.0f;
    for (int s = 0; s < S; ++s) {
      const float w = aexp2(pm[s * rows + row] - M);  // partial maxima are base-2 (x6 forward)
      L += pl[s * rows + row] * w;
      O += a.part[(int64_t)s * n_all + i] * w;
    }
    O /= L;
    a.out[i] = a.gamma[f] * O + a.V[i];
    if (a.onorm) a.onorm[i] = O;
    if (f == 0 && a.rmax) {
      a.rmax[row] = M * ALN2;
      a.rsum[row] = L;
    }
  }
}

// out[i] = sum_{s < S} slab[s][i] in split order
__global__ void attn_slab_sum_kernel(const float* __restrict__ slab, int64_t n, int S, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.0f;
    for (int s = 0; s < S; ++s) acc += slab[(int64_t)s * n + i];
    out[i] = acc;
  }
}

#undef MFMA

enum AttnPass { PASS_FWD, PASS_BWD_Q, PASS_BWD_KV };

// path option attn_x6 = 0 keeps the fp32-MFMA kernels
bool attn_x6_enabled() { return opt(OPT_ATTN_X6) != 0; }

// path option attn_fwd8 = 0 keeps the pipelined forward on 4-wave workgroups (A/B aid)
bool attn_fwd8_enabled() { return opt(OPT_ATTN_FWD8) != 0; }

// path option attn_dh8 = 0 keeps dH on 4-wave workgroups (A/B aid)
bool attn_dh8_enabled() { return opt(OPT_ATTN_DH8) != 0; }

// path option attn_fused_dq = 0 keeps the separate dQ kernel (A/B aid)
bool attn_fused_dq_enabled() { return opt(OPT_ATTN_FUSED_DQ) != 0; }

// path option attn_dh16 = 0 keeps dH on the 32x32x16 kernel
bool attn_dh16_enabled() { return opt(OPT_ATTN_DH16) != 0; }

// path option attn_kq16 = 0 keeps the fused dK / dQ pass on the 32x32x16 kernel
bool attn_kq16_enabled() { return opt(OPT_ATTN_KQ16) != 0; }

// path option attn_pipe = 0 keeps the unpipelined x6 forward (A/B aid)
bool attn_pipe_enabled() { return opt(OPT_ATTN_PIPE) != 0; }

template <int DKP, int NT>
int launch_attn(AttnPass pass, const AttnArgs& a0, int64_t B, int S, hipStream_t st) {
  AttnArgs a = a0;
  // dk in (32, 64] (NodeSelfAtten of input_dim > 256): the fp32-MFMA kernels only
  const bool x6 = DKP <= 32 && attn_x6_enabled() && (pass == PASS_FWD || NT == 4);
  if (!x6 || !a.part) S = 1;
  if (S == 1) {
    a.part = a.part2 = nullptr;
    a.kr = a.N;
  }
  // query-stationary passes (forward, dQ) cover the queries [q0, q1); dK / dH every key
  const int64_t nq = a.q1 - a.q0;
  if (pass != PASS_BWD_KV && nq <= 0) return GRL_OK;  // no query rows: no forward / dQ work
  const dim3 grid((unsigned)ceil_div(pass == PASS_BWD_KV ? a.N : nq, 128), (unsigned)B, (unsigned)S);
  const bool pre = pass == PASS_BWD_KV ? (a.Qpl && a.Opl) : (a.Kpl && a.Hpl);
  const int64_t rows = B * a.N;
  const unsigned red = (unsigned)std::min<int64_t>(ceil_div(rows * std::max(a.dv, 1), 256), 8192);
#define GRL_X6L(KERNEL, ...)                                                                      \
  do {                                                                                              \
    if (pre && S > 1)                                                                               \
      hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, true>), grid, dim3(256), 0, st, a);             \
    else if (pre)                                                                                   \
      hipLaunchKernelGGL((KERNEL<__VA_ARGS__, true, false>), grid, dim3(256), 0, st, a);            \
    else if (S > 1)                                                                                 \
      hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, true>), grid, dim3(256), 0, st, a);            \
    else                                                                                            \
      hipLaunchKernelGGL((KERNEL<__VA_ARGS__, false, false>), grid, dim3(256), 0, st, a);           \
  } while (0)
  if constexpr (DKP > 32) {
    if (pass == PASS_FWD)
      hipLaunchKernelGGL((attn_fwd_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
    else if (pass == PASS_BWD_Q)
      hipLaunchKernelGGL((attn_bwd_q_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((attn_bwd_kv_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
  } else if (pass == PASS_FWD && x6) {
    if (pre && attn_pipe_enabled() && attn_fwd8_enabled()) {  // 256 queries per workgroup
      const dim3 g8((unsigned)ceil_div(nq, 256), (unsigned)B, (unsigned)S);
      if (S > 1)
        hipLaunchKernelGGL((attn_fwd_x6p_kernel<DKP, NT, true, 8>), g8, dim3(512), 0, st, a);
      else
        hipLaunchKernelGGL((attn_fwd_x6p_kernel<DKP, NT, false, 8>), g8, dim3(512), 0, st, a);
    } else if (pre && attn_pipe_enabled()) {
      if (S > 1)
        hipLaunchKernelGGL((attn_fwd_x6p_kernel<DKP, NT, true>), grid, dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL((attn_fwd_x6p_kernel<DKP, NT, false>), grid, dim3(256), 0, st, a);
    } else {
      GRL_X6L(attn_fwd_x6_kernel, DKP, NT);
    }
    if (S > 1) {
      GRL_LAUNCH_CHECK();
      hipLaunchKernelGGL(attn_fwd_combine_kernel, dim3(red), dim3(256), 0, st, a, rows, S);
    }
  } else if (pass == PASS_FWD) {
    hipLaunchKernelGGL((attn_fwd_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
  } else if (x6) {  // backward x6: dv in (96, 128]
    if (pass == PASS_BWD_Q) {
      GRL_X6L(attn_bwd_q_x6_kernel, DKP);
      if (S > 1 && a.dk > 0) {
        GRL_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_slab_sum_kernel, dim3(red), dim3(256), 0, st, a.part, rows * a.dk, S, a.dQ);
      }
    } else {
      if (S > 1) a.part2 = a.part + (int64_t)S * rows * a.dv;
      if (pre && attn_dh8_enabled() && DKP == 16 && attn_dh16_enabled()) {  // dH in 16 x 16 tiles
        const dim3 g8((unsigned)ceil_div(a.N, 256), (unsigned)B, (unsigned)S);
        if (S > 1)
          hipLaunchKernelGGL((attn_bwd_h16_kernel<true>), g8, dim3(512), 0, st, a);
        else
          hipLaunchKernelGGL((attn_bwd_h16_kernel<false>), g8, dim3(512), 0, st, a);
      } else if (pre && attn_dh8_enabled()) {  // dH on 256-key workgroups
        const dim3 g8((unsigned)ceil_div(a.N, 256), (unsigned)B, (unsigned)S);
        if (S > 1)
          hipLaunchKernelGGL((attn_bwd_kv_x6_kernel<DKP, true, true, true, 8>), g8, dim3(512), 0, st, a);
        else
          hipLaunchKernelGGL((attn_bwd_kv_x6_kernel<DKP, true, true, false, 8>), g8, dim3(512), 0, st, a);
      } else {
        GRL_X6L(attn_bwd_kv_x6_kernel, DKP, true);
      }
      GRL_LAUNCH_CHECK();
      bool kq = false;
      if constexpr (DKP == 16) {
        if (a.qslab && pre) {  // dK with dQ folded in (grl_node_attention_bwd skipped the dQ pass)
          kq = true;
          // key chunks of xc workgroups, as many slabs as the workspace holds (a.kr_slabs)
          const int64_t xall = ceil_div(a.N, KQ_KEYS), xc = std::max<int64_t>(1, std::min<int64_t>(xall, a.kq_chunk));
          for (int64_t x0 = 0; x0 < xall; x0 += xc) {
            AttnArgs ac = a;
            ac.k0 = x0 * KQ_KEYS;
            const dim3 gkq((unsigned)std::min<int64_t>(xc, xall - x0), (unsigned)B, (unsigned)S);
            if (attn_kq16_enabled() && S > 1)
              hipLaunchKernelGGL((attn_bwd_kq16_kernel<true>), gkq, dim3(64 * KQ_WAVES), 0, st, ac);
            else if (attn_kq16_enabled())
              hipLaunchKernelGGL((attn_bwd_kq16_kernel<false>), gkq, dim3(64 * KQ_WAVES), 0, st, ac);
            else if (S > 1)
              hipLaunchKernelGGL((attn_bwd_kq_x6_kernel<true>), gkq, dim3(64 * KQ_WAVES), 0, st, ac);
            else
              hipLaunchKernelGGL((attn_bwd_kq_x6_kernel<false>), gkq, dim3(64 * KQ_WAVES), 0, st, ac);
            GRL_LAUNCH_CHECK();
            if (a.dk > 0)
              hipLaunchKernelGGL(attn_qslab_sum_kernel,
                                 dim3((unsigned)std::min<int64_t>(ceil_div(rows * a.dk, 256), 8192)), dim3(256), 0, st,
                                 a.qslab, B, (int64_t)gkq.x, a.N, a.dk, a.dQ, (int)(x0 > 0));
          }
        }
      }
      if (!kq) GRL_X6L(attn_bwd_kv_x6_kernel, DKP, false);
      if (S > 1) {
        GRL_LAUNCH_CHECK();
        hipLaunchKernelGGL(attn_slab_sum_kernel, dim3(red), dim3(256), 0, st, a.part, rows * a.dv, S, a.dH);
        if (a.dk > 0) {
          GRL_LAUNCH_CHECK();
          hipLaunchKernelGGL(attn_slab_sum_kernel, dim3(red), dim3(256), 0, st, a.part2, rows * a.dk, S, a.dK);
        }
      }
    }
#undef GRL_X6L
  } else if (pass == PASS_BWD_Q) {
    hipLaunchKernelGGL((attn_bwd_q_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_kv_kernel<DKP, NT>), grid, dim3(256), 0, st, a);
  }
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}

// Key (forward, dQ) / query (dH, dK) split: the loop range is cut into S
// pieces of >= 256 rows (multiples of 32) whose partials are combined in
// split order (deterministic).  The kernels run 2 four-wave workgroups per
// CU and every workgroup (128 rows x N / S) does the same work, so the grid
// runs in rounds of 2 x CUs and a partial last round idles the rest of the
// chip: S is the one (<= 16) that maximises the filled fraction of the
// rounds, B ceil(N / 128) S / (rounds x 2 CUs), less 0.5 % per extra split
// (partials and their combine).  N = 100k, 782 workgroups: 1.53 rounds
// (76 %) unsplit; S = 7 fills 97 % -- forward 17.6 -> 13.9 ms, forward +
// backward 80.2 -> 61.7 ms (tools/ab_attn_splits.sh).  N = 131072 (1024
// workgroups, two full rounds) stays unsplit.  Returns S, sets *kr (rows
// per split).
int attn_splits(int64_t B, int64_t N, int64_t* kr) {
  const int64_t blocks = ceil_div(N, 128) * B, slots = 2 * (int64_t)device_cu_count();
  const int64_t smax = std::max<int64_t>(1, std::min<int64_t>(16, N / 256));
  auto filled = [&](int64_t s) {
    const int64_t w = blocks * s;
    return (double)w / (double)(ceil_div(w, slots) * slots);
  };
  int64_t S = 1;
  double best = filled(1);
  for (int64_t s = 2; s <= smax; ++s) {
    const double score = filled(s) - 0.005 * (double)(s - 1);
    if (score > best + 1e-9) {
      best = score;
      S = s;
    }
  }
  S = std::max<int64_t>(1, std::min<int64_t>(S, 64));
  *kr = ceil_div(ceil_div(N, S), 32) * 32;
  return (int)ceil_div(N, *kr);
}

int attn_dkp(int dk) { return dk <= 16 ? 16 : 32; }
int attn_dvp(int dv) {
  const int nt = (int)ceil_div(dv, 32);
  return 32 * (nt <= 1 ? 1 : nt <= 2 ? 2 : nt <= 4 ? 4 : 8);
}

template <int DKP>
int dispatch_nt(AttnPass pass, const AttnArgs& a, int64_t B, int S, hipStream_t st) {
  const int nt = attn_dvp(a.dv) / 32;
  if (nt == 1) return launch_attn<DKP, 1>(pass, a, B, S, st);
  if (nt == 2) return launch_attn<DKP, 2>(pass, a, B, S, st);
  if (nt == 4) return launch_attn<DKP, 4>(pass, a, B, S, st);
  return launch_attn<DKP, 8>(pass, a, B, S, st);
}

int dispatch(AttnPass pass, const AttnArgs& a, int64_t B, int S, hipStream_t st) {
  if (a.N == 0 || B == 0) return GRL_OK;
  if (a.dk <= 16) return dispatch_nt<16>(pass, a, B, S, st);
  if (a.dk <= 32) return dispatch_nt<32>(pass, a, B, S, st);
  return dispatch_nt<64>(pass, a, B, S, st);
}

constexpr int64_t kAttnPlaneMinRows = 4096;

// Workspace of the PRE staging: bf16 planes [3][B*N][W] of K, H (forward and
// backward) and Q, dO (backward), each section 256-B aligned
size_t attn_plane_bytes(int64_t rows, int W) { return ((size_t)3 * rows * W * 2 + 255) / 256 * 256; }

// Split `src` [rows][width] into planes at *cursor (advanced); false when
// the workspace is too small (the caller then runs the in-kernel split)
bool attn_split(const float* src, int64_t rows, int width, int W, unsigned char*& cursor, const unsigned char* end,
                const uint16_t** out, hipStream_t st) {
  const size_t need = attn_plane_bytes(rows, W);
  if (!src || cursor + need > end) return false;
  uint16_t* planes = reinterpret_cast<uint16_t*>(cursor);
  const int64_t n4 = rows * (W / 4);
  hipLaunchKernelGGL(attn_split_rows_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n4, 256), 8192)), dim3(256),
                     0, st, src, rows, width, W, planes);
  cursor += need;
  *out = planes;
  return true;
}

int check_dims(const char* who, int64_t B, int64_t N, int dk, int dv) {
  GRL_CHECK_ARG(B >= 0 && N >= 0, "%s: negative size", who);
  // dk = 0 is legal (input_dim < 8 gives Linear(F, 0) in the reference): all
  // scores are 0 and the attention is uniform, which the kernels compute as is.
  GRL_CHECK_ARG(dk >= 0 && dk <= 64, "%s: key width %d outside [0, 64] (NodeSelfAtten: input_dim // 8)", who, dk);
  GRL_CHECK_ARG(dv >= 1 && dv <= 256, "%s: value width %d outside [1, 256]", who, dv);
  GRL_CHECK_ARG(B * ceil_div(N, 128) < 2147483647LL && B < 65536, "%s: grid too large", who);
  return GRL_OK;
}

}  // namespace
}  // namespace grl

using namespace grl;

extern "C" size_t grl_node_attention_workspace_size(int64_t B, int64_t N, int32_t dk, int32_t dv) {
  if (B <= 0 || N <= 0 || dk < 0 || dk > 32 || dv < 1 || dv > 256) return 0;  // dk > 32: fp32 kernels, no workspace
  const int64_t rows = B * N;
  int64_t kr;
  const int S = attn_splits(B, N, &kr);
  const size_t part = S > 1 ? ((size_t)S * rows * (dv + std::max(dk, 2) + 2) * 4 + 255) / 256 * 256 : 0;
  const size_t planes =
      rows >= kAttnPlaneMinRows ? 2 * attn_plane_bytes(rows, 32) + 2 * attn_plane_bytes(rows, attn_dvp(dv)) : 0;
  return planes + part ? planes + part + 512 : 0;
}

// the backward's dQ slabs (attn_bwd_kq_x6_kernel): dk <= 16, x6 planes;
// N^2 / 4 bytes at B = 1 (2.5 GB at N = 100k) in key chunks of at most
// kAttnQslabMax bytes (N = 500k: 3 chunks of 768 key workgroups)
constexpr size_t kAttnQslabMax = (size_t)24 << 30;
static size_t attn_qslab_x_bytes(int64_t B, int64_t N) {  // one key workgroup's slabs
  return (size_t)B * (size_t)(ceil_div(N, 32) * 32) * 16 * 4;
}
static int64_t attn_qslab_chunk(int64_t B, int64_t N) {  // key workgroups per fused launch
  const int64_t o = opt(OPT_ATTN_QSLAB_MAX);  // test aid: a smaller chunk budget (bytes)
  const size_t cap = o > 0 ? (size_t)o : kAttnQslabMax;
  const int64_t all = ceil_div(N, KQ_KEYS), fit = (int64_t)(cap / attn_qslab_x_bytes(B, N));
  if (fit >= all) return all;
  const int64_t cus = device_cu_count();  // one workgroup per CU: whole rounds of the grid
  return std::max<int64_t>(1, fit >= cus ? fit / cus * cus : fit);
}
static size_t attn_qslab_bytes(int64_t B, int64_t N, int dk, int dv) {
  if (!attn_fused_dq_enabled() || dk > 16 || attn_dvp(dv) != 128 || B * N < kAttnPlaneMinRows) return 0;
  const size_t n = (size_t)attn_qslab_chunk(B, N) * attn_qslab_x_bytes(B, N);
  return (n + 255) / 256 * 256;
}

extern "C" size_t grl_node_attention_bwd_workspace_size(int64_t B, int64_t N, int32_t dk, int32_t dv) {
  const size_t base = grl_node_attention_workspace_size(B, N, dk, dv);
  const size_t q = base ? attn_qslab_bytes(B, N, dk, dv) : 0;
  return base + (q ? q + attn_plane_bytes(B * N, 16) : 0);
}

extern "C" int grl_node_attention_fwd_rows(const float* Q, const float* K, const float* H, const float* V,
                                           const float* gamma, float* out, float* o_norm, float* row_max,
                                           float* row_sum, int64_t B, int64_t N, int32_t dk, int32_t dv,
                                           int64_t q_begin, int64_t q_end, void* workspace, size_t workspace_bytes,
                                           grl_stream_t stream) {
  TraceRange trace_("grl_node_attention_fwd");
  int rc = check_dims("grl_node_attention_fwd", B, N, dk, dv);
  if (rc) return rc;
  GRL_CHECK_ARG(0 <= q_begin && q_begin <= q_end && q_end <= N, "grl_node_attention_fwd: query rows [%lld, %lld) "
                "outside [0, %lld)", (long long)q_begin, (long long)q_end, (long long)N);
  if (q_begin == q_end) return GRL_OK;
  if (B == 0 || N == 0) return GRL_OK;
  GRL_CHECK_ARG((dk == 0 || (Q && K)) && H && V && gamma && out, "grl_node_attention_fwd: NULL pointer");
  GRL_CHECK_ARG((row_max == nullptr) == (row_sum == nullptr), "grl_node_attention_fwd: row_max/row_sum: both or none");
  AttnArgs a{};
  a.Q = Q;
  a.K = K;
  a.H = H;
  a.V = V;
  a.gamma = gamma;
  a.out = out;
  a.onorm = o_norm;
  a.rmax = row_max;
  a.rsum = row_sum;
  a.N = N;
  a.dk = dk;
  a.dv = dv;
  a.q0 = q_begin;
  a.q1 = q_end;
  hipStream_t st = as_stream(stream);
  int S = 1;
  // below ~4k rows the per-call split launches cost more than the in-kernel
  // splits they save (a 74-node page: 2 extra launches per call)
  if (workspace && attn_x6_enabled() && dk <= 32) {  // split K and H once for every query block
    unsigned char* cur = reinterpret_cast<unsigned char*>((reinterpret_cast<uintptr_t>(workspace) + 255) & ~(uintptr_t)255);
    const unsigned char* end = static_cast<unsigned char*>(workspace) + workspace_bytes;
    const uint16_t *kp = nullptr, *hp = nullptr;
    if (B * N >= kAttnPlaneMinRows && attn_split(K, B * N, dk, attn_dkp(dk), cur, end, &kp, st) &&
        attn_split(H, B * N, dv, attn_dvp(dv), cur, end, &hp, st)) {
      a.Kpl = kp;
      a.Hpl = hp;
    }
    GRL_LAUNCH_CHECK();
    int64_t kr;
    // small N: key split with (o, m, l) partials.  The split depends on N alone, not on the query range, so
    // a node-range shard's query rows (grl.dist sharded attention) are bitwise the whole-range call's rows.
    S = attn_splits(B, N, &kr);
    if (S > 1 && cur + (size_t)S * B * N * (dv + 2) * 4 <= end) {
      a.part = reinterpret_cast<float*>(cur);
      a.kr = kr;
    } else {
      S = 1;
    }
  }
  return dispatch(PASS_FWD, a, B, S, st);
}

extern "C" int grl_node_attention_bwd_rows(const float* Q, const float* K, const float* H, const float* dO,
                                           const float* row_max, const float* row_sum, const float* D, float* dQ,
                                           float* dK, float* dH, int64_t B, int64_t N, int32_t dk, int32_t dv,
                                           int64_t q_begin, int64_t q_end, void* workspace, size_t workspace_bytes,
                                           grl_stream_t stream) {
  TraceRange trace_("grl_node_attention_bwd");
  int rc = check_dims("grl_node_attention_bwd", B, N, dk, dv);
  if (rc) return rc;
  GRL_CHECK_ARG(0 <= q_begin && q_begin <= q_end && q_end <= N, "grl_node_attention_bwd: query rows [%lld, %lld) "
                "outside [0, %lld)", (long long)q_begin, (long long)q_end, (long long)N);
  if (B == 0 || N == 0) return GRL_OK;
  GRL_CHECK_ARG((dk == 0 || (Q && K && dQ && dK)) && H && dO && row_max && row_sum && D && dH,
                "grl_node_attention_bwd: NULL pointer");
  AttnArgs a{};
  a.Q = Q;
  a.K = K;
  a.H = H;
  a.dO = dO;
  a.smax = row_max;
  a.ssum = row_sum;
  a.Drow = D;
  a.dQ = dQ;
  a.dK = dK;
  a.dH = dH;
  a.N = N;
  a.dk = dk;
  a.dv = dv;
  a.q0 = q_begin;
  a.q1 = q_end;
  const bool ranged = q_begin != 0 || q_end != N;
  hipStream_t st = as_stream(stream);
  int S = 1;
  if (workspace && attn_x6_enabled() && attn_dvp(dv) == 128 && dk <= 32) {  // the x6 backward's operands
    unsigned char* cur = reinterpret_cast<unsigned char*>((reinterpret_cast<uintptr_t>(workspace) + 255) & ~(uintptr_t)255);
    const unsigned char* end = static_cast<unsigned char*>(workspace) + workspace_bytes;
    const uint16_t *kp = nullptr, *hp = nullptr, *qp = nullptr, *op = nullptr;
    if (B * N >= kAttnPlaneMinRows && attn_split(K, B * N, dk, 32, cur, end, &kp, st) &&
        attn_split(H, B * N, dv, 128, cur, end, &hp, st) &&
        attn_split(Q, B * N, dk, 32, cur, end, &qp, st) && attn_split(dO, B * N, dv, 128, cur, end, &op, st)) {
      a.Kpl = kp;
      a.Hpl = hp;
      a.Qpl = qp;
      a.Opl = op;
    }
    GRL_LAUNCH_CHECK();
    int64_t kr;
    S = ranged ? 1 : attn_splits(B, N, &kr);  // small N: key / query split with ordered partial sums
    if (S > 1 && cur + (size_t)S * B * N * (dv + dk) * 4 <= end) {
      a.part = reinterpret_cast<float*>(cur);
      a.kr = kr;
      cur += ((size_t)S * B * N * (dv + dk) * 4 + 255) / 256 * 256;
    } else {
      S = 1;
    }
    const size_t qs = ranged ? 0 : attn_qslab_bytes(B, N, dk, dv);  // ranged: the dQ kernel (no slabs)
    const uint16_t* q16 = nullptr;
    if (qs && a.Qpl && dk > 0 && cur + qs <= end) {
      a.qslab = reinterpret_cast<float*>(cur);
      a.kq_chunk = attn_qslab_chunk(B, N);
      cur += qs;
      if (attn_split(Q, B * N, dk, 16, cur, end, &q16, st)) {
        a.Qpl16 = q16;
      } else {
        a.qslab = nullptr;
      }
      GRL_LAUNCH_CHECK();
    }
  }
  if (!a.qslab) {
    rc = dispatch(PASS_BWD_Q, a, B, S, st);
    if (rc) return rc;
  }
  return dispatch(PASS_BWD_KV, a, B, S, st);
}

extern "C" int grl_node_attention_fwd(const float* Q, const float* K, const float* H, const float* V,
                                      const float* gamma, float* out, float* o_norm, float* row_max, float* row_sum,
                                      int64_t B, int64_t N, int32_t dk, int32_t dv, void* workspace,
                                      size_t workspace_bytes, grl_stream_t stream) {
  return grl_node_attention_fwd_rows(Q, K, H, V, gamma, out, o_norm, row_max, row_sum, B, N, dk, dv, 0, N, workspace,
                                     workspace_bytes, stream);
}

extern "C" int grl_node_attention_bwd(const float* Q, const float* K, const float* H, const float* dO,
                                      const float* row_max, const float* row_sum, const float* D, float* dQ,
                                      float* dK, float* dH, int64_t B, int64_t N, int32_t dk, int32_t dv,
                                      void* workspace, size_t workspace_bytes, grl_stream_t stream) {
  return grl_node_attention_bwd_rows(Q, K, H, dO, row_max, row_sum, D, dQ, dK, dH, B, N, dk, dv, 0, N, workspace,
                                     workspace_bytes, stream);
}
