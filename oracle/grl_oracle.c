/*
 * grl_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the GraphCNNDropEdge aggregation hot path, used as the
 * parity checker for the HIP engine and as the CPU baseline timed by
 * bench.py ("cpu_baseline.kind": "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (graph-representation-learning_amd/) never does.
 *
 * What it restates (reference paths relative to the reference repo root):
 *  - A_pre = preprocess_adj(A): gnn/models/networks/robust_gcn.py:53-72.
 *    A_pre[b, n*(L+1)+l, m] = (l == 0 ? delta(n,m) : A[b, n, l-1, m]) where A is
 *    the collate layout (B, N, L, N) permuted at drop_robust_gcn.py:63.
 *  - new_V = matmul(A_drop, V): robust_gcn.py:45-47, summed here over the
 *    nonzeros of A_pre only (typed CSR), in ascending-m order per row with
 *    one fmaf per nonzero.
 *  - edge_dropout = nn.Dropout(p) over A_pre (drop_robust_gcn.py:38,76,80,85):
 *    keep with probability 1-p, scale by float(1/(1-p)) (torch
 *    native_dropout).  The Bernoulli draw is replaced by the engine's
 *    regenerable counter hash, restated below from its specification
 *    (include/grl.h, GrlDropEdge) -- not from the engine's source.
 *  - autograd of the bmm (BmmBackward0): dV = A_drop^T dZ.
 *
 * Parity pin: the fixtures in tests/golden/ were produced by the reference's own
 * GraphConv / GraphCNNDropEdge (imported from /root/reference by
 * tests/golden/make_golden.py); tests/test_oracle.py checks this file and
 * oracle/dense_ref.py against them.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------- DropEdge hash (spec: include/grl.h) ------------------- */
static inline uint64_t o_mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

uint64_t oracle_dropedge_key(uint64_t seed, uint64_t call) {
  return o_mix64(o_mix64(seed ^ 0x6A09E667F3BCC909ull) + call * 0x9E3779B97F4A7C15ull);
}

uint32_t oracle_dropedge_bits(uint64_t key, uint64_t id) {
  return (uint32_t)(o_mix64(key ^ (id * 0xD1B54A32D192ED03ull)) >> 32);
}

typedef struct {
  uint64_t key;
  uint32_t threshold;
  float scale;
  int32_t active;
  int32_t drop_self;
} ODrop;

void oracle_dropedge_init(ODrop* d, float p, uint64_t seed, uint64_t call, int32_t drop_self) {
  d->key = oracle_dropedge_key(seed, call);
  d->drop_self = drop_self ? 1 : 0;
  if (p <= 0.0f) {
    d->active = 0;
    d->threshold = 0;
    d->scale = 1.0f;
    return;
  }
  d->active = 1;
  if (p >= 1.0f) {
    d->threshold = 0xFFFFFFFFu;
    d->scale = 0.0f;
    return;
  }
  double thr = floor((double)p * 4294967296.0);
  d->threshold = thr >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)thr;
  d->scale = (float)(1.0 / (1.0 - (double)p));
}

static inline float o_weight(const ODrop* d, float v, uint64_t id) {
  if (!d || !d->active) return v;
  return oracle_dropedge_bits(d->key, id) >= d->threshold ? v * d->scale : 0.0f;
}

void oracle_dropedge_mask(const ODrop* d, uint64_t id_base, int64_t count, uint8_t* keep) {
  for (int64_t i = 0; i < count; ++i) keep[i] = o_weight(d, 1.0f, id_base + (uint64_t)i) != 0.0f;
}

/* ---------------- typed SpMM forward / backward ------------------------- */
/* Sum of w_e * src[idx[e]] over edges [e0, e1) as one fmaf chain from 0 (the
 * reference's bmm row restricted to nonzeros, in CSR/CSC order). */
static void o_chain(float* acc, int32_t e0, int32_t e1, const int32_t* idx, const int32_t* eid, const float* vals,
                    uint64_t edge_base, const float* src, int64_t lds, int32_t F, const ODrop* d) {
  for (int32_t e = e0; e < e1; ++e) {
    const float v = vals ? vals[e] : 1.0f;
    const uint64_t id = edge_base + (eid ? (uint64_t)(uint32_t)eid[e] : (uint64_t)e);
    const float w = o_weight(d, v, id);
    if (w == 0.0f) continue;
    const float* xr = src + (int64_t)idx[e] * lds;
    for (int f = 0; f < F; ++f) acc[f] = fmaf(w, xr[f], acc[f]);
  }
}

/* Segment [e0, e1) of a row: plain fmaf chain, or -- for rows the engine
 * splits (row edges > split_threshold >= 0) -- chunks of split_chunk edges,
 * each its own chain from 0, added in chunk order onto acc's initial value
 * (the engine's load-balanced summation order; include/grl.h GrlSplitPlan). */
static void o_segment(float* acc, float* tmp, int heavy, int32_t chunk, int32_t e0, int32_t e1, const int32_t* idx,
                      const int32_t* eid, const float* vals, uint64_t edge_base, const float* src, int64_t lds,
                      int32_t F, const ODrop* d) {
  if (!heavy) {
    o_chain(acc, e0, e1, idx, eid, vals, edge_base, src, lds, F, d);
    return;
  }
  for (int32_t c = e0; c < e1; c += chunk) {
    for (int f = 0; f < F; ++f) tmp[f] = 0.0f;
    o_chain(tmp, c, c + chunk < e1 ? c + chunk : e1, idx, eid, vals, edge_base, src, lds, F, d);
    for (int f = 0; f < F; ++f) acc[f] = acc[f] + tmp[f];
  }
}

/* X: gathered rows (colidx indexes it); Xself: row n's own features
 * (NULL = X, i.e. rows and sources share numbering). */
void oracle_spmm_fwd(int64_t rows, int32_t S, int32_t hs, const int32_t* rowptr, const int32_t* colidx,
                     const float* vals, uint64_t edge_base, uint64_t self_base, const float* X, const float* Xself,
                     int64_t ldx, int32_t F, float* Z, const ODrop* d, int32_t nthreads, int32_t split_threshold,
                     int32_t split_chunk) {
  if (!Xself) Xself = X;
  const int64_t ldz = (int64_t)(S + hs) * F;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    float* tmp = (float*)malloc(sizeof(float) * (size_t)F);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (int64_t n = 0; n < rows; ++n) {
      float* zr = Z + n * ldz;
      if (hs) {
        float w = 1.0f;
        if (d && d->active && d->drop_self) w = o_weight(d, 1.0f, self_base + (uint64_t)n);
        const float* xr = Xself + n * ldx;
        for (int f = 0; f < F; ++f) zr[f] = w != 0.0f ? w * xr[f] : 0.0f;
      }
      const int heavy = split_threshold >= 0 && rowptr[(n + 1) * S] - rowptr[n * S] > split_threshold;
      for (int t = 0; t < S; ++t) {
        float* acc = zr + (int64_t)(hs + t) * F;
        for (int f = 0; f < F; ++f) acc[f] = 0.0f;
        const int64_t s = n * S + t;
        o_segment(acc, tmp, heavy, split_chunk, rowptr[s], rowptr[s + 1], colidx, NULL, vals, edge_base, X, ldx, F,
                  d);
      }
    }
    free(tmp);
  }
}

void oracle_spmm_bwd(int64_t rows, int64_t self_rows, int32_t S, int32_t hs, const int32_t* colptr,
                     const int32_t* zrow, const int32_t* eid, const float* cvals, uint64_t edge_base,
                     uint64_t self_base, const float* dZ, int32_t F, float* dX, int64_t lddx, const ODrop* d,
                     int32_t nthreads, int32_t split_threshold, int32_t split_chunk) {
  const int64_t ldz = (int64_t)(S + hs) * F;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
  {
    float* tmp = (float*)malloc(sizeof(float) * (size_t)F);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (int64_t m = 0; m < rows; ++m) {
      float* acc = dX + m * lddx;
      for (int f = 0; f < F; ++f) acc[f] = 0.0f;
      if (hs && m < self_rows) {
        float w = 1.0f;
        if (d && d->active && d->drop_self) w = o_weight(d, 1.0f, self_base + (uint64_t)m);
        if (w != 0.0f) {
          const float* zr = dZ + m * ldz;
          for (int f = 0; f < F; ++f) acc[f] = w * zr[f];
        }
      }
      const int heavy = split_threshold >= 0 && colptr[m + 1] - colptr[m] > split_threshold;
      o_segment(acc, tmp, heavy, split_chunk, colptr[m], colptr[m + 1], zrow, eid, cvals, edge_base, dZ, F, F, d);
    }
    free(tmp);
  }
}

/* ---------------- format conversions ------------------------------------ */
/* dense A[b, n, t, m] (element strides) -> typed CSR rows (b*N+n)*L+t,
 * global source b*N+m, ascending m.  Returns nnz; pass colidx == NULL to
 * only fill rowptr. */
int64_t oracle_dense_to_csr(const float* A, int64_t B, int64_t N, int32_t L, const int64_t* st, int32_t* rowptr,
                            int32_t* colidx, float* vals) {
  int64_t nnz = 0;
  int64_t r = 0;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t n = 0; n < N; ++n)
      for (int32_t t = 0; t < L; ++t, ++r) {
        rowptr[r] = (int32_t)nnz;
        const float* row = A + b * st[0] + n * st[1] + (int64_t)t * st[2];
        for (int64_t m = 0; m < N; ++m) {
          const float v = row[m * st[3]];
          if (v != 0.0f) {
            if (colidx) colidx[nnz] = (int32_t)(b * N + m);
            if (colidx && vals) vals[nnz] = v;
            ++nnz;
          }
        }
      }
  rowptr[r] = (int32_t)nnz;
  return nnz;
}

/* stable counting sort by source column */
void oracle_csr_to_csc(int64_t rows, int32_t S, int32_t hs, const int32_t* rowptr, const int32_t* colidx,
                       const float* vals, int64_t ncols, int32_t* colptr, int32_t* zrow, int32_t* eid,
                       float* cvals) {
  const int64_t nnz = rowptr[rows * S];
  memset(colptr, 0, sizeof(int32_t) * (size_t)(ncols + 1));
  for (int64_t e = 0; e < nnz; ++e) colptr[colidx[e] + 1]++;
  for (int64_t c = 0; c < ncols; ++c) colptr[c + 1] += colptr[c];
  int32_t* cur = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ncols + 1));
  memcpy(cur, colptr, sizeof(int32_t) * (size_t)(ncols + 1));
  for (int64_t s = 0; s < rows * S; ++s) {
    const int64_t n = s / S, t = s % S;
    for (int32_t e = rowptr[s]; e < rowptr[s + 1]; ++e) {
      const int32_t o = cur[colidx[e]]++;
      zrow[o] = (int32_t)(n * (S + hs) + hs + t);
      eid[o] = e;
      if (cvals) cvals[o] = vals[e];
    }
  }
  free(cur);
}

/* ---------------- synthetic graphs (spec: include/grl.h GrlSynthSpec) ---- */
static inline uint64_t o_synth_bits(uint64_t seed, uint64_t k, uint32_t lane) {
  return o_mix64(o_mix64(seed + 0x243F6A8885A308D3ull * (uint64_t)(lane + 1)) ^ (k * 0x9E3779B97F4A7C15ull));
}

static void o_synth_edge(int kind, int L, int64_t N, int scale, uint64_t seed, uint64_t k, int64_t* src,
                         int64_t* dst, int* type) {
  const uint64_t h1 = o_synth_bits(seed, k, 1);
  *type = (int)(((h1 & 0xFFFFFFFFull) * (uint64_t)L) >> 32);
  if (kind == 0) {
    const uint64_t h0 = o_synth_bits(seed, k, 0);
    *src = (int64_t)(((h0 & 0xFFFFFFFFull) * (uint64_t)N) >> 32);
    *dst = (int64_t)(((h0 >> 32) * (uint64_t)N) >> 32);
  } else {
    /* R-MAT a,b,c,d = 0.57, 0.19, 0.19, 0.05: thresholds floor(x * 2^32) */
    const uint64_t A = 2448131358ull, AB = 3264175144ull, ABC = 4080218931ull;
    int64_t u = 0, v = 0;
    for (int lvl = 0; lvl < scale; ++lvl) {
      const uint64_t h = o_synth_bits(seed, k, 2 + (uint32_t)(lvl >> 1));
      const uint64_t r = (lvl & 1) ? (h >> 32) : (h & 0xFFFFFFFFull);
      const int q = r < A ? 0 : (r < AB ? 1 : (r < ABC ? 2 : 3));
      u = (u << 1) | (q >> 1);
      v = (v << 1) | (q & 1);
    }
    *src = u;
    *dst = v;
  }
}

static int o_cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : (x > y);
}

/* Returns nnz; rowptr [(re-rb)*L+1]; colidx capacity = candidates in range. */
int64_t oracle_synth(int32_t kind, int32_t L, int64_t N, int64_t C, uint64_t seed, int64_t rb, int64_t re,
                     int32_t* rowptr, int32_t* colidx, int64_t cap) {
  int scale = 0;
  if (kind == 1)
    while ((1LL << scale) < N) ++scale;
  uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(cap > 0 ? cap : 1));
  int64_t cnt = 0;
  /* the candidate scan runs in parallel; the keys are sorted afterwards, so
     the insertion order (and hence the thread count) cannot matter */
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < C; ++k) {
    int64_t s, d;
    int t;
    o_synth_edge(kind, L, N, scale, seed, (uint64_t)k, &s, &d, &t);
    if (s >= rb && s < re) {
      int64_t slot;
#pragma omp atomic capture
      slot = cnt++;
      if (slot < cap) keys[slot] = ((uint64_t)(s - rb) * (uint64_t)L + (uint64_t)t) * (uint64_t)N + (uint64_t)d;
    }
  }
  if (cnt > cap) cnt = cap;
  qsort(keys, (size_t)cnt, sizeof(uint64_t), o_cmp_u64);
  int64_t nnz = 0;
  const int64_t nseg = (re - rb) * L;
  int64_t seg = 0;
  for (int64_t i = 0; i < cnt; ++i) {
    if (i > 0 && keys[i] == keys[i - 1]) continue;
    const int64_t s = (int64_t)(keys[i] / (uint64_t)N);
    while (seg <= s) rowptr[seg++] = (int32_t)nnz;
    colidx[nnz++] = (int32_t)(keys[i] % (uint64_t)N);
  }
  while (seg <= nseg) rowptr[seg++] = (int32_t)nnz;
  free(keys);
  return nnz;
}

int64_t oracle_synth_count(int32_t kind, int32_t L, int64_t N, int64_t C, uint64_t seed, int64_t rb, int64_t re) {
  int scale = 0;
  if (kind == 1)
    while ((1LL << scale) < N) ++scale;
  int64_t cnt = 0;
#pragma omp parallel for schedule(static) reduction(+ : cnt)
  for (int64_t k = 0; k < C; ++k) {
    int64_t s, d;
    int t;
    o_synth_edge(kind, L, N, scale, seed, (uint64_t)k, &s, &d, &t);
    cnt += (s >= rb && s < re);
  }
  return cnt;
}

int32_t oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
