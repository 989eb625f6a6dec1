// Internal helpers shared by the gfx950 translation units of libgrl.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>

#include "grl.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace grl {

// ---- thread-local error string (grl_last_error) --------------------------
void set_error(const char* fmt, ...);

#define GRL_FAIL(code, ...)          \
  do {                               \
    ::grl::set_error(__VA_ARGS__);   \
    return (code);                   \
  } while (0)

#define GRL_CHECK_ARG(cond, ...)                         \
  do {                                                   \
    if (!(cond)) GRL_FAIL(GRL_E_INVALID, __VA_ARGS__);   \
  } while (0)

#define GRL_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess)                                                    \
      GRL_FAIL(GRL_E_HIP, "%s failed: %s (%s:%d)", #call,                    \
               hipGetErrorString(_e), __FILE__, __LINE__);                   \
  } while (0)

// Launch-error check after <<<>>> (no device sync: stream-ordered API).
#define GRL_LAUNCH_CHECK() GRL_HIP(hipGetLastError())

inline hipStream_t as_stream(grl_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// ---- DropEdge counter hash -------------------------------------------------
// splitmix64 finalizer (Steele, Lea, Flood 2014).  The same function is
// restated independently in oracle/grl_oracle.c and oracle/hash.py.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

__host__ __device__ __forceinline__ uint64_t dropedge_key(uint64_t seed, uint64_t call) {
  return mix64(mix64(seed ^ 0x6A09E667F3BCC909ull) + call * 0x9E3779B97F4A7C15ull);
}

__host__ __device__ __forceinline__ uint32_t dropedge_bits(uint64_t key, uint64_t id) {
  return static_cast<uint32_t>(mix64(key ^ (id * 0xD1B54A32D192ED03ull)) >> 32);
}

// Synthetic-graph candidate hash: 64 random bits for (seed, candidate, lane).
__host__ __device__ __forceinline__ uint64_t synth_bits(uint64_t seed, uint64_t k, uint32_t lane) {
  return mix64(mix64(seed + 0x243F6A8885A308D3ull * (uint64_t)(lane + 1)) ^ (k * 0x9E3779B97F4A7C15ull));
}

// Row-range typed-SpMM forward (spmm.hip) used by grl_graphconv_fwd.
int spmm_fwd_rows(const GrlTypedCsr* g, int64_t r0, int64_t rows, const float* X, int64_t ldx, int F, float* Z,
                  const GrlDropEdge* de, hipStream_t st);

// Fused one-kernel GraphConv forward (graphconv.hip), used by grl_graphconv_fwd.
bool graphconv_fused_enabled();
bool graphconv_fused_shape_ok(int F, int C, int L);
size_t graphconv_fused_ws_bytes(int64_t K, int C);
int graphconv_fused_fwd(const GrlTypedCsr* g, const float* X, int64_t ldx, int F, const float* W, const float* bias,
                        int C, int relu, float* out, const GrlDropEdge* de, void* ws, hipStream_t st,
                        float* Z = nullptr);
int graphconv_fused_bwd_data(const GrlTypedCsr* gt, const int32_t* eid, const float* G, int64_t ldg, int64_t self_rows,
                             int Cin, const float* W, int Cout, float* dX, float* Gagg, const GrlDropEdge* de, void* ws,
                             hipStream_t st);

// Plain-data copy of GrlDropEdge passed by value to kernels.
struct DropDev {
  uint64_t key;
  uint32_t threshold;
  float scale;
  int32_t active;
  int32_t drop_self;
  const uint64_t* seed_dev;  // non-null: key = dropedge_key(*seed_dev, call) (resolve_key)
  uint64_t call;
};

inline DropDev to_dev(const GrlDropEdge* de) {
  DropDev d{0, 0, 1.0f, 0, 0, nullptr, 0};
  if (de && de->active) {
    d.key = de->key;
    d.threshold = de->threshold;
    d.scale = de->scale;
    d.active = 1;
    d.drop_self = de->drop_self;
    d.seed_dev = de->seed_dev;
    d.call = de->call_id;
  }
  return d;
}

// Device-resident seed: every kernel taking a DropDev resolves its key once
// at entry (one uniform 8-byte load; a graph replay sees the seed written
// before it on the same stream).
__device__ __forceinline__ DropDev resolve_key(DropDev d) {
  if (d.active && d.seed_dev) d.key = dropedge_key(*d.seed_dev, d.call);
  return d;
}

// weight of an entry with value v and global id `id` under DropEdge d
__device__ __forceinline__ float dropedge_weight(const DropDev& d, float v, uint64_t id) {
  if (!d.active) return v;
  return dropedge_bits(d.key, id) >= d.threshold ? v * d.scale : 0.0f;
}

__device__ __forceinline__ int readlane_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float readlane_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// roctx range around a C-ABI entry point: `rocprofv3 --marker-trace` shows
// where host time goes between kernels (a no-op call without a profiler).
struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

// Number of CUs of the current device (cached per process).
int device_cu_count();

// Path options (grl_set_option / grl_get_option, include/grl.h): the test and
// A/B hooks that select among kernel forms of one entry point.  Defaults are
// the production choices; nothing in the library reads the environment.
enum GrlOpt {
  OPT_GEMM_X6,              // 1: split-bf16 (x6) GEMMs where sized for them; 0: fp32-MFMA kernels
  OPT_GRAPHCONV_FUSED,      // 1: one-kernel GraphConv forward where eligible; 0: SpMM + GEMM
  OPT_GRAPHCONV_FUSED_BWD,  // 1: one-kernel GraphConv data gradient (read by the host layer)
  OPT_FG_WS,                // 1: persistent warp-specialized one-kernel form; 0: phase-alternating
  OPT_SPMM_WIDE,            // -1: whole-row waves for tables > 12 GB; 1 / 0: always / never
  OPT_SPMM_BLOCKS_PER_CU,   // SpMM workgroups per CU (24)
  OPT_ATTN_X6,              // 1: x6 attention kernels; 0: fp32-MFMA kernels
  OPT_ATTN_FWD8,            // 1: 8-wave pipelined forward; 0: 4-wave
  OPT_ATTN_DH8,             // 1: 8-wave dH pass; 0: 4-wave
  OPT_ATTN_FUSED_DQ,        // 1: dQ folded into the dK pass; 0: separate dQ kernel
  OPT_ATTN_PIPE,            // 1: software-pipelined x6 forward; 0: unpipelined
  OPT_ATTN_DH16,            // 1: dH pass on 16x16x32 MFMAs (dk <= 16; default); 0: the 32x32x16 kernel
  OPT_ATTN_KQ16,            // 1: fused dK/dQ pass on 16x16x32 MFMAs (dk <= 16; default); 0: the 32x32x16 kernel
  OPT_ATTN_QSLAB_MAX,       // fused dK/dQ slab budget in bytes (0: 24 GiB)
  OPT_WS_SPIN,              // persistent kernels' bounded-wait limit (0: 2^24 sleeps)
  OPT_WS_STATUS_SYNC,       // 1: an eager one-kernel call checks its own status (debug)
  OPT_COUNT
};
int64_t opt(GrlOpt o);

}  // namespace grl
