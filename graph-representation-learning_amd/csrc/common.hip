// Library identity, thread-local error reporting, device queries and the
// path options.
#include <atomic>
#include <cstring>
#include <mutex>

#include "grl_internal.h"

namespace grl {
namespace {
thread_local char g_err[1024] = "";
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int device_cu_count() {
  // One process drives one GPU (torch.distributed one-rank-per-device), so the
  // current device's CU count is fixed for the life of the process.
  static int cached = 0;
  static std::once_flag once;
  std::call_once(once, [] {
    int dev = 0;
    int cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      cached = cus;
    else
      cached = 256;  // MI355X
  });
  return cached;
}

namespace {
struct OptDef {
  const char* name;
  int64_t def, lo, hi;
};
constexpr OptDef kOpts[OPT_COUNT] = {
    {"gemm_x6", 1, 0, 1},
    {"graphconv_fused", 1, 0, 1},
    {"graphconv_fused_bwd", 1, 0, 1},
    {"fg_ws", 1, 0, 1},
    {"spmm_wide", -1, -1, 1},
    {"spmm_blocks_per_cu", 24, 1, 64},
    {"attn_x6", 1, 0, 1},
    {"attn_fwd8", 1, 0, 1},
    {"attn_dh8", 1, 0, 1},
    {"attn_fused_dq", 1, 0, 1},
    {"attn_pipe", 1, 0, 1},
    {"attn_dh16", 1, 0, 1},
    {"attn_kq16", 1, 0, 1},
    {"attn_qslab_max", 0, 0, INT64_MAX},
    {"ws_spin", 0, 0, (int64_t)1 << 30},
    {"ws_status_sync", 0, 0, 1},
};
std::atomic<int64_t> g_opt[OPT_COUNT] = {
    {kOpts[0].def},  {kOpts[1].def},  {kOpts[2].def},  {kOpts[3].def},  {kOpts[4].def},
    {kOpts[5].def},  {kOpts[6].def},  {kOpts[7].def},  {kOpts[8].def},  {kOpts[9].def},
    {kOpts[10].def}, {kOpts[11].def}, {kOpts[12].def}, {kOpts[13].def}, {kOpts[14].def},
    {kOpts[15].def},
};
static_assert(OPT_COUNT == 16, "one default per option");

int find_opt(const char* name) {
  for (int i = 0; name && i < OPT_COUNT; ++i)
    if (strcmp(name, kOpts[i].name) == 0) return i;
  return -1;
}
}  // namespace

int64_t opt(GrlOpt o) { return g_opt[o].load(std::memory_order_relaxed); }

}  // namespace grl

extern "C" int grl_set_option(const char* name, int64_t value) {
  using namespace grl;
  const int i = find_opt(name);
  GRL_CHECK_ARG(i >= 0, "grl_set_option: unknown option '%s'", name ? name : "(null)");
  GRL_CHECK_ARG(value >= kOpts[i].lo && value <= kOpts[i].hi, "grl_set_option: %s = %lld outside [%lld, %lld]",
                name, (long long)value, (long long)kOpts[i].lo, (long long)kOpts[i].hi);
  g_opt[i].store(value, std::memory_order_relaxed);
  return GRL_OK;
}

extern "C" int grl_get_option(const char* name, int64_t* value) {
  using namespace grl;
  const int i = find_opt(name);
  GRL_CHECK_ARG(i >= 0, "grl_get_option: unknown option '%s'", name ? name : "(null)");
  GRL_CHECK_ARG(value != nullptr, "grl_get_option: null value pointer");
  *value = g_opt[i].load(std::memory_order_relaxed);
  return GRL_OK;
}

extern "C" const char* grl_version(void) { return "grl-mi355x 0.1.0 (gfx950)"; }

extern "C" const char* grl_last_error(void) { return grl::g_err; }
