// Library identity, thread-local error reporting and device queries.
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

}  // namespace grl

extern "C" const char* grl_version(void) { return "grl-mi355x 0.1.0 (gfx950)"; }

extern "C" const char* grl_last_error(void) { return grl::g_err; }
