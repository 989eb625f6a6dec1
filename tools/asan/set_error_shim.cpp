// ASan build of layout_graph.cpp alone: the thread-local error channel that
// libgrl's common.hip provides (grl_last_error), restated for host code.
#include <cstdarg>
#include <cstdio>

namespace grl {
thread_local char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
}  // namespace grl

extern "C" const char* grl_last_error(void) { return grl::g_err; }
