// capi.hip — error reporting and device queries of the C ABI (include/tuplewise.h).
#include "tw_common.h"

namespace tw {
static thread_local char g_err[512] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tw

extern "C" const char* tw_last_error(void) { return tw::g_err; }
extern "C" int tw_version(void) { return 1; }
extern "C" int tw_device_count(int* out_count) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  if (out_count) *out_count = n;
  return TW_OK;
}
