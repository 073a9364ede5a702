// capi.hip — error reporting, device queries and host-memory mapping of the C ABI
// (include/tuplewise.h).
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

// The device address of pinned (page-locked, mapped) host memory, so a kernel can read a
// staging buffer the host filled without a separate copy call (the replay loop's draws).
// TW_ERR_ARG when the pointer is not device-accessible host memory.
extern "C" int tw_host_device_pointer(void* host, void** out_dev) {
  TW_ARG_CHECK(host != nullptr && out_dev != nullptr, "tw_host_device_pointer: null");
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
  if (e != hipSuccess || d == nullptr) {
    (void)hipGetLastError();
    tw::set_error("tw_host_device_pointer: not mapped host memory (%s)", hipGetErrorString(e));
    return TW_ERR_ARG;
  }
  *out_dev = d;
  return TW_OK;
}
