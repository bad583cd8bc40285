// Error plumbing + library identity for libmrg.so.
#include "mrg_common.h"
#include <cstdarg>

namespace mrg {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mrg

MRG_API const char* mrg_last_error(void) { return mrg::g_err; }

MRG_API int mrg_version(void) { return 100; }

// Device query used by the host side to size persistent grids.
MRG_API int mrg_device_cu_count(int device, int* out) {
  hipDeviceProp_t p;
  MRG_HIP(hipGetDeviceProperties(&p, device));
  *out = p.multiProcessorCount;
  return 0;
}
