// Library-level entry points: version, thread-local error message, device check.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/rsys_hip.h"

namespace rs {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace rs

extern "C" int rs_version(void) { return 1; }

extern "C" const char* rs_last_error(void) { return rs::g_err; }

extern "C" int rs_device_check(void) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    rs::set_error("hipGetDevice: %s", hipGetErrorString(e));
    return (int)e;
  }
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) {
    rs::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    rs::set_error("device %d is %s, librsys_hip is built for gfx950 only", dev, prop.gcnArchName);
    return -1;
  }
  return 0;
}
