// Library-level C ABI: error reporting, version, device enumeration.
#include <hip/hip_runtime.h>

#include <string>

#include "cm_common.h"

namespace cm {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
}  // namespace cm

extern "C" {
const char *cm_last_error(void) { return cm::g_last_error.c_str(); }
int cm_version(void) { return 100; }  // 0.1.0
int cm_device_count(int *n) {
  if (!n) CM_FAIL(CM_EINVAL, "n is NULL");
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    CM_FAIL(CM_EDEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  return CM_OK;
}
}
