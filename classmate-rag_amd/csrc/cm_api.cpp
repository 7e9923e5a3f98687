// Library-level C ABI: error reporting, version, device enumeration.
#include <hip/hip_ext.h>
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
// A stream whose kernels run only on the CUs set in cu_mask (n_words 32-bit words, bit i = CU i):
// lets a latency-bound side stream (BM25) keep off part of the chip while another stream runs.
int cm_stream_create_cu_masked(int device, const uint32_t *cu_mask, int n_words, void **out_stream) {
  if (!cu_mask || n_words <= 0 || !out_stream) CM_FAIL(CM_EINVAL, "cu_mask / n_words / out_stream");
  CM_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  CM_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, cu_mask));
  *out_stream = (void *)s;
  return CM_OK;
}
int cm_stream_destroy(void *stream) {
  if (stream) CM_HIP(hipStreamDestroy((hipStream_t)stream));
  return CM_OK;
}
}
