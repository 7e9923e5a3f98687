// Shared host/device helpers for libclassmate_hip (gfx950 only).
#pragma once
#include <cstdlib>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "classmate_hip.h"

namespace cm {

void set_error(const std::string &msg);

// Set the error message and return `code` from the enclosing API function.
#define CM_FAIL(code, msg)            \
  do {                                \
    ::cm::set_error(msg);             \
    return (code);                    \
  } while (0)

#define CM_HIP(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      ::cm::set_error(std::string("HIP error in ") + #expr + ": " + hipGetErrorString(_e)); \
      return CM_EDEVICE;                                                                     \
    }                                                                                        \
  } while (0)

// RAII: make `dev` current for the duration of an API call, restore after.
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Grow-only device buffer.
struct DevBuf {
  void *ptr = nullptr;
  size_t bytes = 0;
  int ensure(size_t need) {
    if (need <= bytes) return CM_OK;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    if (need == 0) return CM_OK;
    if (hipMalloc(&ptr, need) != hipSuccess) {
      set_error("hipMalloc failed for " + std::to_string(need) + " bytes");
      return CM_ENOMEM;
    }
    bytes = need;
    return CM_OK;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  template <typename T>
  T *as() const {
    return reinterpret_cast<T *>(ptr);
  }
};

// Orderable encodings so that an unsigned integer compare gives the float order.
__host__ __device__ inline uint32_t f32_order(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float f32_unorder(uint32_t u) {
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __builtin_bit_cast(float, u);
}
__host__ __device__ inline uint64_t f64_order(double d) {
  uint64_t u = __builtin_bit_cast(uint64_t, d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__host__ __device__ inline double f64_unorder(uint64_t u) {
  u = (u & 0x8000000000000000ull) ? (u & 0x7fffffffffffffffull) : ~u;
  return __builtin_bit_cast(double, u);
}

// Optional per-handle kernel timer: HIP events recorded on the launch stream
// around the dominant kernel of each search (bench roofline); drained after a sync.
struct KernelTimer {
  bool on = false, armed = false;
  std::vector<hipEvent_t> ev;  // begin/end pairs
  size_t used = 0;
  void begin(hipStream_t st) {
    armed = false;
    if (!on) return;
    grow();
    armed = ev.size() >= used + 2 && hipEventRecord(ev[used], st) == hipSuccess;
  }
  void end(hipStream_t st) {
    if (!armed) return;
    armed = false;
    if (hipEventRecord(ev[used + 1], st) == hipSuccess) used += 2;
  }
  void grow() {
    while (ev.size() < used + 2) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return;
      ev.push_back(e);
    }
  }
  // elapsed ms of the recorded pairs (up to cap) -> out; returns the pair count or < 0
  int drain(float *out, int cap) {
    int n = 0;
    for (size_t i = 0; i + 1 < used; i += 2) {
      if (hipEventSynchronize(ev[i + 1]) != hipSuccess) return CM_EDEVICE;
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, ev[i], ev[i + 1]) != hipSuccess) return CM_EDEVICE;
      if (n < cap && out) out[n] = ms;
      ++n;
    }
    used = 0;
    return n;
  }
  void release() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    ev.clear();
    used = 0;
  }
};

// K10 split planes (cm_gemm.hip): fp32 v = hi + lo as two f16 halves.  An M x K matrix is one
// buffer of 2 KiB "split blocks": block (row / 16, k / 32) = [hi 1 KiB][lo 1 KiB], each half in
// fragment-major order (lane slot (row % 16) + 16 ((k % 32) / 8), 8 halves of k).  Offset (in
// halves) of the hi element; the lo element is 512 halves after it.  Buffers hold
// f16x3_plane_rows(M) rows (a multiple of every K10 tile height: the last tile reads no clamp).
constexpr int64_t kF16x3RowAlign = 384;
__host__ __device__ inline int64_t f16x3_plane_rows(int64_t M) {
  return (M + kF16x3RowAlign - 1) / kF16x3RowAlign * kF16x3RowAlign;
}
__host__ __device__ inline int64_t f16x3_plane_off(int64_t row, int k, int kb32) {
  return (((row >> 4) * kb32 + (k >> 5)) * 128 + (row & 15) + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
}
__device__ inline void f16x3_split1(float a, _Float16 &h, _Float16 &l) {
  h = (_Float16)a;
  l = (_Float16)(a - (float)h);
}
// the same split of two values, returned as packed pairs (element a in the low half): the
// conversions run as v_cvt_pk_f16_f32 (round to nearest even, like the scalar form: equal bits)
__device__ inline void f16x3_split2(float a, float b, uint32_t &hi, uint32_t &lo) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  const h2 h = __builtin_convertvector(v, h2);
  const h2 l = __builtin_convertvector(v - __builtin_convertvector(h, f2), h2);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}

constexpr uint64_t kEmptyKey = ~0ull;
constexpr int kMaxTopK = 256;

// A/B knob read at every launch (not cached: a benchmark flips it between measurements in one
// process): unset -> dflt, "0" -> false, anything else -> true
inline bool env_knob(const char *name, bool dflt) {
  const char *e = getenv(name);
  return e ? e[0] != '0' : dflt;
}

}  // namespace cm
