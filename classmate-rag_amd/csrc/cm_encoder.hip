// E5 (XLM-R) encoder epilogue fused for the query/passage encode:
//   out[row] = LayerNorm(round_T(x[row] + r[row % r_rows])) * gamma + beta
// i.e. the "residual add, then LayerNorm" that closes every attention and MLP block of
// XLM-R (and the embeddings' word + position/type sum).  torch runs it as two kernels
// (an elementwise add that writes the sum back to HBM, then the LayerNorm that reads it
// again); here one wave owns one row, keeps it in registers and touches HBM once per
// operand: bytes per row = (2 + [r]) * D * sizeof(T) + gamma/beta (L2-resident).
// The sum is rounded to T before the statistics, as torch's `x + r` is, and the
// statistics are fp32 two-pass (mean, then sum of squared deviations) from registers.
#include "cm_common.h"

#include <hip/hip_bf16.h>

namespace cm {

constexpr int kLnWaves = 4;   // rows per workgroup
constexpr int kLnMaxPer = 8;  // 4-feature chunks per lane -> D <= 2048

__device__ inline void ln_load4(const float *p, float (&v)[4]) {
  const float4 x = *reinterpret_cast<const float4 *>(p);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
__device__ inline void ln_load4(const __hip_bfloat16 *p, float (&v)[4]) {
  const uint2 x = *reinterpret_cast<const uint2 *>(p);
  v[0] = __uint_as_float(x.x << 16);
  v[1] = __uint_as_float(x.x & 0xffff0000u);
  v[2] = __uint_as_float(x.y << 16);
  v[3] = __uint_as_float(x.y & 0xffff0000u);
}
__device__ inline float ln_round(float f, float) { return f; }
__device__ inline float ln_round(float f, __hip_bfloat16) { return __bfloat162float(__float2bfloat16(f)); }
__device__ inline void ln_store4(float *p, const float (&v)[4]) {
  *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ inline uint32_t bf16_bits(float f) {
  return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(f));
}
__device__ inline void ln_store4(__hip_bfloat16 *p, const float (&v)[4]) {
  uint2 o;
  o.x = bf16_bits(v[0]) | (bf16_bits(v[1]) << 16);
  o.y = bf16_bits(v[2]) | (bf16_bits(v[3]) << 16);
  *reinterpret_cast<uint2 *>(p) = o;
}

template <typename T, int PER>
__global__ void __launch_bounds__(64 * kLnWaves)
    add_layernorm_kernel(const T *x, const T *__restrict__ r, int64_t r_rows, const T *__restrict__ gamma,
                         const T *__restrict__ beta, int64_t rows, int D, float eps, T *out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= rows) return;  // whole wave exits together
  const int D4 = D >> 2;
  const T *xr = x + row * D;
  const T *rr = r ? r + (row % r_rows) * D : nullptr;
  float v[PER][4];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = lane + 64 * u;
    if (c < D4) {
      ln_load4(xr + 4 * c, v[u]);
      if (rr) {
        float w[4];
        ln_load4(rr + 4 * c, w);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[u][e] = ln_round(v[u][e] + w[e], T());
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) s += v[u][e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = 0.f;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)D;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = lane + 64 * u;
    if (c < D4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[u][e] - mean;
        q += d * d;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = rsqrtf(q / (float)D + eps);
  T *orow = out + row * D;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = lane + 64 * u;
    if (c < D4) {
      float g[4], b[4], y[4];
      ln_load4(gamma + 4 * c, g);
      ln_load4(beta + 4 * c, b);
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (v[u][e] - mean) * rstd * g[e] + b[e];
      ln_store4(orow + 4 * c, y);
    }
  }
}

template <typename T>
int launch_add_ln(const void *x, const void *r, int64_t r_rows, const void *g, const void *b, int64_t rows, int D,
                  float eps, void *out, hipStream_t st) {
  const int per = (int)ceil_div(D / 4, 64);
  const dim3 grid((unsigned)ceil_div(rows, kLnWaves)), block(64 * kLnWaves);
#define CM_LN_CASE(P)                                                                                          \
  case P:                                                                                                       \
    hipLaunchKernelGGL((add_layernorm_kernel<T, P>), grid, block, 0, st, (const T *)x, (const T *)r, r_rows, \
                       (const T *)g, (const T *)b, rows, D, eps, (T *)out);                                   \
    break;
  switch (per) {
    CM_LN_CASE(1)
    CM_LN_CASE(2)
    CM_LN_CASE(3)
    CM_LN_CASE(4)
    CM_LN_CASE(6)
    CM_LN_CASE(8)
    case 5:
      hipLaunchKernelGGL((add_layernorm_kernel<T, 6>), grid, block, 0, st, (const T *)x, (const T *)r, r_rows,
                         (const T *)g, (const T *)b, rows, D, eps, (T *)out);
      break;
    default:
      hipLaunchKernelGGL((add_layernorm_kernel<T, 8>), grid, block, 0, st, (const T *)x, (const T *)r, r_rows,
                         (const T *)g, (const T *)b, rows, D, eps, (T *)out);
  }
#undef CM_LN_CASE
  CM_HIP(hipGetLastError());
  return CM_OK;
}

}  // namespace cm

using namespace cm;

extern "C" int cm_add_layernorm(const void *x_dev, const void *r_dev, int64_t r_rows, const void *gamma_dev,
                                const void *beta_dev, int64_t rows, int32_t D, float eps, int32_t dtype, void *out_dev,
                                void *stream) {
  if (rows <= 0) return CM_OK;
  if (!x_dev || !gamma_dev || !beta_dev || !out_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (D <= 0 || D % 4 != 0 || D > 4 * 64 * kLnMaxPer) CM_FAIL(CM_EINVAL, "D must be a multiple of 4, <= 2048");
  if (r_dev && r_rows <= 0) CM_FAIL(CM_EINVAL, "r_rows must be > 0 with a residual");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case CM_DTYPE_F32: return launch_add_ln<float>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, st);
    case CM_DTYPE_BF16:
      return launch_add_ln<__hip_bfloat16>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, st);
    default: CM_FAIL(CM_EINVAL, "dtype must be f32/bf16");
  }
}
