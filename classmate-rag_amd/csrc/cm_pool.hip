// E5 sentence embedding epilogue (K6): masked mean over tokens + L2 normalise.
// Mirrors sentence-transformers Pooling(mean) + Normalize as invoked by
// E5MultilingualEmbedder.encode_* (rag/embeddings/__init__.py:85-105):
//   mean = sum_s h[s]*m[s] / max(sum_s m[s], 1e-9);  out = mean / max(||mean||, 1e-12)
// One workgroup per sequence; each lane owns 4 consecutive features and reads
// them with one 8-byte (bf16/f16) or 16-byte (f32) load per token, so a token
// row is one coalesced sweep.  fp32 accumulation.  HBM-bound: bytes per
// sequence = S*D*sizeof(h) + S*sizeof(mask) + D*4.
#include "cm_common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace cm {

constexpr int kPoolThreads = 256;

template <typename T>
__device__ inline void load4(const T *p, float (&v)[4]);
template <>
__device__ inline void load4<float>(const float *p, float (&v)[4]) {
  const float4 x = *reinterpret_cast<const float4 *>(p);
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
template <>
__device__ inline void load4<__hip_bfloat16>(const __hip_bfloat16 *p, float (&v)[4]) {
  const uint2 x = *reinterpret_cast<const uint2 *>(p);
  v[0] = __uint_as_float(x.x << 16);
  v[1] = __uint_as_float(x.x & 0xffff0000u);
  v[2] = __uint_as_float(x.y << 16);
  v[3] = __uint_as_float(x.y & 0xffff0000u);
}
template <>
__device__ inline void load4<__half>(const __half *p, float (&v)[4]) {
  const uint2 x = *reinterpret_cast<const uint2 *>(p);
  v[0] = __half2float(__ushort_as_half((unsigned short)(x.x & 0xffff)));
  v[1] = __half2float(__ushort_as_half((unsigned short)(x.x >> 16)));
  v[2] = __half2float(__ushort_as_half((unsigned short)(x.y & 0xffff)));
  v[3] = __half2float(__ushort_as_half((unsigned short)(x.y >> 16)));
}

template <typename T, typename M>
__global__ void __launch_bounds__(kPoolThreads) meanpool_l2norm_kernel(const T *__restrict__ h, const M *__restrict__ mask,
                                                                       int S, int D, int normalize,
                                                                       float *__restrict__ out) {
  const int b = blockIdx.x;
  const T *hb = h + (int64_t)b * S * D;
  const M *mb = mask + (int64_t)b * S;
  __shared__ float red[kPoolThreads / 64];
  __shared__ float msum_s;
  // mask sum (same for all features)
  float ms = 0.f;
  for (int s = threadIdx.x; s < S; s += kPoolThreads) ms += (float)mb[s];
  for (int o = 32; o > 0; o >>= 1) ms += __shfl_xor(ms, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ms;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < kPoolThreads / 64; ++w) t += red[w];
    msum_s = fmaxf(t, 1e-9f);
  }
  __syncthreads();
  const float msum = msum_s;
  const int D4 = D / 4;
  float sq = 0.f;
  constexpr int kPer = 4;  // D <= 4096
  float acc[kPer][4];
#pragma unroll
  for (int u = 0; u < kPer; ++u) acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0.f;
  for (int s = 0; s < S; ++s) {
    const float m = (float)mb[s];
    if (m == 0.f) continue;  // uniform across the block
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int c = threadIdx.x + u * kPoolThreads;
      if (c < D4) {
        float v[4];
        load4<T>(hb + (int64_t)s * D + 4 * c, v);
        acc[u][0] += v[0] * m;
        acc[u][1] += v[1] * m;
        acc[u][2] += v[2] * m;
        acc[u][3] += v[3] * m;
      }
    }
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    for (int e = 0; e < 4; ++e) {
      acc[u][e] = acc[u][e] / msum;
      sq += acc[u][e] * acc[u][e];
    }
  float inv = 1.f;
  if (normalize) {
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < kPoolThreads / 64; ++w) t += red[w];
    inv = 1.f / fmaxf(sqrtf(t), 1e-12f);
  }
  float *ob = out + (int64_t)b * D;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int c = threadIdx.x + u * kPoolThreads;
    if (c < D4) {
      float4 r;
      r.x = acc[u][0] * inv; r.y = acc[u][1] * inv; r.z = acc[u][2] * inv; r.w = acc[u][3] * inv;
      *reinterpret_cast<float4 *>(ob + 4 * c) = r;
    }
  }
}

template <typename T>
int launch_pool(const void *h, const void *m, int mdt, int B, int S, int D, int nz, float *out, hipStream_t st) {
  if (mdt == CM_DTYPE_I32)
    hipLaunchKernelGGL((meanpool_l2norm_kernel<T, int32_t>), dim3(B), dim3(kPoolThreads), 0, st,
                       (const T *)h, (const int32_t *)m, S, D, nz, out);
  else
    hipLaunchKernelGGL((meanpool_l2norm_kernel<T, int64_t>), dim3(B), dim3(kPoolThreads), 0, st,
                       (const T *)h, (const int64_t *)m, S, D, nz, out);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

}  // namespace cm

using namespace cm;

extern "C" int cm_meanpool_l2norm(const void *hidden_dev, int32_t hidden_dtype, const void *mask_dev,
                                  int32_t mask_dtype, int32_t B, int32_t S, int32_t D, int32_t normalize,
                                  float *out_dev, void *stream) {
  if (B <= 0) return CM_OK;
  if (!hidden_dev || !mask_dev || !out_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (S <= 0 || D <= 0 || D % 4 != 0 || D > 4 * 4 * kPoolThreads) CM_FAIL(CM_EINVAL, "D must be a multiple of 4, <= 4096");
  if (mask_dtype != CM_DTYPE_I32 && mask_dtype != CM_DTYPE_I64) CM_FAIL(CM_EINVAL, "mask dtype must be int32/int64");
  hipStream_t st = (hipStream_t)stream;
  switch (hidden_dtype) {
    case CM_DTYPE_F32: return launch_pool<float>(hidden_dev, mask_dev, mask_dtype, B, S, D, normalize, out_dev, st);
    case CM_DTYPE_BF16: return launch_pool<__hip_bfloat16>(hidden_dev, mask_dev, mask_dtype, B, S, D, normalize, out_dev, st);
    case CM_DTYPE_F16: return launch_pool<__half>(hidden_dev, mask_dev, mask_dtype, B, S, D, normalize, out_dev, st);
    default: CM_FAIL(CM_EINVAL, "hidden dtype must be f32/bf16/f16");
  }
}
