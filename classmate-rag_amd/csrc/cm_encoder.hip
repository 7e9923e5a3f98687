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

// SPLIT (fp32 only): also write the row as K10 split planes (hi/lo f16 halves of y * a_scale,
// fragment-major, cm_common.h f16x3_plane_off): the next projection's operand, so the GEMM
// streams it with LDS-DMA and does no conversion work.  A lane's 4 features are 8 bytes of one
// lane slot of a plane block.
template <typename T, int PER, bool SPLIT = false>
__global__ void __launch_bounds__(64 * kLnWaves)
    add_layernorm_kernel(const T *x, const T *__restrict__ r, int64_t r_rows, const T *__restrict__ gamma,
                         const T *__restrict__ beta, int64_t rows, int D, float eps, T *out, float a_scale = 1.f,
                         _Float16 *__restrict__ ph = nullptr) {
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
      if constexpr (SPLIT) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        h4 hh, ll;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          _Float16 a, b2;
          f16x3_split1(y[e] * a_scale, a, b2);
          hh[e] = a;
          ll[e] = b2;
        }
        const int64_t off = f16x3_plane_off(row, 4 * c, D >> 5);
        *reinterpret_cast<h4 *>(ph + off) = hh;
        *reinterpret_cast<h4 *>(ph + off + 512) = ll;
      }
    }
  }
}

// K8 with the planes written per 16-row block: a workgroup of 16 waves takes one row block (a row per
// wave, as add_layernorm_kernel: in registers, fp32 two-pass statistics, fp32 rows stored directly),
// stages the block's hi / lo halves in LDS in the plane order and then writes the block's D / 32
// split blocks -- one contiguous 64 D-byte run -- with 16-byte stores across the workgroup, instead
// of every lane storing 8-byte pieces 256 B apart.  Same values, bit for bit.  Ingest shape (65536
// rows): 216 -> 135 us per call (5.97 TB/s); query batch (6144 rows) within noise
// (profiles/r05_ln_ab.txt).
template <int PER>
__global__ void __launch_bounds__(1024)
    add_layernorm_split_rb_kernel(const float *x, const float *__restrict__ r, int64_t r_rows,
                                  const float *__restrict__ gamma, const float *__restrict__ beta, int64_t rows, int D,
                                  float eps, float *out, float a_scale, _Float16 *__restrict__ ph) {
  extern __shared__ __attribute__((aligned(16))) _Float16 stage[];   // [kb][hi/lo][slot 64][8]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t rb = blockIdx.x;
  const int D4 = D >> 2;
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const int rr = wave;
  const int64_t row = rb * 16 + rr;
  const bool live = row < rows;                        // rows past the end: zero planes (buffer padding)
  const float *xr = x + row * D;
  const float *rrow = r ? r + (row % r_rows) * D : nullptr;
  float v[PER][4];
  float sum = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = lane + 64 * u;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[u][e] = 0.f;
    if (live && c < D4) {
      ln_load4(xr + 4 * c, v[u]);
      if (rrow) {
        float w[4];
        ln_load4(rrow + 4 * c, w);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[u][e] = v[u][e] + w[e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) sum += v[u][e];
    }
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  const float mean = sum / (float)D;
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
  float *orow = out + row * D;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int c = lane + 64 * u;
    if (c < D4) {
      float y[4] = {0.f, 0.f, 0.f, 0.f};
      if (live) {
        float g[4], b[4];
        ln_load4(gamma + 4 * c, g);
        ln_load4(beta + 4 * c, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = (v[u][e] - mean) * rstd * g[e] + b[e];
        ln_store4(orow + 4 * c, y);
      }
      h4 hh, ll;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        _Float16 a, b2;
        f16x3_split1(y[e] * a_scale, a, b2);
        hh[e] = a;
        ll[e] = b2;
      }
      const int k = 4 * c, so = (((k >> 5) * 2) * 64 + rr + 16 * ((k & 31) >> 3)) * 8 + (k & 7);
      *reinterpret_cast<h4 *>(stage + so) = hh;
      *reinterpret_cast<h4 *>(stage + so + 512) = ll;
    }
  }
  __syncthreads();
  const int n16 = 4 * D;                               // 16-byte pieces of the row block's planes
  uint4 *dst = reinterpret_cast<uint4 *>(ph + rb * (int64_t)(D >> 5) * 1024);
  const uint4 *src = reinterpret_cast<const uint4 *>(stage);
  for (int i = threadIdx.x; i < n16; i += 1024) dst[i] = src[i];
}

template <int PER>
int launch_add_ln_split(const float *x, const float *r, int64_t r_rows, const float *g, const float *b, int64_t rows,
                        int D, float eps, float *out, float a_scale, _Float16 *ph, hipStream_t st) {
  if (env_knob("CM_LN_RB", true)) {   // planes per 16-row block (CM_LN_RB=0: per-lane pieces, A/B)
    const size_t lds = (size_t)64 * D;
    if (lds > 64 * 1024)
      CM_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&add_layernorm_split_rb_kernel<PER>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((add_layernorm_split_rb_kernel<PER>), dim3((unsigned)ceil_div(rows, 16)), dim3(1024),
                       lds, st, x, r, r_rows, g, b, rows, D, eps, out, a_scale, ph);
    CM_HIP(hipGetLastError());
    return CM_OK;
  }
  const dim3 grid((unsigned)ceil_div(rows, kLnWaves)), block(64 * kLnWaves);
  hipLaunchKernelGGL((add_layernorm_kernel<float, PER, true>), grid, block, 0, st, x, r, r_rows, g, b, rows, D, eps,
                     out, a_scale, ph);
  CM_HIP(hipGetLastError());
  return CM_OK;
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

// Short-sequence self-attention for the unpadded query encode (XLM-R, S <= 64, head dim 64):
// reads Q/K/V straight from the fused QKV GEMM output (B, S, 3, H, 64) and writes the
// context in (B, S, H*64) — the layout the output projection consumes — so the permute /
// transpose copies around torch's SDPA disappear.  One wave per (sequence, head); lane i
// owns query row i: its q row in registers, K and V rows of the head staged in LDS (read as
// broadcasts), fp32 online softmax.  bytes per (b, h) = 4*S*64*sizeof(T) (q, k, v in, o out).
constexpr int kAttnDh = 64;
constexpr int kAttnMaxS = 64;

__device__ inline void ld8(const float *p, float (&v)[8]) {
  ln_load4(p, *reinterpret_cast<float(*)[4]>(&v[0]));
  ln_load4(p + 4, *reinterpret_cast<float(*)[4]>(&v[4]));
}
__device__ inline void ld8(const __hip_bfloat16 *p, float (&v)[8]) {
  const uint4 x = *reinterpret_cast<const uint4 *>(p);
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}

// SPLIT (fp32): write the context as K10 split planes of o * a_scale (the O projection's
// operand) instead of fp32 rows: 8 features = one 16-byte lane slot per plane.
template <typename T, bool SPLIT = false>
__global__ void __launch_bounds__(64) short_attention_kernel(const T *__restrict__ qkv, int S, int H, float scale,
                                                             T *__restrict__ out, float a_scale = 1.f,
                                                             _Float16 *__restrict__ ph = nullptr) {
  constexpr int VPR = kAttnDh * sizeof(T) / 16;  // 16-byte vectors per head row
  __shared__ __attribute__((aligned(16))) T ks[kAttnMaxS * kAttnDh];
  __shared__ __attribute__((aligned(16))) T vs[kAttnMaxS * kAttnDh];
  const int lane = threadIdx.x;
  const int h = blockIdx.x % H;
  const int64_t b = blockIdx.x / H;
  const int64_t tok_stride = 3LL * H * kAttnDh;
  const T *base = qkv + b * S * tok_stride + (int64_t)h * kAttnDh;
  // stage K and V rows of this head: S * VPR 16-byte vectors each
  for (int t = lane; t < S * VPR; t += 64) {
    const int s = t / VPR, v = t % VPR;
    const uint4 *ksrc = reinterpret_cast<const uint4 *>(base + s * tok_stride + (int64_t)H * kAttnDh) + v;
    const uint4 *vsrc = reinterpret_cast<const uint4 *>(base + s * tok_stride + 2LL * H * kAttnDh) + v;
    reinterpret_cast<uint4 *>(ks)[t] = *ksrc;
    reinterpret_cast<uint4 *>(vs)[t] = *vsrc;
  }
  __syncthreads();
  if (lane >= S) return;
  float q[kAttnDh], acc[kAttnDh];
  const T *qrow = base + lane * tok_stride;
#pragma unroll
  for (int c = 0; c < kAttnDh / 8; ++c) {
    float t8[8];
    ld8(qrow + 8 * c, t8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      q[8 * c + e] = t8[e] * scale;
      acc[8 * c + e] = 0.f;
    }
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < S; ++j) {
    float sc = 0.f;
#pragma unroll
    for (int c = 0; c < kAttnDh / 8; ++c) {
      float k8[8];
      ld8(ks + j * kAttnDh + 8 * c, k8);
#pragma unroll
      for (int e = 0; e < 8; ++e) sc += q[8 * c + e] * k8[e];
    }
    const float mn = fmaxf(m, sc);
    const float corr = __expf(m - mn);
    const float p = __expf(sc - mn);
    l = l * corr + p;
    m = mn;
#pragma unroll
    for (int c = 0; c < kAttnDh / 8; ++c) {
      float v8[8];
      ld8(vs + j * kAttnDh + 8 * c, v8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[8 * c + e] = acc[8 * c + e] * corr + p * v8[e];
    }
  }
  const float inv = 1.f / l;
  if constexpr (SPLIT) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const int64_t row = b * S + lane;
    const int kb32 = H * kAttnDh / 32;
#pragma unroll
    for (int c = 0; c < kAttnDh / 8; ++c) {
      h8 hh, ll;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 a, b2;
        f16x3_split1(acc[8 * c + e] * inv * a_scale, a, b2);
        hh[e] = a;
        ll[e] = b2;
      }
      const int64_t off = f16x3_plane_off(row, h * kAttnDh + 8 * c, kb32);
      *reinterpret_cast<h8 *>(ph + off) = hh;
      *reinterpret_cast<h8 *>(ph + off + 512) = ll;
    }
  } else {
    T *orow = out + (b * S + lane) * (int64_t)H * kAttnDh + (int64_t)h * kAttnDh;
#pragma unroll
    for (int c = 0; c < kAttnDh / 4; ++c) {
      float y[4] = {acc[4 * c] * inv, acc[4 * c + 1] * inv, acc[4 * c + 2] * inv, acc[4 * c + 3] * inv};
      ln_store4(orow + 4 * c, y);
    }
  }
}

// bf16, S <= 32: the same attention on the matrix cores.  Per (sequence, head) one wave runs
// S^T = K Q^T as 2x2 tiles of v_mfma_f32_16x16x32_bf16 (K = head dim 64 in two steps), the
// softmax over keys on the accumulators (a query is one lane column: 8 registers x 4 lane
// groups, two xor-shuffles), and O = P V as one K=32 MFMA per output tile: the S^T
// accumulator layout (col = query on the lane, rows = keys in registers) IS the A-operand
// layout of P once the key order inside the K=32 reduction is permuted — key slot (g, j)
// of lane group g holds key 4g + j (j < 4) or 16 + 4g + j - 4 — and V^T is staged in LDS
// in that order.  Padded keys (>= S) get probability 0 and zero V rows; padded queries
// are computed and not stored.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 h16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) short_attention_mfma_kernel(const __hip_bfloat16 *__restrict__ qkv, int S, int H,
                                                                  float scale, __hip_bfloat16 *__restrict__ out) {
  constexpr int VT = 36;  // V^T row stride (keys): 72 B keeps 8-byte reads aligned
  __shared__ __attribute__((aligned(16))) __bf16 vt[kAttnDh * VT];
  const int lane = threadIdx.x;
  const int g = lane >> 4, c = lane & 15;
  const int h = blockIdx.x % H;
  const int64_t b = blockIdx.x / H;
  const int64_t tok = 3LL * H * kAttnDh;
  const __bf16 *base = reinterpret_cast<const __bf16 *>(qkv) + b * S * tok + (int64_t)h * kAttnDh;
  const __bf16 *kb = base + (int64_t)H * kAttnDh;
  const __bf16 *vb = base + 2LL * H * kAttnDh;
  // V rows as 16-byte vectors, all four loads of a lane in flight together, then transposed into LDS
  bf16x8_t vv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = lane + 64 * u, kk = t >> 3;
    vv[u] = kk < S ? *reinterpret_cast<const bf16x8_t *>(vb + kk * tok + 8 * (t & 7)) : bf16x8_t{};
  }
  bf16x8_t qf[2][2], kf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int r = 16 * t + c;
      const int d0 = 32 * st + 8 * g;
      qf[t][st] = r < S ? *reinterpret_cast<const bf16x8_t *>(base + r * tok + d0) : bf16x8_t{};
      kf[t][st] = r < S ? *reinterpret_cast<const bf16x8_t *>(kb + r * tok + d0) : bf16x8_t{};
    }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = lane + 64 * u, kk = t >> 3, d0 = 8 * (t & 7);
#pragma unroll
    for (int e = 0; e < 8; ++e) vt[(d0 + e) * VT + kk] = vv[u][e];
  }
  f32x4_t sc[2][2];  // [key tile][query tile]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][0], qf[it][0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][1], qf[it][1], a, 0, 0, 0);
      sc[kt][it] = a;
    }
  bf16x8_t pa[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float v[8];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kt = j >> 2, r = j & 3;
      const int kk = 16 * kt + 4 * g + r;
      v[j] = kk < S ? sc[kt][it][r] * scale : -INFINITY;
      m = fmaxf(m, v[j]);
    }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = v[j] == -INFINITY ? 0.f : __expf(v[j] - m);
      sum += v[j];
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.f / sum;
#pragma unroll
    for (int j = 0; j < 8; ++j) pa[it][j] = (__bf16)(v[j] * inv);
  }
  __syncthreads();  // V^T staged
#pragma unroll
  for (int dt = 0; dt < kAttnDh / 16; ++dt) {
    const int d = 16 * dt + c;
    bf16x8_t vf;
    const uint2 lo = *reinterpret_cast<const uint2 *>(&vt[d * VT + 4 * g]);
    const uint2 hi = *reinterpret_cast<const uint2 *>(&vt[d * VT + 16 + 4 * g]);
    const uint4 w = make_uint4(lo.x, lo.y, hi.x, hi.y);
    vf = *reinterpret_cast<const bf16x8_t *>(&w);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x4_t o = {0.f, 0.f, 0.f, 0.f};
      o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[it], vf, o, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * it + 4 * g + r;
        if (i < S) out[(b * S + i) * (int64_t)H * kAttnDh + (int64_t)h * kAttnDh + d] = __float2bfloat16(o[r]);
      }
    }
  }
}

// fp32-accurate twin of short_attention_mfma_kernel for the K10 path (fp32 query encode, S <= 32):
// every MFMA operand is split into f16 halves (v = hi + lo) and each product is lo.hi + hi.lo +
// hi.hi on v_mfma_f32_16x16x32_f16 (as K10, cm_gemm.hip): S^T = K Q^T from fp32 Q/K fragments
// split in registers, fp32 softmax on the accumulators, O = P V with P split in registers and
// V^T staged split in LDS in the permuted key order of the accumulator layout.  The context is
// written as K10 planes of o * a_scale (the O projection's operand) through an LDS image of the
// (S x 64) head slice: 16-byte slot stores.
// f16 range: a lo half below 2^-14 is subnormal, with an absolute precision of 2^-24 instead of
// 11 significant bits (a probability of 0.05 has a lo half of ~2e-5), and the unscaled split of
// Q, K, V and P measured 1.3e-4 context errors at S = 24 against 1e-5 for torch's fp32.  Every
// operand is therefore split after an exact power-of-two scale that puts the wave's largest |x|
// in [2^13, 2^14) -- Q, K and V by their per-(sequence, head) maxima, P (<= 1) by 2^14 -- so the
// split keeps 22 significant bits, and the scales are undone exactly on the fp32 accumulators.
__device__ inline float pow2_scale_for(float amax) {
  if (!(amax > 0.f)) return 1.f;
  int e;
  (void)frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1)
  return ldexpf(1.f, 14 - e);
}
__device__ inline float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ inline void load_frag8(const float *p, bool ok, float (&x)[8]) {
  float4 u = make_float4(0.f, 0.f, 0.f, 0.f), v = u;
  if (ok) {
    u = reinterpret_cast<const float4 *>(p)[0];
    v = reinterpret_cast<const float4 *>(p)[1];
  }
  x[0] = u.x, x[1] = u.y, x[2] = u.z, x[3] = u.w, x[4] = v.x, x[5] = v.y, x[6] = v.z, x[7] = v.w;
}
__device__ inline void split_frag8(const float (&x)[8], float s, h16x8_t &hi, h16x8_t &lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    _Float16 h, l;
    f16x3_split1(x[e] * s, h, l);
    hi[e] = h;
    lo[e] = l;
  }
}

__device__ inline f32x4_t mfma3(const h16x8_t &ah, const h16x8_t &al, const h16x8_t &bh, const h16x8_t &bl, f32x4_t c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
}

// key_mask (optional, B x S, nonzero = attend): padded keys leave the softmax (probability 0), as
// the XLM-R extended attention mask does; padded query rows are computed like any other row.
__global__ void __launch_bounds__(64) short_attention_f16x3_kernel(const float *__restrict__ qkv, int S, int H,
                                                                   float scale, float a_scale,
                                                                   const int32_t *__restrict__ key_mask,
                                                                   _Float16 *__restrict__ planes) {
  constexpr int VT = 40;  // V^T row stride (keys, halves): 80 B keeps the 8-byte reads aligned
  constexpr float kPScale = 16384.f;  // P in [0, 1] -> [0, 2^14]
  __shared__ __attribute__((aligned(16))) _Float16 vt[2][kAttnDh * VT];
  const int lane = threadIdx.x;
  const int g = lane >> 4, c = lane & 15;
  const int h = blockIdx.x % H;
  const int64_t b = blockIdx.x / H;
  const int64_t tok = 3LL * H * kAttnDh;
  const float *base = qkv + b * S * tok + (int64_t)h * kAttnDh;
  const float *kb = base + (int64_t)H * kAttnDh;
  const float *vb = base + 2LL * H * kAttnDh;
  // every load of the wave first: V (lane: key kk = t >> 4, dims 4 (t & 15) .. + 3), Q and K fragments
  float4 vv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int t = lane + 64 * u, kk = t >> 4, d0 = 4 * (t & 15);
    vv[u] = kk < S ? *reinterpret_cast<const float4 *>(vb + kk * tok + d0) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float qx[2][2][8], kx[2][2][8];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int r = 16 * t + c;
      const int d0 = 32 * st + 8 * g;
      load_frag8(base + r * tok + d0, r < S, qx[t][st]);
      load_frag8(kb + r * tok + d0, r < S, kx[t][st]);
    }
  // this lane's 8 keys (kk = 16 kt + 4 g + r): attended or not (the mask loads issued with the others,
  // not between the two MFMA stages)
  uint32_t kmask = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kk = 16 * (j >> 2) + 4 * g + (j & 3);
    if (kk < S && (!key_mask || key_mask[b * S + kk] != 0)) kmask |= 1u << j;
  }
  float mq = 0.f, mk = 0.f, mv = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mq = fmaxf(mq, fabsf(qx[t][st][e]));
        mk = fmaxf(mk, fabsf(kx[t][st][e]));
      }
#pragma unroll
  for (int u = 0; u < 8; ++u)
    mv = fmaxf(mv, fmaxf(fmaxf(fabsf(vv[u].x), fabsf(vv[u].y)), fmaxf(fabsf(vv[u].z), fabsf(vv[u].w))));
  const float sq = pow2_scale_for(wave_max(mq)), sk = pow2_scale_for(wave_max(mk)), sv = pow2_scale_for(wave_max(mv));
  // split V^T into LDS
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int t = lane + 64 * u, kk = t >> 4, d0 = 4 * (t & 15);
    const float x[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      _Float16 hh, ll;
      f16x3_split1(x[e] * sv, hh, ll);
      vt[0][(d0 + e) * VT + kk] = hh;
      vt[1][(d0 + e) * VT + kk] = ll;
    }
  }
  h16x8_t qh[2][2], ql[2][2], kh[2][2], kl[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      split_frag8(qx[t][st], sq, qh[t][st], ql[t][st]);
      split_frag8(kx[t][st], sk, kh[t][st], kl[t][st]);
    }
  f32x4_t sc[2][2];  // [key tile][query tile]: S^T (times sq sk)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
      a = mfma3(kh[kt][0], kl[kt][0], qh[it][0], ql[it][0], a);
      a = mfma3(kh[kt][1], kl[kt][1], qh[it][1], ql[it][1], a);
      sc[kt][it] = a;
    }
  const float lscale = scale / (sq * sk);  // exact: sq sk is a power of two
  h16x8_t ph[2], pl[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float v[8];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kt = j >> 2, r = j & 3;
      const int kk = 16 * kt + 4 * g + r;
      v[j] = ((kmask >> j) & 1u) ? sc[kt][it][r] * lscale : -INFINITY;
      (void)kk;
      m = fmaxf(m, v[j]);
    }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = v[j] == -INFINITY ? 0.f : __expf(v[j] - m);
      sum += v[j];
    }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.f / sum;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 hh, ll;
      f16x3_split1(v[j] * inv * kPScale, hh, ll);
      ph[it][j] = hh;
      pl[it][j] = ll;
    }
  }
  __syncthreads();  // V^T staged
  const float oscale = a_scale / (kPScale * sv);  // exact power-of-two ratio
  // O straight from the accumulators into the planes (no LDS transpose: the block's LDS is V^T alone,
  // twice the resident blocks per CU): lane (g, c) holds rows 16 it + 4 g + r of column d = 16 dt + c;
  // lanes c and c ^ 1 swap half their rows (DPP quad_perm 1,0,3,2) so each stores 4-byte column pairs
  // (c even: rows 0-1, c odd: rows 2-3 of its group) -- K10's planes epilogue
  const int kb32 = H * kAttnDh / 32;
  const bool odd = c & 1;
#pragma unroll
  for (int dt = 0; dt < kAttnDh / 16; ++dt) {
    const int d = 16 * dt + c;
    auto vfrag = [&](int pl2) __attribute__((always_inline)) {
      const uint2 lo4 = *reinterpret_cast<const uint2 *>(&vt[pl2][d * VT + 4 * g]);
      const uint2 hi4 = *reinterpret_cast<const uint2 *>(&vt[pl2][d * VT + 16 + 4 * g]);
      const uint4 w = make_uint4(lo4.x, lo4.y, hi4.x, hi4.y);
      return *reinterpret_cast<const h16x8_t *>(&w);
    };
    const h16x8_t vh = vfrag(0), vl = vfrag(1);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x4_t o = {0.f, 0.f, 0.f, 0.f};
      o = mfma3(ph[it], pl[it], vh, vl, o);
      uint32_t hh[4], ll[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        _Float16 a, b2;
        f16x3_split1(o[r] * oscale, a, b2);
        hh[r] = __builtin_bit_cast(uint16_t, a);
        ll[r] = __builtin_bit_cast(uint16_t, b2);
      }
      // even lane keeps rows 0-1 and sends 2-3; odd lane keeps 2-3 and sends 0-1
      const uint32_t sh = odd ? (hh[0] | hh[1] << 16) : (hh[2] | hh[3] << 16);
      const uint32_t sl = odd ? (ll[0] | ll[1] << 16) : (ll[2] | ll[3] << 16);
      const uint32_t rh = (uint32_t)__builtin_amdgcn_mov_dpp((int)sh, 0xB1, 0xF, 0xF, false);
      const uint32_t rl = (uint32_t)__builtin_amdgcn_mov_dpp((int)sl, 0xB1, 0xF, 0xF, false);
      const int r0 = odd ? 2 : 0;
      const int c0 = h * kAttnDh + (d & ~1);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = 16 * it + 4 * g + r0 + q;
        const uint32_t mine_h = hh[r0 + q], mine_l = ll[r0 + q];
        const uint32_t oth_h = (rh >> (16 * q)) & 0xffffu, oth_l = (rl >> (16 * q)) & 0xffffu;
        // column c0 (even) in the low half, c0 + 1 in the high half
        const uint32_t wh = odd ? (oth_h | mine_h << 16) : (mine_h | oth_h << 16);
        const uint32_t wl = odd ? (oth_l | mine_l << 16) : (mine_l | oth_l << 16);
        if (i < S) {
          const int64_t off = f16x3_plane_off(b * S + i, c0, kb32);
          *reinterpret_cast<uint32_t *>(planes + off) = wh;
          *reinterpret_cast<uint32_t *>(planes + off + 512) = wl;
        }
      }
    }
  }
}

// K9L: fp32-accurate attention for sequences of any length (passages: S up to 512, padded or not)
// on the K10 path, replacing torch SDPA + a split pass.  One workgroup of 4 waves per (sequence,
// head, block of 64 queries), 16 queries per wave; the keys stream through LDS in chunks of 64 with
// a flash-style online softmax (running max m and sum l per query, in fp32).  Per chunk the
// workgroup loads K and V once, splits them after exact power-of-two scales of the chunk's max|K| /
// max|V| (as K9s does per sequence: every lo half stays a normal f16) into MFMA fragment order in
// LDS: K as the A operand of S^T = K Q^T, V in the permuted key order that lets the S^T accumulator
// be the P operand of O = P V (short_attention_f16x3_kernel's trick).  Products are lo.hi + hi.lo +
// hi.hi on v_mfma_f32_16x16x32_f16 (K10's split precision); P = exp(s - m) <= 1 is split after a
// 2^14 scale; each chunk's P V lands in a fresh accumulator and joins the running output as
// o = o alpha + (P V) / (2^14 sv) in fp32.  The context is written as K10 planes of o * a_scale.
constexpr int kLaKeys = 64;  // keys per chunk

__global__ void __launch_bounds__(256) long_attention_f16x3_kernel(const float *__restrict__ qkv, int S, int H,
                                                                   float scale, float a_scale,
                                                                   const int32_t *__restrict__ key_mask,
                                                                   _Float16 *__restrict__ planes) {
  constexpr float kPScale = 16384.f;
  constexpr int OST = kAttnDh + 4;                      // output image row stride (floats)
  // [kt 4][st 2][hi/lo][lane 64][8 halves] K fragments, then [u 2][dt 4][hi/lo][lane][8] V fragments;
  // after the last chunk the same bytes hold the 4 waves' 16 x 64 fp32 output images
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * 16 * 512];
  __shared__ float red[2][4];
  __shared__ uint32_t kbits[2];
  _Float16 *kst = lds, *vst = lds + 16 * 512;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int nqb = (S + 63) >> 6;
  const int qb = (int)(blockIdx.x % nqb);
  const int h = (int)((blockIdx.x / nqb) % H);
  const int64_t b = blockIdx.x / ((int64_t)nqb * H);
  const int64_t tok = 3LL * H * kAttnDh;
  const float *base = qkv + b * S * tok + (int64_t)h * kAttnDh;
  const float *kbp = base + (int64_t)H * kAttnDh;
  const float *vbp = base + 2LL * H * kAttnDh;
  const int q0 = qb * 64 + wave * 16;
  // Q fragments (B operand): lane (g, c) = query q0 + c, dims 32 st + 8 g .. + 7
  float qx[2][8];
  float mq = 0.f;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    load_frag8(base + (int64_t)(q0 + c) * tok + 32 * st + 8 * g, q0 + c < S, qx[st]);
#pragma unroll
    for (int e = 0; e < 8; ++e) mq = fmaxf(mq, fabsf(qx[st][e]));
  }
  const float sq = pow2_scale_for(wave_max(mq));
  h16x8_t qh[2], ql[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) split_frag8(qx[st], sq, qh[st], ql[st]);

  float m_run = -INFINITY, l_run = 0.f;               // per query column c (same in every g)
  f32x4_t o_run[4];                                   // [dt]: O[query 4 g + r][dim 16 dt + c]
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o_run[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int vk = 4 * (tid >> 4), vd = 4 * (tid & 15);  // V staging: keys vk .. + 3, dims vd .. + 3

  for (int k0 = 0; k0 < S; k0 += kLaKeys) {
    // ---- the chunk's K (two fragment combos per thread) and V rows, their maxima, the key mask
    float kx[2][8];
    float mk = 0.f, mv = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cb = tid + 256 * i, cc = cb & 15, gg = (cb >> 4) & 3, st = (cb >> 6) & 1, kt = cb >> 7;
      const int key = k0 + 16 * kt + cc;
      load_frag8(kbp + (int64_t)key * tok + 32 * st + 8 * gg, key < S, kx[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) mk = fmaxf(mk, fabsf(kx[i][e]));
    }
    float4 vv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = k0 + vk + j;
      vv[j] = key < S ? *reinterpret_cast<const float4 *>(vbp + (int64_t)key * tok + vd) : make_float4(0.f, 0.f, 0.f, 0.f);
      mv = fmaxf(mv, fmaxf(fmaxf(fabsf(vv[j].x), fabsf(vv[j].y)), fmaxf(fabsf(vv[j].z), fabsf(vv[j].w))));
    }
    mk = wave_max(mk);
    mv = wave_max(mv);
    if (lane == 0) {
      red[0][wave] = mk;
      red[1][wave] = mv;
    }
    if (wave == 0) {
      const int key = k0 + lane;
      const bool ok = key < S && (!key_mask || key_mask[b * S + key] != 0);
      const uint64_t bits = __ballot(ok);
      if (lane == 0) {
        kbits[0] = (uint32_t)bits;
        kbits[1] = (uint32_t)(bits >> 32);
      }
    }
    __syncthreads();                                  // maxima + mask published; previous chunk's reads done
    const float sk = pow2_scale_for(fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3])));
    const float sv = pow2_scale_for(fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3])));
    // the mask is read before the staging barrier: wave 0 rewrites it for the next chunk as soon as
    // every wave has passed that barrier
    const uint64_t kb = (uint64_t)kbits[0] | ((uint64_t)kbits[1] << 32);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int cb = tid + 256 * i, cc = cb & 15, gg = (cb >> 4) & 3, st = (cb >> 6) & 1, kt = cb >> 7;
      h16x8_t hh, ll;
      split_frag8(kx[i], sk, hh, ll);
      const int o = ((kt * 2 + st) * 2) * 512 + (gg * 16 + cc) * 8;
      *reinterpret_cast<h16x8_t *>(kst + o) = hh;
      *reinterpret_cast<h16x8_t *>(kst + o + 512) = ll;
    }
    {
      // V fragment (u, dt): lane (g', c') holds keys pi(8 g' + e) of 32-key step u, dim 16 dt + c';
      // pi(8 g' + e) = 4 g' + e (e < 4), 16 + 4 g' + e - 4 (e >= 4): this thread's 4 keys are 4
      // consecutive e of one lane per dim
      const int kk = vk & 31, u = vk >> 5, gv = (kk & 15) >> 2, e0 = (kk >> 4) << 2, dt = vd >> 4;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const float x4[4] = {(&vv[0].x)[e4], (&vv[1].x)[e4], (&vv[2].x)[e4], (&vv[3].x)[e4]};
        _Float16 hh[4], ll[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) f16x3_split1(x4[j] * sv, hh[j], ll[j]);
        const int o = ((u * 4 + dt) * 2) * 512 + (gv * 16 + (vd & 15) + e4) * 8 + e0;
        *reinterpret_cast<uint2 *>(vst + o) = *reinterpret_cast<const uint2 *>(hh);
        *reinterpret_cast<uint2 *>(vst + o + 512) = *reinterpret_cast<const uint2 *>(ll);
      }
    }
    __syncthreads();                                  // fragments staged
    // ---- S^T = K Q^T: sc[kt] lane (g, c) = keys 16 kt + 4 g + r, query c
    f32x4_t sc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const h16x8_t kh = *reinterpret_cast<const h16x8_t *>(kst + ((kt * 2 + st) * 2) * 512 + lane * 8);
        const h16x8_t kl = *reinterpret_cast<const h16x8_t *>(kst + ((kt * 2 + st) * 2 + 1) * 512 + lane * 8);
        a = mfma3(kh, kl, qh[st], ql[st], a);
      }
      sc[kt] = a;
    }
    const float lscale = scale / (sq * sk);           // exact power-of-two ratio times scale
    float mloc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = 16 * kt + 4 * g + r;
        const float v = ((kb >> j) & 1ull) ? sc[kt][r] * lscale : -INFINITY;
        sc[kt][r] = v;
        mloc = fmaxf(mloc, v);
      }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = m_new == -INFINITY ? 0.f : __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sc[kt][r];
        const float p = v == -INFINITY ? 0.f : __expf(v - m_new);
        sc[kt][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16);
    psum += __shfl_xor(psum, 32);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    // P fragments of the two 32-key steps (A operand: row = query c, k-slot e = key pi(8 g + e))
    h16x8_t ph[2], pl[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hh, ll;
        f16x3_split1(sc[2 * u + (e >> 2)][e & 3] * kPScale, hh, ll);
        ph[u][e] = hh;
        pl[u][e] = ll;
      }
    float ar[4];                                      // alpha of query 4 g + r (held by lane c = 4 g + r)
#pragma unroll
    for (int r = 0; r < 4; ++r) ar[r] = __shfl(alpha, 4 * g + r);
    const float inv_pv = 1.f / (kPScale * sv);        // exact power of two
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4_t oc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const h16x8_t vh = *reinterpret_cast<const h16x8_t *>(vst + ((u * 4 + dt) * 2) * 512 + lane * 8);
        const h16x8_t vl = *reinterpret_cast<const h16x8_t *>(vst + ((u * 4 + dt) * 2 + 1) * 512 + lane * 8);
        oc = mfma3(ph[u], pl[u], vh, vl, oc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) o_run[dt][r] = o_run[dt][r] * ar[r] + oc[r] * inv_pv;
    }
  }
  __syncthreads();                                    // every wave's last fragment reads are done
  // ---- O / l * a_scale -> this wave's 16 x 64 image -> K10 planes (16-byte slots)
  float *oimg = reinterpret_cast<float *>(lds) + wave * 16 * OST;
  float lr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) lr[r] = __shfl(l_run, 4 * g + r);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      oimg[(4 * g + r) * OST + 16 * dt + c] = lr[r] > 0.f ? o_run[dt][r] / lr[r] * a_scale : 0.f;
  __syncthreads();
  const int kb32 = H * kAttnDh / 32;
#pragma unroll
  for (int u2 = 0; u2 < 2; ++u2) {
    const int t = lane + 64 * u2, i = t >> 3, s8 = t & 7;
    if (q0 + i < S) {
      h16x8_t hh, ll;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 a, b2;
        f16x3_split1(oimg[i * OST + 8 * s8 + e], a, b2);
        hh[e] = a;
        ll[e] = b2;
      }
      const int64_t off = f16x3_plane_off(b * S + q0 + i, h * kAttnDh + 8 * s8, kb32);
      *reinterpret_cast<h16x8_t *>(planes + off) = hh;
      *reinterpret_cast<h16x8_t *>(planes + off + 512) = ll;
    }
  }
}

// K9P: K9L's math on operands that are already split.  The QKV projection writes its output as
// planes (cm_linear_f16x3 with CM_EPI_PLANES_QKV, one exact power-of-two scale s for Q, K and V from
// the host's rigorous bound): Q and K in the standard layout, V transposed in 32-key units whose
// lane slots are already in the permuted key order of the P V operand (k10_epilogue).  So every
// fragment of the attention is a 1 KiB block of HBM: no fp32 loads, no maxima, no split work.  One
// workgroup of K9P_WAVES = 8 waves (16 queries each) per (sequence, head, 128-query block), two per
// CU, the query blocks of a (sequence, head) on one XCD (its keys and values come from that L2 for
// the second); the 64-key chunks stream through a two-slot LDS ring by LDS-DMA (32 one-KiB pieces
// per chunk, the next chunk in flight while this one is consumed, one barrier per chunk).  Per chunk
// and wave: K9L's 48 MFMAs, the online softmax in the log2 domain; the context is written as planes
// of o * a_scale with K10's DPP pair stores.  S % 64 == 0.  Ingest shape: 247 us per layer (K9L 496;
// 16 waves per workgroup: 281), profiles/r05_k9p_ab.txt.
constexpr int kApSlot = 32 * 1024;  // one chunk: K 16 KiB + V 16 KiB
#ifndef K9P_WAVES
#define K9P_WAVES 8                 // waves (16 queries each) per workgroup: 8 or 16 (A/B)
#endif

template <bool MASKED>
__global__ void __launch_bounds__(1024) planes_attention_kernel(const _Float16 *__restrict__ qkv, int nseq, int S, int H,
                                                                float scale, float s_qkv, float a_scale,
                                                                const int32_t *__restrict__ key_mask,
                                                                _Float16 *__restrict__ planes) {
  constexpr float kPScale = 16384.f;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * kApSlot];
  __shared__ uint64_t kmask[8];                        // per 64-key chunk (S <= 512)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = blockDim.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  // XCD-aware order: the nqb query blocks of one (sequence, head) are blockIdx w, w + 8, ... (one XCD
  // under round-robin dispatch, so the keys and values DMA'd by the first stay in that XCD's L2 for
  // the others); the grid is padded to whole groups of 8 (sequence, head) pairs
  const int nqb = (S + 16 * nw - 1) / (16 * nw);
  const int64_t grp = blockIdx.x / (8 * nqb);
  const int qb = (int)((blockIdx.x >> 3) % nqb);
  const int64_t pair = grp * 8 + (blockIdx.x & 7);
  if (pair >= (int64_t)nseq * H) return;          // padding: the whole workgroup, before any barrier
  const int h = (int)(pair % H);
  const int64_t b = pair / H;
  const int D = H * kAttnDh, kb3 = 3 * D / 32, kbd = D / 32;   // split blocks per row block: qkv, context
  const int nch = S / 64;
  const int q0 = qb * 16 * nw + wave * 16;
  const bool qok = q0 < S;                             // wave-uniform: a partial last block's spare waves
  const unsigned char *src = reinterpret_cast<const unsigned char *>(qkv);

  // key mask bits of every chunk (all keys attend without a mask)
  if constexpr (MASKED)
    for (int ch = wave; ch < nch; ch += nw) {
      const uint64_t bits = __ballot(key_mask[b * S + 64 * ch + lane] != 0);
      if (lane == 0) kmask[ch] = bits;
    }
  // Q fragments (B operand of S^T = K Q^T): lane (g, c) = query q0 + c, dims 32 st + 8 g .. + 7
  h16x8_t qh[2], ql[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    if (qok) {
      const int64_t o = ((((b * S + q0) >> 4) * kb3 + 2 * h + st) * 128 + lane) * 8;
      qh[st] = *reinterpret_cast<const h16x8_t *>(qkv + o);
      ql[st] = *reinterpret_cast<const h16x8_t *>(qkv + o + 512);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) qh[st][e] = ql[st][e] = (_Float16)0.f;
    }
  }
  // chunk ch's 32 DMA pieces: p < 16 K block (kt = p / 4, st, plane), else V^T block (u, dt, plane).
  // Piece p of chunk ch sits at (first key row / 16) x kb3 split blocks + a per-piece offset (the V^T
  // 32-row units: 2 u_g = krow / 16 since krow is a multiple of 64); this wave's pieces p = wave +
  // i nw and their offsets are fixed for the kernel
  int64_t poff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = wave + i * nw;
    int64_t blk = 0;
    if (p < 16) {
      const int kt = p >> 2, st = (p >> 1) & 1;
      blk = (int64_t)kt * kb3 + kbd + 2 * h + st;
    } else if (p < 32) {
      const int u = (p - 16) >> 3, dt = ((p - 16) >> 1) & 3;
      const int dblk = 4 * h + dt;                       // 16-dim block of V
      blk = (int64_t)(2 * u + dblk / kbd) * kb3 + 2 * kbd + dblk % kbd;
    }
    poff[i] = blk * 2048 + (p & 1) * 1024 + lane * 16;
  }
  const unsigned char *seq_src = src + ((b * S) >> 4) * kb3 * 2048;
  auto issue = [&](int ch) __attribute__((always_inline)) {
    unsigned char *slot = lds + (ch & 1) * kApSlot;
    const unsigned char *cs = seq_src + (int64_t)(4 * ch) * kb3 * 2048;   // 64 keys = 4 row blocks
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = wave + i * nw;
      if (p >= 32) break;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(cs + poff[i]),
                                       (__attribute__((address_space(3))) void *)(slot + p * 1024), 16, 0, 0);
    }
  };
  issue(0);

  // softmax in the base-2 domain: p = 2^(s lscale2 - m) with lscale2 = scale log2(e) / s_qkv^2 (one
  // fma + v_exp per score); masked scores are -inf (2^-inf = 0), and m_safe keeps a chunk whose keys
  // are all masked so far from producing -inf - -inf
  const float lscale2 = scale / (s_qkv * s_qkv) * 1.4426950408889634f;
  const float inv_pv = 1.f / (kPScale * s_qkv);
  float m_run = -INFINITY, l_run = 0.f;               // per query column c (same in every g), log2 domain
  f32x4_t o_run[4];                                   // [dt]: O[query 4 g + r][dim 16 dt + c]
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o_run[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < nch; ++ch) {
    // this wave's pieces of chunk ch landed; the barrier publishes everyone's (and the mask) and
    // retires every read of the other slot, which the next chunk's pieces then overwrite
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ch + 1 < nch) issue(ch + 1);
    const _Float16 *kst = reinterpret_cast<const _Float16 *>(lds + (ch & 1) * kApSlot);
    const _Float16 *vst = kst + 16 * 512;
    f32x4_t sc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const h16x8_t kh = *reinterpret_cast<const h16x8_t *>(kst + ((kt * 2 + st) * 2) * 512 + lane * 8);
        const h16x8_t kl = *reinterpret_cast<const h16x8_t *>(kst + ((kt * 2 + st) * 2 + 1) * 512 + lane * 8);
        a = mfma3(kh, kl, qh[st], ql[st], a);
      }
      sc[kt] = a;
    }
    if constexpr (MASKED) {                           // keys 16 kt + 4 g + r of the chunk
      const uint64_t kb = kmask[ch];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const uint32_t nib = (uint32_t)(kb >> (16 * kt + 4 * g));
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!((nib >> r) & 1u)) sc[kt][r] = -INFINITY;
      }
    }
    float mloc = fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3]));
#pragma unroll
    for (int kt = 1; kt < 4; ++kt) mloc = fmaxf(mloc, fmaxf(fmaxf(sc[kt][0], sc[kt][1]), fmaxf(sc[kt][2], sc[kt][3])));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
    const float m_new = fmaxf(m_run, mloc * lscale2);
    const float m_safe = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_safe);
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sc[kt][r], lscale2, -m_safe));
        sc[kt][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16);
    psum += __shfl_xor(psum, 32);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    h16x8_t ph[2], pl[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 hh, ll;
        f16x3_split1(sc[2 * u + (e >> 2)][e & 3] * kPScale, hh, ll);
        ph[u][e] = hh;
        pl[u][e] = ll;
      }
    float ar[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ar[r] = __shfl(alpha, 4 * g + r);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f32x4_t oc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const h16x8_t vh = *reinterpret_cast<const h16x8_t *>(vst + ((u * 4 + dt) * 2) * 512 + lane * 8);
        const h16x8_t vl = *reinterpret_cast<const h16x8_t *>(vst + ((u * 4 + dt) * 2 + 1) * 512 + lane * 8);
        oc = mfma3(ph[u], pl[u], vh, vl, oc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) o_run[dt][r] = fmaf(o_run[dt][r], ar[r], oc[r] * inv_pv);
    }
  }
  if (!qok) return;                                   // no barrier follows
  // ---- O / l * a_scale -> context planes: lanes c, c ^ 1 swap halves so each stores 4-byte
  //      column pairs (k10_epilogue's planes store)
  float lr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) lr[r] = __shfl(l_run, 4 * g + r);
  const bool odd = c & 1;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    uint32_t hh[4], ll[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      _Float16 a, b2;
      f16x3_split1(lr[r] > 0.f ? o_run[dt][r] / lr[r] * a_scale : 0.f, a, b2);
      hh[r] = __builtin_bit_cast(uint16_t, a);
      ll[r] = __builtin_bit_cast(uint16_t, b2);
    }
    const uint32_t sh = odd ? (hh[0] | hh[1] << 16) : (hh[2] | hh[3] << 16);
    const uint32_t sl = odd ? (ll[0] | ll[1] << 16) : (ll[2] | ll[3] << 16);
    const uint32_t rh = (uint32_t)__builtin_amdgcn_mov_dpp((int)sh, 0xB1, 0xF, 0xF, false);
    const uint32_t rl = (uint32_t)__builtin_amdgcn_mov_dpp((int)sl, 0xB1, 0xF, 0xF, false);
    const int r0 = odd ? 2 : 0;
    const int c0 = h * kAttnDh + 16 * dt + (c & ~1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t mine_h = hh[r0 + q], mine_l = ll[r0 + q];
      const uint32_t oth_h = (rh >> (16 * q)) & 0xffffu, oth_l = (rl >> (16 * q)) & 0xffffu;
      const uint32_t wh = odd ? (oth_h | mine_h << 16) : (mine_h | oth_h << 16);
      const uint32_t wl = odd ? (oth_l | mine_l << 16) : (mine_l | oth_l << 16);
      const int64_t off = f16x3_plane_off(b * S + q0 + 4 * g + r0 + q, c0, kbd);
      *reinterpret_cast<uint32_t *>(planes + off) = wh;
      *reinterpret_cast<uint32_t *>(planes + off + 512) = wl;
    }
  }
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

extern "C" int cm_short_attention(const void *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim, float scale,
                                  int32_t dtype, void *out_dev, void *stream) {
  if (B <= 0) return CM_OK;
  if (!qkv_dev || !out_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (head_dim != kAttnDh) CM_FAIL(CM_EINVAL, "head_dim must be 64");
  if (S <= 0 || S > kAttnMaxS || H <= 0) CM_FAIL(CM_EINVAL, "need 0 < S <= 64 and H > 0");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((int64_t)B * H)), block(64);
  switch (dtype) {
    case CM_DTYPE_F32:
      hipLaunchKernelGGL(short_attention_kernel<float>, grid, block, 0, st, (const float *)qkv_dev, S, H, scale,
                         (float *)out_dev);
      break;
    case CM_DTYPE_BF16:
      if (S <= 32)
        hipLaunchKernelGGL(short_attention_mfma_kernel, grid, block, 0, st, (const __hip_bfloat16 *)qkv_dev, S, H,
                           scale, (__hip_bfloat16 *)out_dev);
      else
        hipLaunchKernelGGL(short_attention_kernel<__hip_bfloat16>, grid, block, 0, st, (const __hip_bfloat16 *)qkv_dev,
                           S, H, scale, (__hip_bfloat16 *)out_dev);
      break;
    default: CM_FAIL(CM_EINVAL, "dtype must be f32/bf16");
  }
  CM_HIP(hipGetLastError());
  return CM_OK;
}

extern "C" int cm_add_layernorm_split(const float *x_dev, const float *r_dev, int64_t r_rows, const float *gamma_dev,
                                      const float *beta_dev, int64_t rows, int32_t D, float eps, float *out_dev,
                                      float a_scale, void *planes_dev, void *stream) {
  if (rows <= 0) return CM_OK;
  if (!x_dev || !gamma_dev || !beta_dev || !out_dev || !planes_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (D <= 0 || D % 32 != 0 || D > 4 * 64 * kLnMaxPer) CM_FAIL(CM_EINVAL, "D must be a multiple of 32, <= 2048");
  if (r_dev && r_rows <= 0) CM_FAIL(CM_EINVAL, "r_rows must be > 0 with a residual");
  hipStream_t st = (hipStream_t)stream;
  _Float16 *ph = (_Float16 *)planes_dev;
  switch ((int)ceil_div(D / 4, 64)) {
    case 1: return launch_add_ln_split<1>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, a_scale, ph, st);
    case 2: return launch_add_ln_split<2>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, a_scale, ph, st);
    case 3: return launch_add_ln_split<3>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, a_scale, ph, st);
    case 4: return launch_add_ln_split<4>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, a_scale, ph, st);
    default: return launch_add_ln_split<8>(x_dev, r_dev, r_rows, gamma_dev, beta_dev, rows, D, eps, out_dev, a_scale, ph, st);
  }
}

extern "C" int cm_short_attention_split_masked(const float *qkv_dev, int32_t B, int32_t S, int32_t H,
                                               int32_t head_dim, float scale, float a_scale,
                                               const int32_t *key_mask_dev, void *planes_dev, void *stream) {
  if (B <= 0) return CM_OK;
  if (!qkv_dev || !planes_dev || !key_mask_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (head_dim != kAttnDh) CM_FAIL(CM_EINVAL, "head_dim must be 64");
  if (S <= 0 || S > 32 || H <= 0) CM_FAIL(CM_EUNSUPPORTED, "masked attention: need 0 < S <= 32 and H > 0");
  hipLaunchKernelGGL(short_attention_f16x3_kernel, dim3((unsigned)((int64_t)B * H)), dim3(64), 0, (hipStream_t)stream,
                     qkv_dev, S, H, scale, a_scale, key_mask_dev, (_Float16 *)planes_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

extern "C" int cm_short_attention_split(const float *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim,
                                        float scale, float a_scale, void *planes_dev, void *stream) {
  if (B <= 0) return CM_OK;
  if (!qkv_dev || !planes_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (head_dim != kAttnDh) CM_FAIL(CM_EINVAL, "head_dim must be 64");
  if (S <= 0 || S > kAttnMaxS || H <= 0) CM_FAIL(CM_EINVAL, "need 0 < S <= 64 and H > 0");
  if (S <= 32)   // matrix cores, split precision
    hipLaunchKernelGGL(short_attention_f16x3_kernel, dim3((unsigned)((int64_t)B * H)), dim3(64), 0,
                       (hipStream_t)stream, qkv_dev, S, H, scale, a_scale, (const int32_t *)nullptr,
                       (_Float16 *)planes_dev);
  else
    hipLaunchKernelGGL((short_attention_kernel<float, true>), dim3((unsigned)((int64_t)B * H)), dim3(64), 0,
                       (hipStream_t)stream, qkv_dev, S, H, scale, nullptr, a_scale, (_Float16 *)planes_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

extern "C" int cm_planes_attention(const void *qkv_planes, int32_t B, int32_t S, int32_t H, int32_t head_dim,
                                   float scale, float s_qkv, float a_scale, const int32_t *key_mask_dev,
                                   void *planes_dev, void *stream) {
  if (B <= 0) return CM_OK;
  if (!qkv_planes || !planes_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (head_dim != kAttnDh) CM_FAIL(CM_EINVAL, "head_dim must be 64");
  if (S <= 0 || S % 64 || S > 512 || H <= 0) CM_FAIL(CM_EINVAL, "need S % 64 == 0, 0 < S <= 512 and H > 0");
  if (!(s_qkv > 0.f) || !(a_scale > 0.f)) CM_FAIL(CM_EINVAL, "scales must be > 0");
  if (((uintptr_t)qkv_planes & 15) || ((uintptr_t)planes_dev & 15)) CM_FAIL(CM_EINVAL, "planes must be 16-byte aligned");
  // 8 waves (128 queries) per workgroup: two resident per CU (LDS 2 x 64 KiB, 4 waves per SIMD), so one
  // workgroup's first DMA and epilogue overlap the other's chunks (247 vs 281 us per layer at 16 waves)
  const int nw = std::min(K9P_WAVES, S / 16);
  const int64_t blocks = ceil_div((int64_t)B * H, 8) * 8 * ((S + 16 * nw - 1) / (16 * nw));
  if (blocks > INT32_MAX) CM_FAIL(CM_EINVAL, "too many (sequence, head, query block) workgroups");
  if (key_mask_dev)
    hipLaunchKernelGGL(planes_attention_kernel<true>, dim3((unsigned)blocks), dim3(64 * nw), 0,
                       (hipStream_t)stream, (const _Float16 *)qkv_planes, B, S, H, scale, s_qkv, a_scale, key_mask_dev, (_Float16 *)planes_dev);
  else
    hipLaunchKernelGGL(planes_attention_kernel<false>, dim3((unsigned)blocks), dim3(64 * nw), 0,
                       (hipStream_t)stream, (const _Float16 *)qkv_planes, B, S, H, scale, s_qkv, a_scale, key_mask_dev, (_Float16 *)planes_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}

extern "C" int cm_long_attention_split(const float *qkv_dev, int32_t B, int32_t S, int32_t H, int32_t head_dim,
                                       float scale, float a_scale, const int32_t *key_mask_dev, void *planes_dev,
                                       void *stream) {
  if (B <= 0) return CM_OK;
  if (!qkv_dev || !planes_dev) CM_FAIL(CM_EINVAL, "NULL argument");
  if (head_dim != kAttnDh) CM_FAIL(CM_EINVAL, "head_dim must be 64");
  if (S <= 0 || S > 4096 || H <= 0) CM_FAIL(CM_EINVAL, "need 0 < S <= 4096 and H > 0");
  const int64_t blocks = (int64_t)B * H * ((S + 63) / 64);
  if (blocks > INT32_MAX) CM_FAIL(CM_EINVAL, "too many (sequence, head, query block) workgroups");
  hipLaunchKernelGGL(long_attention_f16x3_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, qkv_dev,
                     S, H, scale, a_scale, key_mask_dev, (_Float16 *)planes_dev);
  CM_HIP(hipGetLastError());
  return CM_OK;
}
