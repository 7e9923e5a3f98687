// Microbenchmark: cycles per 32-MFMA "chunk" (v_mfma_f32_16x16x32_f16, 16 accumulators, the K1c
// register tile) for one wave per SIMD, with optional per-chunk extras that K1c's chunk carries:
//   MODE bit 0: 16 AGPR->VGPR operand copies per chunk (the compiler's query-fragment staging)
//   MODE bit 1: 8 ds_read_b128 of the next chunk's fragments + lgkmcnt wait
//   MODE bit 2: one s_barrier per chunk (4 waves per workgroup)
//   MODE bit 3: an epilogue every 12 chunks (max-reduce of the 16 accumulators, ballot, zeroing)
// hipcc --offload-arch=gfx950 -O3 -o tools/mfma_micro tools/mfma_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256, 1) micro(const f16x8 *__restrict__ q, float *__restrict__ out, int chunks,
                                                long long *cycles) {
  __shared__ f16x8 lds[8 * 64 * 2];
  const int lane = threadIdx.x & 63;
  f16x8 qa[12][4][2];  // resident "query" fragments
#pragma unroll
  for (int c = 0; c < 12; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) qa[c][t][s] = q[((c * 4 + t) * 2 + s) * 64 + lane];
  f16x8 xf[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      xf[r][s] = q[(r * 2 + s) * 64 + lane + 3000];
      lds[(r * 2 + s) * 64 + lane] = xf[r][s];
    }
  __syncthreads();
  f32x4 acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float best = 0.f;
  const long long t0 = clock64();
  for (int it = 0; it < chunks / 12; ++it) {
#pragma unroll
    for (int c = 0; c < 12; ++c) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[r][0], qa[(MODE & 1) ? c : 0][t][0], acc[r][t], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xf[r][1], qa[(MODE & 1) ? c : 0][t][1], acc[r][t], 0, 0, 0);
      }
      if (MODE & 2) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int s = 0; s < 2; ++s) xf[r][s] = lds[(r * 2 + s) * 64 + ((lane + c + it) & 63)];
      }
      if (MODE & 4) __builtin_amdgcn_s_barrier();
    }
    if (MODE & 8) {
      float m = -1e30f;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) m = fmaxf(m, acc[r][t][i]);
      if (__ballot(m > 1e30f)) best += 1.f;
      best += m;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const long long t1 = clock64();
  float s = best;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < 4; ++t) s += acc[r][t][0] + acc[r][t][1] + acc[r][t][2] + acc[r][t][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const f16x8 *q, float *out, long long *cyc, int chunks, int blocks) {
  hipLaunchKernelGGL(micro<MODE>, dim3(blocks), dim3(256), 0, 0, q, out, chunks, cyc);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(micro<MODE>, dim3(blocks), dim3(256), 0, 0, q, out, chunks, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  long long h[1];
  hipMemcpy(h, cyc, sizeof(long long), hipMemcpyDeviceToHost);
  const double mfmas = 32.0 * chunks;
  printf("mode=%2d  chunks=%d  clock64 cycles/chunk=%.1f  wall ms=%.3f  -> %.1f ns/chunk, %.1f TFLOP/s (%d WGs)\n",
         MODE, chunks, (double)h[0] / chunks, ms, ms * 1e6 / chunks, mfmas * 16384.0 * 4 * blocks / (ms * 1e-3) / 1e12,
         blocks);
}

int main() {
  const int chunks = 12 * 2000, blocks = 256;
  f16x8 *q;
  float *out;
  long long *cyc;
  hipMalloc(&q, 8192 * sizeof(f16x8));
  hipMemset(q, 0, 8192 * sizeof(f16x8));
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipMalloc(&cyc, blocks * sizeof(long long));
  run<0>(q, out, cyc, chunks, blocks);
  run<1>(q, out, cyc, chunks, blocks);
  run<2>(q, out, cyc, chunks, blocks);
  run<4>(q, out, cyc, chunks, blocks);
  run<8>(q, out, cyc, chunks, blocks);
  run<3>(q, out, cyc, chunks, blocks);
  run<7>(q, out, cyc, chunks, blocks);
  run<15>(q, out, cyc, chunks, blocks);
  return 0;
}
