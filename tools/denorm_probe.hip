// Does v_mfma_f32_16x16x32_f16 keep subnormal f16 inputs?  A = one subnormal (or normal) value in
// every lane's first element, B = 1.0 in the first element: k = 0, 8, 16, 24 pair up, D = 4 a
//   hipcc --offload-arch=gfx950 -O2 tools/denorm_probe.hip -o tools/denorm_probe && ./tools/denorm_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k(float a, float *out) {
  h8 A = {}, B = {};
  A[0] = (_Float16)a;
  B[0] = (_Float16)1.0f;
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, c, 0, 0, 0);
  // VALU reference: the same f16 value widened
  if (threadIdx.x == 0) {
    out[0] = c[0];
    out[1] = (float)A[0];
    out[2] = (float)((_Float16)a * (_Float16)1.0f);
  }
}

int main() {
  float *d;
  (void)hipMalloc(&d, 16);
  const float vals[] = {1e-3f, 6.2e-5f, 6.0e-5f, 3.0e-5f, 1e-6f, 2.0e-7f, 6.0e-8f};
  for (float v : vals) {
    k<<<1, 64>>>(v, d);
    float h[3];
    (void)hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
    printf("a=%.3e  f16(a)=%.6e  mfma=%.6e  valu=%.6e  %s\n", v, h[1], h[0], h[2],
           h[0] == 4.0f * h[1] ? "kept (4 products)" : "CHANGED");
  }
  return 0;
}
