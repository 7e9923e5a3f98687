// Operand lane map of v_mfma_i32_16x16x64_i8 on gfx950, checked with exact integer data and an
// asymmetric B (cdna_hip_programming.md: "check the map with exact integer data").  Two candidate
// maps for lane l (i = l & 15, g = l >> 4), byte j = 0..15 of its 16-byte fragment:
//   H1: A[row i][k = 16 g + j],                B[k = 16 g + j][col i]
//   H2: A[row i][k = 8 g + j (j < 8), 32 + 8 g + j - 8 (j >= 8)], B likewise
// For each map, A and B fragments are packed from known matrices; the MFMA result is compared with
// the host product (C/D map: col = l & 15, row = 4 (l >> 4) + r, dtype-independent on gfx950).
// Measured: BOTH maps reproduce the product exactly -- a k permutation applied to A and B alike
// leaves the dot product unchanged, so K1q's correctness needs only that rows and queries are
// packed with the same map (they are: q8_plane_off / q8_query_off share q8_ge).
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_probe.hip -o tools/mfma_i8_probe && ./tools/mfma_i8_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void mfma_i8(const int8_t *A, const int8_t *B, int *D) {  // A, B: 64 lanes x 16 bytes, D: 64 x 4
  const int l = threadIdx.x;
  const i32x4 a = *reinterpret_cast<const i32x4 *>(A + 16 * l);
  const i32x4 b = *reinterpret_cast<const i32x4 *>(B + 16 * l);
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[4 * l + r] = c[r];
}

static int kmap(int h, int g, int j) { return h == 1 ? 16 * g + j : (j < 8 ? 8 * g + j : 32 + 8 * g + j - 8); }

int main() {
  int8_t Am[16][64], Bm[64][16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 64; ++k) Am[i][k] = (int8_t)(((i * 7 + k * 3) % 23) - 11);
  for (int k = 0; k < 64; ++k)
    for (int c = 0; c < 16; ++c) Bm[k][c] = (int8_t)(((k * 5 + c * 11 + k * c) % 19) - 9);
  int ref[16][16];
  for (int i = 0; i < 16; ++i)
    for (int c = 0; c < 16; ++c) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += Am[i][k] * Bm[k][c];
      ref[i][c] = s;
    }
  int8_t *dA, *dB;
  int *dD;
  (void)hipMalloc(&dA, 1024);
  (void)hipMalloc(&dB, 1024);
  (void)hipMalloc(&dD, 64 * 4 * 4);
  for (int h = 1; h <= 2; ++h) {
    int8_t hA[1024], hB[1024];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 16; ++j) {
        const int i = l & 15, g = l >> 4, k = kmap(h, g, j);
        hA[16 * l + j] = Am[i][k];
        hB[16 * l + j] = Bm[k][i];
      }
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_i8, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    int hD[256];
    const hipError_t e = hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) bad += hD[4 * l + r] != ref[4 * (l >> 4) + r][l & 15];
    printf("map H%d: %s, %d of 256 outputs differ\n", h, e == hipSuccess ? "ran" : hipGetErrorString(e), bad);
  }
  return 0;
}
