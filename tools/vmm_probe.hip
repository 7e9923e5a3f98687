// VMM behaviour probe (GPU box): reserve a range, map chunks one after another, set access per
// chunk or over the whole mapped prefix, touch every byte from a kernel.
//   hipcc --offload-arch=gfx950 -O2 tools/vmm_probe.hip -o tools/vmm_probe && ./tools/vmm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define P(x)                                                                   \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    printf("%-60s -> %s\n", #x, e_ == hipSuccess ? "ok" : hipGetErrorString(e_)); \
  } while (0)

__global__ void fill(unsigned *p, size_t n, unsigned v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v + (unsigned)i;
}

int main() {
  int vmm = 0;
  P(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
  printf("vmm supported: %d\n", vmm);
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  P(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
  P(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity min %zu rec %zu\n", gmin, grec);
  const size_t g = grec ? grec : (2u << 20);
  void *base = nullptr;
  const size_t R = 512ull << 30;
  P(hipMemAddressReserve(&base, R, g, nullptr, 0));
  printf("base %p\n", base);
  hipMemAccessDesc a{};
  a.location = prop.location;
  a.flags = hipMemAccessFlagsProtReadWrite;
  std::vector<size_t> sizes = {g, 3 * g, 16 * g};
  size_t off = 0;
  int mode = 0;
  for (size_t sz : sizes) {
    hipMemGenericAllocationHandle_t h{};
    P(hipMemCreate(&h, sz, &prop, 0));
    P(hipMemMap((char *)base + off, sz, 0, h, 0));
    hipError_t e = hipMemSetAccess((char *)base + off, sz, &a, 1);
    printf("setaccess chunk [%zu, +%zu): %s\n", off, sz, e == hipSuccess ? "ok" : hipGetErrorString(e));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      e = hipMemSetAccess(base, off + sz, &a, 1);
      printf("setaccess whole [0, %zu): %s\n", off + sz, e == hipSuccess ? "ok" : hipGetErrorString(e));
      mode = 1;
    }
    off += sz;
    fill<<<256, 256>>>((unsigned *)base, off / 4, 7u);
    P(hipGetLastError());
    P(hipDeviceSynchronize());
    std::vector<unsigned> hb(off / 4);
    P(hipMemcpy(hb.data(), base, off, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < hb.size(); ++i) bad += hb[i] != 7u + (unsigned)i;
    printf("mapped %zu bytes, bad words %zu (mode %d)\n", off, bad, mode);
  }
  // big chunk: 8 GiB
  {
    const size_t sz = 8ull << 30;
    hipMemGenericAllocationHandle_t h{};
    P(hipMemCreate(&h, sz, &prop, 0));
    P(hipMemMap((char *)base + off, sz, 0, h, 0));
    hipError_t e = hipMemSetAccess((char *)base + off, sz, &a, 1);
    printf("setaccess 8G chunk: %s\n", e == hipSuccess ? "ok" : hipGetErrorString(e));
    if (e != hipSuccess) {
      e = hipMemSetAccess(base, off + sz, &a, 1);
      printf("setaccess whole: %s\n", e == hipSuccess ? "ok" : hipGetErrorString(e));
    }
    off += sz;
    P(hipMemsetAsync(base, 0, off, nullptr));
    P(hipDeviceSynchronize());
    size_t fr = 0, tot = 0;
    P(hipMemGetInfo(&fr, &tot));
    printf("free %zu total %zu\n", fr, tot);
  }
  printf("done\n");
  return 0;
}
