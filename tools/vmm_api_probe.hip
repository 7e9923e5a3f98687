// VMM rule probe, API calls only: which hipMemSetAccess ranges does this ROCm accept
// on a reserved address range mapped chunk by chunk?  Nothing here touches the mapped memory -- no
// kernel, no copy, no memset -- so a rejected range cannot turn into a device fault (the round-3
// probe wrote through ranges whose access call had failed).
//   hipcc --offload-arch=gfx950 -O2 tools/vmm_api_probe.hip -o tools/vmm_api_probe && ./tools/vmm_api_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

static const char *rc(hipError_t e) { return e == hipSuccess ? "ok" : hipGetErrorString(e); }

int main() {
  int vmm = 0;
  hipError_t e = hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0);
  printf("vmm supported: %d (%s)\n", vmm, rc(e));
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gmin = 0, grec = 0;
  printf("granularity min: %s, ", rc(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum)));
  printf("rec: %s -> min %zu rec %zu\n", rc(hipMemGetAllocationGranularity(&grec, &prop, hipMemAllocationGranularityRecommended)),
         gmin, grec);
  const size_t g = grec ? grec : (2u << 20);
  hipMemAccessDesc a{};
  a.location = prop.location;
  a.flags = hipMemAccessFlagsProtReadWrite;
  // case table: chunk sizes in granules, mapped back to back from offset 0 of one reservation
  struct Case {
    const char *name;
    std::vector<size_t> chunks;
  };
  const Case cases[] = {{"equal 1g", {1, 1, 1, 1}},
                        {"growing 1,3,16", {1, 3, 16}},
                        {"growing x1.5 (dense_grow)", {64, 32, 48, 72}},
                        {"one big", {4096}}};
  for (const Case &cs : cases) {
    void *base = nullptr;
    const size_t R = 64ull << 30;
    e = hipMemAddressReserve(&base, R, g, nullptr, 0);
    printf("[%s] reserve %zu GiB align %zu: %s base %p\n", cs.name, R >> 30, g, rc(e), base);
    if (e != hipSuccess) continue;
    size_t off = 0;
    std::vector<std::pair<size_t, hipMemGenericAllocationHandle_t>> maps;
    for (size_t n : cs.chunks) {
      const size_t sz = n * g;
      hipMemGenericAllocationHandle_t h{};
      hipError_t ec = hipMemCreate(&h, sz, &prop, 0);
      hipError_t em = ec == hipSuccess ? hipMemMap((char *)base + off, sz, 0, h, 0) : ec;
      hipError_t ea = em == hipSuccess ? hipMemSetAccess((char *)base + off, sz, &a, 1) : em;
      hipError_t ew = hipSuccess;
      if (ea != hipSuccess) {
        (void)hipGetLastError();
        ew = hipMemSetAccess(base, off + sz, &a, 1);          // the whole mapped prefix instead
        (void)hipGetLastError();
      }
      printf("  chunk at +%zu MiB size %zu MiB (offset %% size = %zu): create %s map %s setaccess(chunk) %s%s%s\n",
             off >> 20, sz >> 20, sz ? off % sz : 0, rc(ec), rc(em), rc(ea), ea != hipSuccess ? " setaccess(prefix) " : "",
             ea != hipSuccess ? rc(ew) : "");
      if (em == hipSuccess) maps.emplace_back(sz, h);
      off += sz;
    }
    size_t o2 = 0;
    for (auto &m : maps) {
      (void)hipMemUnmap((char *)base + o2, m.first);
      (void)hipMemRelease(m.second);
      o2 += m.first;
    }
    (void)hipGetLastError();
    printf("  release: %s\n", rc(hipMemAddressFree(base, R)));
  }
  printf("done\n");
  return 0;
}
