// Probe: HIP VMM double mapping on the device (used to decide hip_buffer's ring strategy).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
__global__ void fill(unsigned* p, size_t n) { size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; if (i < n) p[i] = (unsigned)i; }
__global__ void check(const unsigned* p, size_t n, size_t off, int* bad) { size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; if (i < n && p[off + i] != (unsigned)i) atomicAdd(bad, 1); }
int main() {
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  printf("dev %s gcn %s CUs %d clock %d kHz mem %zu GB l2 %d\n", pr.name, pr.gcnArchName, pr.multiProcessorCount, pr.clockRate, pr.totalGlobalMem >> 30, pr.l2CacheSize);
  int vmm = 0; CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
  printf("VMM supported attr: %d\n", vmm);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned; prop.location.type = hipMemLocationTypeDevice; prop.location.id = 0;
  size_t gran = 0; CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  size_t rgran = 0; CK(hipMemGetAllocationGranularity(&rgran, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity min %zu rec %zu\n", gran, rgran);
  size_t sz = gran * 4;
  hipMemGenericAllocationHandle_t h; CK(hipMemCreate(&h, sz, &prop, 0));
  void* va = nullptr; CK(hipMemAddressReserve(&va, 2 * sz, 0, nullptr, 0));
  CK(hipMemMap(va, sz, 0, h, 0));
  CK(hipMemMap((char*)va + sz, sz, 0, h, 0));
  hipMemAccessDesc ad = {}; ad.location = prop.location; ad.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, 2 * sz, &ad, 1));
  size_t n = sz / 4;
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, (unsigned*)va, n);
  int* bad; CK(hipMalloc(&bad, 4)); CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, (const unsigned*)va, n, n, bad);
  int hb = -1; CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("mirror check bad=%d (0 means double mapping works)\n", hb);
  // write through the mirror half, read from first half
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, 0, (unsigned*)va + n, n);
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, (const unsigned*)va, n, 0, bad);
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  printf("reverse mirror check bad=%d\n", hb);
  CK(hipDeviceSynchronize());
  CK(hipMemUnmap(va, sz)); CK(hipMemUnmap((char*)va + sz, sz)); CK(hipMemAddressFree(va, 2 * sz)); CK(hipMemRelease(h));
  printf("VMM OK\n");
  return 0;
}
