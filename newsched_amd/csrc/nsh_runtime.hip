// libnsh_hip.so: device, stream, event and memory entry points of include/nsh_hip.h,
// including the HIP-VMM double-mapped ring behind gr::hip_buffer.
//
// Replaces the per-buffer cudaMalloc pair + pinned host half + private stream of
// cuda_buffer (reference runtime/lib/cudabuffer.cu:17-38) and its mirror-copy
// double-buffering (cudabuffer.cu:116-176): the ring here is one physical allocation
// mapped twice, so no byte is ever copied to keep a span contiguous.
#include "nsh_common.hpp"

#include <cstring>
#include <map>
#include <mutex>

namespace nsh {
static thread_local std::string t_err;
void set_error(const std::string& msg) { t_err = msg; }
void clear_error() { t_err.clear(); }
} // namespace nsh

using namespace nsh;

// nsh_clock_sample: one wave, lane 0 reads the counters; the store is a vector store from lane 0
__global__ __launch_bounds__(64) void k_clock_sample(unsigned long long* out, unsigned long long ticks)
{
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    unsigned long long t1 = t0;
    for (int it = 0; it < (1 << 16) && t1 - t0 < ticks; ++it) { // <= 2^16 sleeps (~0.2 s at 2.4 GHz)
        __builtin_amdgcn_s_sleep(127);                            // 127 x 64 cycles
        t1 = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = c1 - c0;
    out[1] = t1 - t0;
}

extern "C" {

int nsh_abi_version(void) { return NSH_ABI_VERSION; }
const char* nsh_last_error(void) { return t_err.c_str(); }

int nsh_get_device_count(int* count)
{
    NSH_CK(hipGetDeviceCount(count));
    return 0;
}

int nsh_set_device(int dev)
{
    NSH_CK(hipSetDevice(dev));
    return 0;
}

int nsh_device_info(int dev, int* n_cu, int* clock_khz, size_t* hbm_bytes, char* arch, int arch_len)
{
    hipDeviceProp_t p;
    NSH_CK(hipGetDeviceProperties(&p, dev));
    if (n_cu) *n_cu = p.multiProcessorCount;
    if (clock_khz) *clock_khz = p.clockRate;
    if (hbm_bytes) *hbm_bytes = p.totalGlobalMem;
    if (arch && arch_len > 0) {
        std::strncpy(arch, p.gcnArchName, (size_t)arch_len - 1);
        arch[arch_len - 1] = 0;
    }
    return 0;
}

int nsh_device_pci_id(int dev, char* buf, int len)
{
    if (!buf || len < 13) return ::nsh::fail(hipErrorInvalidValue, "nsh_device_pci_id: buffer too small");
    NSH_CK(hipDeviceGetPCIBusId(buf, len, dev));
    return 0;
}

int nsh_pointer_device(const void* ptr, int* device)
{
    if (!device) return ::nsh::fail(hipErrorInvalidValue, "nsh_pointer_device: device is NULL");
    *device = -1;
    if (!ptr) return 0;
    hipPointerAttribute_t a{};
    const hipError_t e = hipPointerGetAttributes(&a, ptr);
    if (e != hipSuccess) { // pageable host memory (never registered with HIP): not device memory
        (void)hipGetLastError();
        return 0;
    }
    if (a.type == hipMemoryTypeDevice) *device = a.device;
    return 0;
}

int nsh_device_sync(void)
{
    NSH_CK(hipDeviceSynchronize());
    return 0;
}

int nsh_stream_create(int dev, void** stream)
{
    NSH_CK(hipSetDevice(dev));
    hipStream_t s;
    NSH_CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return 0;
}
int nsh_stream_destroy(void* stream)
{
    NSH_CK(hipStreamDestroy(S(stream)));
    return 0;
}
int nsh_stream_sync(void* stream)
{
    NSH_CK(hipStreamSynchronize(S(stream)));
    return 0;
}
int nsh_stream_query(void* stream)
{
    const hipError_t e = hipStreamQuery(S(stream));
    if (e == hipSuccess) return 0;
    if (e == hipErrorNotReady) return 1;
    fail(e, "hipStreamQuery");
    return -1;
}
int nsh_event_create(void** event)
{
    hipEvent_t e;
    NSH_CK(hipEventCreateWithFlags(&e, hipEventDefault));
    *event = e;
    return 0;
}
int nsh_event_destroy(void* event)
{
    NSH_CK(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
    return 0;
}
int nsh_event_record(void* event, void* stream)
{
    NSH_CK(hipEventRecord(reinterpret_cast<hipEvent_t>(event), S(stream)));
    return 0;
}
int nsh_time_next_launch(void* start_event, void* stop_event)
{
    auto& e = next_launch_events();
    e.start = reinterpret_cast<hipEvent_t>(start_event);
    e.stop = reinterpret_cast<hipEvent_t>(stop_event);
    return 0;
}
int nsh_timed_launches(uint64_t* count)
{
    if (!count) return nsh::fail_msg("nsh_timed_launches: null count");
    *count = timed_launch_count();
    return 0;
}
int nsh_clock_sample(void* out_dev, int64_t real_ticks, void* stream)
{
    if (!out_dev) return nsh::fail_msg("nsh_clock_sample: null output");
    if (real_ticks < 1 || real_ticks > ((int64_t)1 << 32)) return nsh::fail_msg("nsh_clock_sample: real_ticks out of range");
    hipLaunchKernelGGL(k_clock_sample, dim3(1), dim3(64), 0, nsh::S(stream), (unsigned long long*)out_dev,
                       (unsigned long long)real_ticks);
    NSH_CK_LAUNCH("nsh_clock_sample");
    return 0;
}

int nsh_event_query(void* event)
{
    hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(event));
    if (e == hipSuccess) return 0;
    if (e == hipErrorNotReady) return 1;
    fail(e, "hipEventQuery");
    return -1;
}
int nsh_event_sync(void* event)
{
    NSH_CK(hipEventSynchronize(reinterpret_cast<hipEvent_t>(event)));
    return 0;
}
int nsh_event_elapsed_ms(void* start, void* stop, float* ms)
{
    NSH_CK(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
    return 0;
}
int nsh_stream_wait_event(void* stream, void* event)
{
    NSH_CK(hipStreamWaitEvent(S(stream), reinterpret_cast<hipEvent_t>(event), 0));
    return 0;
}

int nsh_malloc(int dev, size_t bytes, void** ptr)
{
    NSH_CK(hipSetDevice(dev));
    NSH_CK(hipMalloc(ptr, bytes ? bytes : 16));
    return 0;
}
int nsh_free(void* ptr)
{
    NSH_CK(hipFree(ptr));
    return 0;
}
int nsh_host_alloc(size_t bytes, void** ptr)
{
    NSH_CK(hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault));
    return 0;
}
int nsh_host_free(void* ptr)
{
    NSH_CK(hipHostFree(ptr));
    return 0;
}
int nsh_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream)
{
    if (bytes == 0) return 0;
    hipMemcpyKind k = hipMemcpyDefault;
    switch (kind) {
    case NSH_H2D: k = hipMemcpyHostToDevice; break;
    case NSH_D2H: k = hipMemcpyDeviceToHost; break;
    case NSH_D2D: k = hipMemcpyDeviceToDevice; break;
    default: k = hipMemcpyDefault; break;
    }
    NSH_CK(hipMemcpyAsync(dst, src, bytes, k, S(stream)));
    return 0;
}
int nsh_memset_async(void* ptr, int value, size_t bytes, void* stream)
{
    if (bytes == 0) return 0;
    NSH_CK(hipMemsetAsync(ptr, value, bytes, S(stream)));
    return 0;
}

// ---- double-mapped ring --------------------------------------------------------------
namespace {
struct ring_rec {
    bool vmm;
    size_t bytes; // physical size (one copy)
    hipMemGenericAllocationHandle_t handle;
};
std::mutex g_ring_mtx;
std::map<void*, ring_rec> g_rings;
} // namespace

int nsh_ring_alloc(int dev, size_t min_bytes, void** base, size_t* actual_bytes, int* double_mapped)
{
    NSH_CK(hipSetDevice(dev));
    if (min_bytes == 0) min_bytes = 1;
    int vmm = 0;
    if (hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev) != hipSuccess)
        vmm = 0;
    if (vmm) {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t gran = 0;
        if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) == hipSuccess && gran) {
            const size_t sz = (min_bytes + gran - 1) / gran * gran;
            hipMemGenericAllocationHandle_t h;
            void* va = nullptr;
            bool ok = hipMemCreate(&h, sz, &prop, 0) == hipSuccess;
            if (ok) {
                ok = hipMemAddressReserve(&va, 2 * sz, 0, nullptr, 0) == hipSuccess;
                if (!ok) (void)hipMemRelease(h);
            }
            if (ok) {
                ok = hipMemMap(va, sz, 0, h, 0) == hipSuccess &&
                     hipMemMap((char*)va + sz, sz, 0, h, 0) == hipSuccess;
                if (ok) {
                    hipMemAccessDesc ad = {};
                    ad.location = prop.location;
                    ad.flags = hipMemAccessFlagsProtReadWrite;
                    ok = hipMemSetAccess(va, 2 * sz, &ad, 1) == hipSuccess;
                }
                if (!ok) {
                    (void)hipMemUnmap(va, sz);
                    (void)hipMemUnmap((char*)va + sz, sz);
                    (void)hipMemAddressFree(va, 2 * sz);
                    (void)hipMemRelease(h);
                }
            }
            if (ok) {
                std::lock_guard<std::mutex> g(g_ring_mtx);
                g_rings[va] = ring_rec{ true, sz, h };
                *base = va;
                *actual_bytes = sz;
                *double_mapped = 1;
                (void)hipGetLastError(); // clear sticky errors from probing
                return 0;
            }
            (void)hipGetLastError();
        }
    }
    // Fallback: plain allocation; the caller caps spans at the wrap point.
    void* p = nullptr;
    const size_t sz = (min_bytes + 255) / 256 * 256;
    NSH_CK(hipMalloc(&p, sz));
    std::lock_guard<std::mutex> g(g_ring_mtx);
    g_rings[p] = ring_rec{ false, sz, {} };
    *base = p;
    *actual_bytes = sz;
    *double_mapped = 0;
    return 0;
}

int nsh_ring_free(void* base)
{
    ring_rec r;
    {
        std::lock_guard<std::mutex> g(g_ring_mtx);
        auto it = g_rings.find(base);
        if (it == g_rings.end()) return fail_msg("nsh_ring_free: unknown ring base");
        r = it->second;
        g_rings.erase(it);
    }
    if (!r.vmm) {
        NSH_CK(hipFree(base));
        return 0;
    }
    NSH_CK(hipDeviceSynchronize()); // no kernel may still touch the mapping
    NSH_CK(hipMemUnmap(base, r.bytes));
    NSH_CK(hipMemUnmap((char*)base + r.bytes, r.bytes));
    NSH_CK(hipMemAddressFree(base, 2 * r.bytes));
    NSH_CK(hipMemRelease(r.handle));
    return 0;
}

// ---- inter-process device memory (p2p edge transport) ----------------------------------
static_assert(sizeof(hipIpcMemHandle_t) == NSH_IPC_HANDLE_BYTES, "hipIpcMemHandle_t size");

int nsh_ipc_mem_export(void* dev_ptr, void* handle_out)
{
    if (!dev_ptr || !handle_out) return fail(hipErrorInvalidValue, "nsh_ipc_mem_export: NULL argument");
    hipIpcMemHandle_t h;
    NSH_CK(hipIpcGetMemHandle(&h, dev_ptr));
    std::memcpy(handle_out, &h, sizeof(h));
    return 0;
}

int nsh_ipc_mem_open(int dev, const void* handle, void** ptr)
{
    if (!handle || !ptr) return fail(hipErrorInvalidValue, "nsh_ipc_mem_open: NULL argument");
    NSH_CK(hipSetDevice(dev));
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    NSH_CK(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    return 0;
}

int nsh_ipc_mem_close(void* ptr)
{
    NSH_CK(hipIpcCloseMemHandle(ptr));
    return 0;
}

} // extern "C"
