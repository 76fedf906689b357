// Shared helpers for the libnsh_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <string>

#include "nsh_hip.h"

namespace nsh {

// Thread-local text of the last failure, returned by nsh_last_error().
void set_error(const std::string& msg);
void clear_error();

inline int fail(hipError_t e, const char* what)
{
    // reported here, by return code: clear HIP's per-thread last error too, or the next entry
    // point's launch check (NSH_CK_LAUNCH: hipGetLastError) would blame its own launch for it
    (void)hipGetLastError();
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e ? (int)e : -1;
}
inline int fail_msg(const char* what)
{
    set_error(what);
    return -1;
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Timing of the next kernel launch on this thread (nsh_time_next_launch): a start / stop event
// pair that the launch itself records, as part of the kernel's dispatch (hipExtLaunchKernelGGL),
// instead of two separate event packets around it on the stream. Taken (and cleared) by the first
// launch() after it was set.
struct launch_events {
    hipEvent_t start = nullptr, stop = nullptr;
};
inline launch_events& next_launch_events()
{
    static thread_local launch_events e;
    return e;
}
// Launches on this thread that recorded a pair (nsh_timed_launches): a caller that armed a pair
// tells from the count whether a launch took it or it was dropped unrecorded.
inline uint64_t& timed_launch_count()
{
    static thread_local uint64_t n = 0;
    return n;
}
template <typename K, typename... A>
inline void launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, A... args)
{
    launch_events& e = next_launch_events();
    if (e.start || e.stop) {
        const launch_events t = e;
        e = launch_events();
        ++timed_launch_count();
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t.start, t.stop, 0u, args...);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}

// The pending pair, taken (and cleared) by an entry point that times several launches as one:
// start recorded by the first kernel's dispatch, stop by the last one's (launch_timed).
inline launch_events take_launch_events()
{
    const launch_events t = next_launch_events();
    next_launch_events() = launch_events();
    return t;
}
template <typename K, typename... A>
inline void launch_timed(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, hipEvent_t start, hipEvent_t stop,
                         A... args)
{
    if (start || stop) {
        ++timed_launch_count();
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, start, stop, 0u, args...);
    } else
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}
// Clears the pending pair when an entry point returns, whatever the path (early returns, errors,
// kernels that do not consume it): an armed pair must never be recorded around a later, unrelated
// launch on this thread.
struct launch_events_guard {
    ~launch_events_guard() { next_launch_events() = launch_events(); }
};

// Grid for a grid-stride streaming kernel: enough workgroups to fill 256 CUs several
// times over, capped so each thread still walks several 16-byte vectors.
inline unsigned stream_grid(int64_t n_vec, int block)
{
    int64_t g = (n_vec + block - 1) / block;
    const int64_t cap = 256 * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (unsigned)g;
}

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup-scope fence on all
// address spaces, which on gfx950 waits for every outstanding global load and store
// (s_waitcnt vmcnt(0)) -- in a streaming kernel that drains the register prefetch of the
// next chunks at every step. Kernels whose waves share data only through LDS use this.
// The empty asm statements with a memory clobber keep the compiler from moving LDS accesses
// across the barrier: the fences alone did not stop it sinking loads issued before the barrier
// into the branches after it (seen in an experimental two-wave kernel, where the partner wave
// then overwrote the data first).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    asm volatile("" ::: "memory");
}

// Raw buffer resource over chunk ch of a stream of n items (8 B each), chunk = CH items:
// [base + CH ch, + min(n - CH ch, CH) items), at least 0. Out-of-range lanes read 0 and their
// stores are dropped, so a streaming step issues the same loads and stores for a full chunk
// and for the stream's partial last one: no per-sample branches, and the compiler's vmcnt
// waits count exactly. Built from wave-uniform values only (no waterfall loops).
template <int CH>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const float2* base, int64_t ch, int64_t n)
{
    int64_t items = n - ch * CH;
    items = items < 0 ? 0 : (items > CH ? CH : items);
    const uint64_t a = (uint64_t)(base + ch * CH);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(items * 8));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes, 0x00020000);
}
constexpr int AUX_NT = 2; // gfx950 cache policy bits: nt (streaming)
// streaming loads / stores (ablation builds override: tools/probe/build_file_abl.sh)
#ifndef NSH_AUX_LD
#define NSH_AUX_LD 2
#endif
#ifndef NSH_AUX_ST
#define NSH_AUX_ST 2
#endif
constexpr int AUX_LD = NSH_AUX_LD, AUX_ST = NSH_AUX_ST;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float buf_f4 __attribute__((ext_vector_type(4)));
typedef float buf_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 buf_load_f4(__amdgpu_buffer_rsrc_t r, int byte_off)
{
    const buf_f4 t = __builtin_bit_cast(buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, AUX_LD));
    return make_float4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ void buf_store_f2(__amdgpu_buffer_rsrc_t r, int byte_off, buf_f2 v)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, byte_off, 0, AUX_ST);
}

__device__ __forceinline__ float2 buf_load_f2(__amdgpu_buffer_rsrc_t r, int byte_off)
{
    const buf_f2 t = __builtin_bit_cast(buf_f2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, AUX_LD));
    return make_float2(t.x, t.y);
}

} // namespace nsh

#define NSH_CK(expr)                                                    \
    do {                                                                \
        hipError_t _e = (expr);                                         \
        if (_e != hipSuccess) return ::nsh::fail(_e, #expr);            \
    } while (0)

// Launch-error check: every entry point checks the launch it just issued.
#define NSH_CK_LAUNCH(what)                                             \
    do {                                                                \
        hipError_t _e = hipGetLastError();                              \
        if (_e != hipSuccess) return ::nsh::fail(_e, what);             \
    } while (0)
