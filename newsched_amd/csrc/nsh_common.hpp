// Shared helpers for the libnsh_hip.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
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
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e ? (int)e : -1;
}
inline int fail_msg(const char* what)
{
    set_error(what);
    return -1;
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

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
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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
