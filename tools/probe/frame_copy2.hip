// Probe: the channelizer's frame access shape (one wave per 1024-sample frame, 16 b64 loads per
// lane, then 16 stores) against the grid: G workgroups of 4 waves walking the frames grid-stride
// (frame = (b + G i) 4 + w) or blocked (workgroup b takes a contiguous run of frames), with an
// optional dependent VALU spin standing in for the transforms; 50 KiB of LDS per workgroup as
// k_chan1024 (3 resident per CU). 2^28 samples, HIP events, 2 reps.
//   build: hipcc --offload-arch=gfx950 -O3 -o build/probe/frame_copy2 tools/probe/frame_copy2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float spin(float a, int work)
{
    for (int i = 0; i < work; ++i) a = __builtin_fmaf(a, 1.0000001f, 1e-7f);
    return a;
}

template <int BLOCKED>
__global__ __launch_bounds__(256) void k_frames(const f2* __restrict__ in, f2* __restrict__ out, long nframes, int work)
{
    extern __shared__ float pad[];
    if (work < 0) pad[threadIdx.x] = 0.f; // keeps the LDS allocation
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long G = gridDim.x;
    const long per = (nframes / 4 + G - 1) / G; // blocked: frame groups of 4 per workgroup
    for (long i = 0;; ++i) {
        const long grp = BLOCKED ? (long)blockIdx.x * per + i : (long)blockIdx.x + G * i;
        if ((BLOCKED && i >= per) || grp * 4 >= nframes) break;
        const long f = grp * 4 + w;
        const f2* src = in + f * 1024;
        f2* dst = out + f * 1024;
        f2 v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = __builtin_nontemporal_load(src + j + 64 * m);
        v[0].x = spin(v[0].x, work);
#pragma unroll
        for (int m = 0; m < 16; ++m) __builtin_nontemporal_store(v[m], dst + j + 64 * m);
    }
}

int main()
{
    const long n = 1l << 28, nf = n / 1024;
    f2 *x, *y;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMemset(x, 0, n * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int lds = 50 * 1024;
    const unsigned grids[] = { 768, 1024, 4096, 16384, 65536 };
    const int works[] = { 0, 300 };
    for (int rep = 0; rep < 2; ++rep)
        for (int blocked = 0; blocked < 2; ++blocked)
            for (int work : works)
                for (unsigned grid : grids) {
                    auto k = blocked ? k_frames<1> : k_frames<0>;
                    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
                    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, x, y, nf, work);
                    CK(hipEventRecord(a, 0));
                    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, x, y, nf, work);
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    ms /= 10;
                    printf("rep %d %s work %3d grid %6u: %.1f us = %.1f %% of 8 TB/s\n", rep, blocked ? "blocked" : "stride ", work, grid,
                           ms * 1e3, 16.0 * n / (ms * 1e-3) / 8e12 * 100);
                }
    return 0;
}
