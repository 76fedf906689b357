// Probe: the 1024-sample-frame access shape of k_chan1024 / k_fft1024 without their arithmetic.
// One wave per frame, 4 waves per workgroup, grid-stride over frames; each lane loads its 16
// samples (b64: x[j + 64 m]; or b128: samples 2j, 2j+1 of 8 rows of 128), optionally spins for
// `work` iterations of a dependent VALU chain (a stand-in for the transforms), stores them.
// `lds` pads the workgroup's LDS (resident workgroups per CU). 2^28 samples, HIP events.
//   build: hipcc --offload-arch=gfx950 -O3 -o build/probe/frame_copy tools/probe/frame_copy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float spin(float a, int work)
{
    for (int i = 0; i < work; ++i) a = __builtin_fmaf(a, 1.0000001f, 1e-7f);
    return a;
}

template <int W128>
__global__ __launch_bounds__(256) void k_frames(const f2* __restrict__ in, f2* __restrict__ out, long nframes, int work)
{
    extern __shared__ float pad[];
    if (work < 0) pad[threadIdx.x] = 0.f; // keeps the LDS allocation
    const int j = threadIdx.x & 63;
    const long stride = (long)gridDim.x * 4;
    for (long f = (long)blockIdx.x * 4 + (threadIdx.x >> 6); f < nframes; f += stride) {
        const f2* src = in + f * 1024;
        f2* dst = out + f * 1024;
        if (W128) {
            f4 v[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src) + j + 64 * m);
            float a = spin(v[0].x, work);
            v[0].x = a;
#pragma unroll
            for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(v[m], reinterpret_cast<f4*>(dst) + j + 64 * m);
        } else {
            f2 v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = __builtin_nontemporal_load(src + j + 64 * m);
            float a = spin(v[0].x, work);
            v[0].x = a;
#pragma unroll
            for (int m = 0; m < 16; ++m) __builtin_nontemporal_store(v[m], dst + j + 64 * m);
        }
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
    const int works[] = { 0, 200, 400, 800 };
    const int ldss[] = { 50 * 1024, 38 * 1024 };
    for (int rep = 0; rep < 2; ++rep)
        for (int w128 = 0; w128 < 2; ++w128)
            for (int lds : ldss)
                for (int work : works) {
                    auto k = w128 ? k_frames<1> : k_frames<0>;
                    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
                    const unsigned grid = 4096;
                    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, x, y, nf, work);
                    CK(hipEventRecord(a, 0));
                    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, x, y, nf, work);
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    ms /= 10;
                    printf("rep %d %s lds %2d KiB work %4d: %.1f us = %.1f %% of 8 TB/s\n", rep, w128 ? "b128" : "b64 ", lds / 1024,
                           work, ms * 1e3, 16.0 * n / (ms * 1e-3) / 8e12 * 100);
                }
    return 0;
}
