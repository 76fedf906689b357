// Probe: HBM streaming copy variants on gfx950 (what access shape reaches the roofline?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef float nf4 __attribute__((ext_vector_type(4)));

template <int NT_HINT, int UNROLL>
__global__ __launch_bounds__(256) void k_copy(const nf4* __restrict__ in, nf4* __restrict__ out, long nv)
{
    const long stride = (long)gridDim.x * 256 * UNROLL;
    for (long base = (long)blockIdx.x * 256 * UNROLL + threadIdx.x; base < nv; base += stride) {
        nf4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            long i = base + u * 256;
            if (i < nv) v[u] = NT_HINT ? __builtin_nontemporal_load(in + i) : in[i];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            long i = base + u * 256;
            if (i < nv) { if (NT_HINT) __builtin_nontemporal_store(v[u], out + i); else out[i] = v[u]; }
        }
    }
}
// contiguous per-block chunk (like the FIR's per-WG ranges)
template <int UNROLL>
__global__ __launch_bounds__(256) void k_copy_chunked(const nf4* __restrict__ in, nf4* __restrict__ out, long nv)
{
    const long per = (nv + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < nv ? b0 + per : nv;
    for (long base = b0 + threadIdx.x; base < b1; base += 256 * UNROLL) {
        nf4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) { long i = base + u * 256; if (i < b1) v[u] = in[i]; }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) { long i = base + u * 256; if (i < b1) out[i] = v[u]; }
    }
}

int main()
{
    const long n = 1L << 28; // complex samples
    const long nv = n / 2;   // float4
    nf4 *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-40s %8.1f us  %7.0f GB/s\n", name, best * 1e3, 16.0 * n / (best * 1e-3) / 1e9);
    };
    for (int g : {1024, 2048, 4096, 8192, 16384, 65536}) {
        char nm[64];
        snprintf(nm, 64, "plain u1 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy<0, 1>), dim3(g), dim3(256), 0, 0, a, b, nv); });
        snprintf(nm, 64, "nt u1 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy<1, 1>), dim3(g), dim3(256), 0, 0, a, b, nv); });
        snprintf(nm, 64, "plain u4 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy<0, 4>), dim3(g), dim3(256), 0, 0, a, b, nv); });
        snprintf(nm, 64, "nt u4 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy<1, 4>), dim3(g), dim3(256), 0, 0, a, b, nv); });
    }
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, 64, "chunked u4 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy_chunked<4>), dim3(g), dim3(256), 0, 0, a, b, nv); });
        snprintf(nm, 64, "chunked u8 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_copy_chunked<8>), dim3(g), dim3(256), 0, 0, a, b, nv); });
    }
    run("hipMemcpyAsync D2D", [&] { hipMemcpyAsync(b, a, n * 8, hipMemcpyDeviceToDevice, 0); });
    // read-only and write-only ceilings
    return 0;
}
