// Probe: does the order in which 512 workgroups walk 16-KB chunks (the FIR's access shape:
// 256 threads x 4 x 16 B per chunk, two chunks prefetched in registers) change HBM throughput?
//   contiguous: workgroup w owns chunks [w*per, (w+1)*per)      (k_fir_mfma2)
//   interleaved: chunk = it * grid + w                          (grid-stride order)
//   runs of R:   workgroup w walks runs w, w + grid, ... of R consecutive chunks
// Usage: chunk_order [log2 samples, default 25]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef float nf4 __attribute__((ext_vector_type(4)));
constexpr int NT = 256, VPT = 4, CHUNKV = NT * VPT; // float4 per chunk (16 KB)

template <bool INTERLEAVED, int DEPTH, int R = 1>
__global__ __launch_bounds__(NT) void k(const nf4* __restrict__ in, nf4* __restrict__ out, long nchunks)
{
    const long per = (nchunks + gridDim.x - 1) / gridDim.x;
    // INTERLEAVED with R > 1: runs of R chunks dealt round-robin (nchunks % (R * grid) == 0 assumed)
    auto chunk = [&](long it) {
        return INTERLEAVED ? ((it / R) * gridDim.x + blockIdx.x) * R + it % R : blockIdx.x * per + it;
    };
    const long n_it = INTERLEAVED ? (R > 1 ? nchunks / gridDim.x : (nchunks - blockIdx.x + gridDim.x - 1) / gridDim.x)
                                  : (blockIdx.x * per >= nchunks ? 0 : (per < nchunks - blockIdx.x * per ? per : nchunks - blockIdx.x * per));
    if (n_it <= 0) return;
    auto load = [&](nf4 (&v)[VPT], long it) {
        const long c = chunk(it < n_it ? it : n_it - 1);
#pragma unroll
        for (int u = 0; u < VPT; ++u) v[u] = __builtin_nontemporal_load(in + c * CHUNKV + threadIdx.x + NT * u);
    };
    auto store = [&](const nf4 (&v)[VPT], long it) {
        const long c = chunk(it);
#pragma unroll
        for (int u = 0; u < VPT; ++u) __builtin_nontemporal_store(v[u], out + c * CHUNKV + threadIdx.x + NT * u);
    };
    nf4 va[VPT], vb[VPT], vc[VPT];
    load(va, 0);
    if (DEPTH == 1) {
        long it = 0;
        for (; it + 1 < n_it; it += 2) {
            load(vb, it + 1); store(va, it);
            load(va, it + 2); store(vb, it + 1);
        }
        if (it < n_it) store(va, it);
    } else {
        load(vb, 1);
        long it = 0;
        for (; it + 2 < n_it; it += 3) {
            load(vc, it + 2); store(va, it);
            load(va, it + 3); store(vb, it + 1);
            load(vb, it + 4); store(vc, it + 2);
        }
        if (it < n_it) { store(va, it); ++it; }
        if (it < n_it) store(vb, it);
    }
}

int main(int argc, char** argv)
{
    const long n = 1L << (argc > 1 ? atoi(argv[1]) : 25); // complex samples
    const long nv = n / 2, nchunks = nv / CHUNKV;
    nf4 *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        float best = 1e9, sum = 0;
        for (int r = 0; r < 10; ++r) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms; sum += ms;
        }
        printf("%-36s min %7.1f us avg %7.1f us  %6.0f GB/s\n", name, best * 1e3, sum * 100, 16.0 * n / (best * 1e-3) / 1e9);
    };
    {
        char nm[64];
        snprintf(nm, 64, "runs of 16, d2 grid 512"); run(nm, [&] { hipLaunchKernelGGL((k<true, 2, 16>), dim3(512), dim3(NT), 0, 0, a, b, nchunks); });
        snprintf(nm, 64, "runs of 64, d2 grid 512"); run(nm, [&] { hipLaunchKernelGGL((k<true, 2, 64>), dim3(512), dim3(NT), 0, 0, a, b, nchunks); });
    }
    for (int g : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, 64, "contiguous d1 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k<false, 1>), dim3(g), dim3(NT), 0, 0, a, b, nchunks); });
        snprintf(nm, 64, "contiguous d2 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k<false, 2>), dim3(g), dim3(NT), 0, 0, a, b, nchunks); });
        snprintf(nm, 64, "interleaved d2 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k<true, 2>), dim3(g), dim3(NT), 0, 0, a, b, nchunks); });
        snprintf(nm, 64, "interleaved d1 grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k<true, 1>), dim3(g), dim3(NT), 0, 0, a, b, nchunks); });
    }
    return 0;
}
