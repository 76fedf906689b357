// Probe: which access shapes copy at the HBM ceiling, and how occupancy changes that.
// Every kernel moves 2^N complex samples (16 B per sample: 8 read + 8 written) in 16-KB chunks
// (256 threads x 4 x 16 B). Variants:
//   tiles      : k_copy_v4's blocked grid-stride (grid G, chunk = it * G + w)
//   contiguous : workgroup w owns chunks [w*per, (w+1)*per), register prefetch depth 2
//                (the FIR's shape)
// Occupancy is forced with dynamic LDS (workgroups per CU = floor(160 KiB / lds)).
// Usage: shape_probe [log2 samples, default 28]   (build: tools/probe/build_probes.sh shape_probe)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("FAIL %s %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float nf4 __attribute__((ext_vector_type(4)));
constexpr int NT = 256, VPT = 4, CHUNKV = NT * VPT; // float4 per chunk (16 KB)

__device__ __forceinline__ void touch_lds()
{
    extern __shared__ unsigned char lds[];
    if (threadIdx.x == 1023) lds[0] = 1; // never true: keeps the allocation
}

__global__ __launch_bounds__(NT) void k_tiles(const nf4* __restrict__ in, nf4* __restrict__ out, long nchunks)
{
    touch_lds();
    for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
        nf4 v[VPT];
#pragma unroll
        for (int u = 0; u < VPT; ++u) v[u] = __builtin_nontemporal_load(in + c * CHUNKV + threadIdx.x + NT * u);
#pragma unroll
        for (int u = 0; u < VPT; ++u) __builtin_nontemporal_store(v[u], out + c * CHUNKV + threadIdx.x + NT * u);
    }
}

// contiguous ranges, depth-2 register prefetch (chunk it+2 loaded while it is stored)
template <int DEPTH>
__global__ __launch_bounds__(NT) void k_contig(const nf4* __restrict__ in, nf4* __restrict__ out, long nchunks)
{
    touch_lds();
    const long per = (nchunks + gridDim.x - 1) / gridDim.x;
    const long c0 = blockIdx.x * per;
    const long n_it = c0 >= nchunks ? 0 : (per < nchunks - c0 ? per : nchunks - c0);
    if (n_it <= 0) return;
    auto load = [&](nf4 (&v)[VPT], long it) {
        const long c = c0 + (it < n_it ? it : n_it - 1);
#pragma unroll
        for (int u = 0; u < VPT; ++u) v[u] = __builtin_nontemporal_load(in + c * CHUNKV + threadIdx.x + NT * u);
    };
    auto store = [&](const nf4 (&v)[VPT], long it) {
#pragma unroll
        for (int u = 0; u < VPT; ++u) __builtin_nontemporal_store(v[u], out + (c0 + it) * CHUNKV + threadIdx.x + NT * u);
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

// R consecutive chunks per workgroup, grid = nchunks / R, all loads of a chunk issued before
// its stores, the next chunk's loads before this chunk's stores (depth 1). XCD: consecutive
// workgroup ids go round-robin to the 8 XCDs; with XCD remapping XCD x walks its own
// contiguous eighth of the stream. HALO: each workgroup also loads the 1 KiB before its first
// chunk (default cache policy). TAPS: each wave loads 20 KiB of L2-resident "tap fragments".
template <int R, bool XCD, bool HALO, bool TAPS>
__global__ __launch_bounds__(NT) void k_runs(const nf4* __restrict__ in, nf4* __restrict__ out, long nchunks,
                                             const nf4* __restrict__ taps)
{
    touch_lds();
    long w = blockIdx.x;
    if (XCD) {
        const long per_x = gridDim.x / 8;
        w = (blockIdx.x % 8) * per_x + blockIdx.x / 8;
    }
    const long c0 = w * R;
    nf4 acc = {};
    if (TAPS) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < 20; ++j) acc += taps[j * 64 + lane];
    }
    if (HALO && c0 > 0 && threadIdx.x < 64) acc += in[c0 * CHUNKV - 64 + threadIdx.x];
    nf4 va[VPT], vb[VPT];
#pragma unroll
    for (int u = 0; u < VPT; ++u) va[u] = __builtin_nontemporal_load(in + c0 * CHUNKV + threadIdx.x + NT * u);
#pragma unroll
    for (int it = 0; it < R; ++it) {
        nf4 (&cur)[VPT] = (it & 1) ? vb : va;
        nf4 (&nxt)[VPT] = (it & 1) ? va : vb;
        if (it + 1 < R) {
#pragma unroll
            for (int u = 0; u < VPT; ++u) nxt[u] = __builtin_nontemporal_load(in + (c0 + it + 1) * CHUNKV + threadIdx.x + NT * u);
        }
        if (TAPS || HALO) cur[0] += acc * 0.f;
#pragma unroll
        for (int u = 0; u < VPT; ++u) __builtin_nontemporal_store(cur[u], out + (c0 + it) * CHUNKV + threadIdx.x + NT * u);
    }
}

int main(int argc, char** argv)
{
    const long n = 1L << (argc > 1 ? atoi(argv[1]) : 28); // complex samples
    const long nv = n / 2, nchunks = nv / CHUNKV;
    nf4 *a, *b;
    CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 8));
    CK(hipFuncSetAttribute((const void*)k_tiles, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_contig<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)k_contig<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 20; ++w) launch();
        float best = 1e9, sum = 0;
        const int R = 30;
        for (int r = 0; r < R; ++r) {
            hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms; sum += ms;
        }
        printf("%-44s min %7.1f us avg %7.1f us  %6.0f GB/s (avg)\n", name, best * 1e3, sum / R * 1e3,
               16.0 * n / (sum / R * 1e-3) / 1e9);
        fflush(stdout);
    };
    char nm[96];
    nf4* taps;
    CK(hipMalloc(&taps, 20 * 64 * 16));
    CK(hipMemset(taps, 0, 20 * 64 * 16));
#define RUNS(R, X, H, T) \
    CK(hipFuncSetAttribute((const void*)k_runs<R, X, H, T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024)); \
    snprintf(nm, 96, "runs R=%d xcd=%d halo=%d taps=%d, %d WG/CU", R, X, H, T, wpc); \
    run(nm, [&] { hipLaunchKernelGGL((k_runs<R, X, H, T>), dim3(nchunks / R), dim3(NT), lds, 0, a, b, nchunks, taps); });
    if (getenv("RUNS_ONLY")) {
        for (int wpc : {2, 3, 4}) {
            const size_t lds = (160 * 1024) / wpc - 1024;
            snprintf(nm, 96, "tiles grid 65536, %d WG/CU", wpc);
            run(nm, [&] { hipLaunchKernelGGL(k_tiles, dim3(65536), dim3(NT), lds, 0, a, b, nchunks); });
            RUNS(1, false, false, false) RUNS(2, false, false, false) RUNS(4, false, false, false) RUNS(8, false, false, false)
            RUNS(1, true, false, false) RUNS(2, true, false, false) RUNS(4, true, false, false) RUNS(8, true, false, false)
            RUNS(1, false, true, false) RUNS(2, false, true, false) RUNS(4, false, true, false)
            RUNS(1, true, true, false) RUNS(2, true, true, false) RUNS(4, true, true, false)
            RUNS(1, false, true, true) RUNS(2, false, true, true) RUNS(4, false, true, true) RUNS(8, false, true, true)
            RUNS(2, true, true, true) RUNS(4, true, true, true) RUNS(8, true, true, true)
        }
        return 0;
    }
    for (int wpc : {1, 2, 3, 4, 8}) { // workgroups per CU, by LDS
        const size_t lds = wpc >= 8 ? 0 : (160 * 1024) / wpc - 1024;
        for (int g : {65536, 4096, 1024}) {
            snprintf(nm, 96, "tiles grid %d, %d WG/CU", g, wpc);
            run(nm, [&] { hipLaunchKernelGGL(k_tiles, dim3(g), dim3(NT), lds, 0, a, b, nchunks); });
        }
        for (int g : {512, 1024, 2048, 4096, 8192}) {
            snprintf(nm, 96, "contiguous d2 grid %d, %d WG/CU", g, wpc);
            run(nm, [&] { hipLaunchKernelGGL(k_contig<2>, dim3(g), dim3(NT), lds, 0, a, b, nchunks); });
        }
        snprintf(nm, 96, "contiguous d1 grid 4096, %d WG/CU", wpc);
        run(nm, [&] { hipLaunchKernelGGL(k_contig<1>, dim3(4096), dim3(NT), lds, 0, a, b, nchunks); });
    }
    return 0;
}
