// libnsh_hip.so: 1024-point complex FFT (fft_vcc forward/inverse, unnormalised) and the
// fused fft -> multiply -> ifft channelizer of BASELINE config C4.
//
// No reference counterpart (the "Num FFT Blocks" option of
// schedulers/mt/bench/cuda/bm_copy.cpp:42-43 is a mislabelled copy count). Conventions:
//   forward  X[k] = sum_n x[n] e^{-2 pi i kn/1024}            (= numpy.fft.fft)
//   inverse  x[n] = sum_k X[k] e^{+2 pi i kn/1024}            (= 1024 * numpy.fft.ifft)
//
// One 256-thread workgroup per 1024-sample frame (grid-stride over frames): Stockham
// autosort radix-4, five passes, each thread owning one radix-4 butterfly per pass; pass 0
// reads HBM (coalesced: thread j reads samples j, j+256, j+512, j+768), passes ping-pong
// through two 8 KiB LDS images, the last pass writes HBM. Twiddles come from a 1024-entry
// table computed in double on the host (accuracy ~log2(N) * 2^-24 relative).
// The channelizer keeps the spectrum in LDS between the forward and inverse transforms,
// so a frame crosses HBM once each way (16 B/sample instead of 48 B unfused).
#include "nsh_common.hpp"

#include <cmath>
#include <mutex>
#include <vector>

namespace {

constexpr int N = 1024;
constexpr int NT = 256;

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 rot(float2 a)
{
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}

// One Stockham radix-4 pass for butterfly j (0..255): Ns = size of finished sub-FFTs.
template <bool INV>
__device__ __forceinline__ void pass(float2 (&v)[4], int j, int Ns, const float2* __restrict__ tw)
{
    const int k = j & (Ns - 1);
    if (Ns > 1) {
        // twiddle exp(-+2 pi i k r / (4 Ns)) = W[k r N/(4 Ns)], W[t] = e^{-2 pi i t/N}
        const int step = (N / 4) / Ns * k;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
            float2 w = tw[(step * r) & (N - 1)];
            if (INV) w.y = -w.y;
            v[r] = cmul(v[r], w);
        }
    }
    const float2 a0 = cadd(v[0], v[2]);
    const float2 a1 = csub(v[0], v[2]);
    const float2 a2 = cadd(v[1], v[3]);
    const float2 a3 = rot<INV>(csub(v[1], v[3]));
    v[0] = cadd(a0, a2);
    v[1] = cadd(a1, a3);
    v[2] = csub(a0, a2);
    v[3] = csub(a1, a3);
}

__device__ __forceinline__ int expand(int j, int Ns) { return (j / Ns) * Ns * 4 + (j & (Ns - 1)); }

// Full transform of a frame already in LDS image `a` (natural order) -> registers of the
// last pass written to `dst` (global or LDS) in natural order.
template <bool INV, bool FROM_GLOBAL>
__device__ __forceinline__ void fft_frame(const float2* __restrict__ src, float2* __restrict__ dst,
                                          float2* __restrict__ la, float2* __restrict__ lb,
                                          const float2* __restrict__ tw, const float2* __restrict__ mulw)
{
    const int j = threadIdx.x;
    float2 v[4];
    int Ns = 1;
    const float2* cur = src;
    float2* bufs[2] = { la, lb };
    int pp = 0;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = cur[j + r * (N / 4)];
        pass<INV>(v, j, Ns, tw);
        const int e = expand(j, Ns);
        float2* o = (s == 4) ? dst : bufs[pp];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float2 y = v[r];
            if (s == 4 && mulw) y = cmul(y, mulw[e + r * Ns]);
            o[e + r * Ns] = y;
        }
        if (s < 4) {
            __syncthreads();
            cur = bufs[pp];
            pp ^= 1;
        }
        Ns *= 4;
    }
    (void)FROM_GLOBAL;
}

template <bool INV>
__global__ __launch_bounds__(NT) void k_fft1024(const float2* __restrict__ in, float2* __restrict__ out, int64_t nframes,
                                                const float2* __restrict__ tw)
{
    __shared__ float2 la[N], lb[N];
    for (int64_t f = blockIdx.x; f < nframes; f += gridDim.x) {
        fft_frame<INV, true>(in + f * N, out + f * N, la, lb, tw, nullptr);
        __syncthreads();
    }
}

__global__ __launch_bounds__(NT) void k_chan1024(const float2* __restrict__ in, float2* __restrict__ out, int64_t nframes,
                                                 const float2* __restrict__ tw, const float2* __restrict__ w)
{
    __shared__ float2 la[N], lb[N], lc[N];
    for (int64_t f = blockIdx.x; f < nframes; f += gridDim.x) {
        fft_frame<false, true>(in + f * N, lc, la, lb, tw, w); // spectrum * w -> lc
        __syncthreads();
        fft_frame<true, false>(lc, out + f * N, la, lb, tw, nullptr);
        __syncthreads();
    }
}

std::mutex g_tw_mtx;
std::vector<float2*> g_tw(64, nullptr); // per device

int twiddles(int dev, const float2** tw)
{
    std::lock_guard<std::mutex> g(g_tw_mtx);
    if (dev < 0 || dev >= (int)g_tw.size()) return nsh::fail_msg("fft: bad device");
    if (!g_tw[dev]) {
        std::vector<float2> h(N);
        for (int t = 0; t < N; ++t) {
            const double a = -2.0 * M_PI * (double)t / (double)N;
            h[t] = make_float2((float)std::cos(a), (float)std::sin(a));
        }
        float2* d = nullptr;
        NSH_CK(hipMalloc(&d, N * sizeof(float2)));
        NSH_CK(hipMemcpy(d, h.data(), N * sizeof(float2), hipMemcpyHostToDevice));
        g_tw[dev] = d;
    }
    *tw = g_tw[dev];
    return 0;
}

unsigned frame_grid(int64_t nframes)
{
    const int64_t cap = 256 * 32;
    return (unsigned)(nframes < cap ? nframes : cap);
}

} // namespace

extern "C" {

int nsh_fft1024_c2c(const float* in, float* out, int64_t nframes, int inverse, void* stream)
{
    if (nframes <= 0) return 0;
    if (in == out) return nsh::fail_msg("nsh_fft1024_c2c: in-place not supported");
    int dev = 0;
    NSH_CK(hipGetDevice(&dev));
    const float2* tw = nullptr;
    if (int rc = twiddles(dev, &tw)) return rc;
    if (inverse)
        hipLaunchKernelGGL(k_fft1024<true>, dim3(frame_grid(nframes)), dim3(NT), 0, nsh::S(stream),
                           (const float2*)in, (float2*)out, nframes, tw);
    else
        hipLaunchKernelGGL(k_fft1024<false>, dim3(frame_grid(nframes)), dim3(NT), 0, nsh::S(stream),
                           (const float2*)in, (float2*)out, nframes, tw);
    NSH_CK_LAUNCH("nsh_fft1024_c2c");
    return 0;
}

int nsh_channelizer1024(const float* in, float* out, const float* w, int64_t nframes, void* stream)
{
    if (nframes <= 0) return 0;
    if (in == out) return nsh::fail_msg("nsh_channelizer1024: in-place not supported");
    int dev = 0;
    NSH_CK(hipGetDevice(&dev));
    const float2* tw = nullptr;
    if (int rc = twiddles(dev, &tw)) return rc;
    hipLaunchKernelGGL(k_chan1024, dim3(frame_grid(nframes)), dim3(NT), 0, nsh::S(stream),
                       (const float2*)in, (float2*)out, nframes, tw, (const float2*)w);
    NSH_CK_LAUNCH("nsh_channelizer1024");
    return 0;
}

} // extern "C"
