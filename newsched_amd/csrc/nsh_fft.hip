// libnsh_hip.so: 1024-point complex FFT (fft_vcc forward/inverse, unnormalised) and the
// fused fft -> multiply -> ifft channelizer of BASELINE config C4.
//
// No reference counterpart (the "Num FFT Blocks" option of
// schedulers/mt/bench/cuda/bm_copy.cpp:42-43 is a mislabelled copy count). Conventions:
//   forward  X[k] = sum_n x[n] e^{-2 pi i kn/1024}            (= numpy.fft.fft)
//   inverse  x[n] = sum_k X[k] e^{+2 pi i kn/1024}            (= 1024 * numpy.fft.ifft)
//
// One wavefront per 1024-sample frame (4 frames per 256-thread workgroup, grid-stride):
// Stockham autosort in three passes, radix 16 / 16 / 4, each lane owning 16 samples:
//   pass 1 (Ns = 1):   lane j loads x[j + 64 r] (coalesced), DFT16 in registers -> LDS
//   pass 2 (Ns = 16):  reads LDS[j + 64 r], twiddles W_256^{k r}, DFT16 -> LDS
//   pass 3 (Ns = 256): 4 radix-4 butterflies per lane, twiddles W_1024^{k r} -> HBM
// DFT16 = 4 x DFT4, internal W_16 twiddles, 4 x DFT4 (index transpose at compile time). The
// LDS image (one per wave, 8.5 KiB) has one pad sample per 16 so every exchange is
// bank-conflict-free; a wave's LDS operations complete in order, so the passes need no
// workgroup barriers. Twiddles come from a 1024-entry table computed in double on the host
// and staged in LDS once per workgroup. The next frame's samples are prefetched into
// registers while the current frame transforms. The channelizer multiplies the spectrum
// by W in registers and runs the inverse transform directly: pass 3 leaves lane j holding
// indices j + 64 m (m < 16), exactly pass 1's input layout, so a frame crosses HBM once
// each way (16 B/sample instead of 48 B unfused) and LDS twice per transform.
#include "nsh_common.hpp"
#include "nsh_cplx.hpp"

#include <cmath>
#include <mutex>
#include <vector>

namespace {

constexpr int N = 1024;
constexpr int NT = 256;

using nsh::cf;
using nsh::cmulw;
using nsh::dft4;
using nsh::rot;

// the channelizer's spectrum multiply: nsh_mul_const_vcc's two-product rounding exactly, so
// the fused channelizer stays bit-identical to fft -> multiply_const_vcc -> ifft
__device__ __forceinline__ cf cmul_rn(cf a, cf b)
{
    const cf t = a.xx * b;    // (ax bx, ax by), each product rounded
    const cf u = a.yy * b.yx; // (ay by, ay bx)
    return t + u * cf{ -1.f, 1.f }; // (ax bx - ay by, ax by + ay bx): exact sign flip, one rounding
}
// W_16^m, m = 0..9 (forward; conjugated for the inverse)
template <bool INV>
__device__ __forceinline__ cf w16(int m)
{
    constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R2 = 0.70710678118654757f;
    cf w;
    switch (m) {
    case 1: w = cf{ C1, -S1 }; break;
    case 2: w = cf{ R2, -R2 }; break;
    case 3: w = cf{ S1, -C1 }; break;
    case 4: w = cf{ 0.f, -1.f }; break;
    case 6: w = cf{ -R2, -R2 }; break;
    case 9: w = cf{ -C1, S1 }; break;
    default: w = cf{ 1.f, 0.f }; break;
    }
    if (INV) w.y = -w.y;
    return w;
}

// In-place DFT16, natural order in and out: n = 4 n1 + n2, k = k1 + 4 k2,
// X[k] = sum_n2 W_4^{n2 k2} W_16^{n2 k1} sum_n1 x[4 n1 + n2] W_4^{n1 k1}.
template <bool INV>
__device__ __forceinline__ void dft16(cf (&v)[16])
{
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4<INV>(v[n2], v[n2 + 4], v[n2 + 8], v[n2 + 12]); // v[n2 + 4 k1] = Y[n2][k1]
#pragma unroll
    for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
        for (int k1 = 1; k1 < 4; ++k1) {
            const int m = n2 * k1;
            if (m == 4) // W_16^4 = -+i
                v[n2 + 4 * k1] = rot<INV>(v[n2 + 4 * k1]);
            else
                v[n2 + 4 * k1] = cmulw(v[n2 + 4 * k1], w16<INV>(m));
        }
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4<INV>(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]); // v[4 k1 + k2] = X[k1 + 4 k2]
    cf t[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = v[4 * k1 + k2];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = t[k];
}

constexpr int WLDS = N + N / 16; // one wave's padded image
__device__ __forceinline__ int pad(int i) { return i + (i >> 4); }

template <bool INV>
__device__ __forceinline__ cf conj_if(cf w)
{
    if (INV) w.y = -w.y;
    return w;
}

// The passes' twiddles, staged per workgroup. Read from the natural 1024-entry table (the default),
// pass 2's W_1024^{4 k r} (k = lane & 15) puts the 16 lanes of a read group at stride 4 r entries --
// 4- to 16-way LDS bank conflicts (PMC: 36 % of the channelizer's LDS-active cycles are conflict
// cycles) -- and pass 3's W^{2 j'} at stride 2. NSH_FFT_TW_READORDER=1 (a probe, round 6) stages them
// in the order the lanes read them instead, the same floats (bit-identical outputs):
//   T2[r][k]      = W_1024^{4 k r}   (r, k < 16: a read group's lanes take 16 consecutive entries)
//   T3[r - 1][j'] = W_1024^{r j'}    (r = 1..3, j' < 256: consecutive lanes, consecutive entries)
// Conflict-free, and no faster: channelizer 765-769 vs 763-764 us, fft1024 707-708 vs 704 us per
// 2^28 samples, both orders (profiles/r06e_chan_twiddle_layout_ab.log) -- LDS does not bound them.
#ifndef NSH_FFT_TW_READORDER
#define NSH_FFT_TW_READORDER 0
#endif
constexpr int T2N = 16 * 16, T3N = 3 * 256, TWN = NSH_FFT_TW_READORDER ? T2N + T3N : N;
__device__ __forceinline__ void stage_twiddles(cf* __restrict__ t, const float2* __restrict__ tw_g, int tid, int nt)
{
    for (int i = tid; i < TWN; i += nt) {
        int e = i;
        if (NSH_FFT_TW_READORDER)
            e = i < T2N ? (4 * (i & 15) * (i >> 4)) & (N - 1) : ((1 + (i - T2N) / 256) * ((i - T2N) & 255)) & (N - 1);
        t[i] = cf{ tw_g[e].x, tw_g[e].y };
    }
}
// pass 2's W_1024^{4 k2 r} and pass 3's W_1024^{r jp} (r = 1..3) from the staged table
template <bool INV>
__device__ __forceinline__ cf tw_pass2(const cf* __restrict__ tw, int k2, int r)
{
    return conj_if<INV>(NSH_FFT_TW_READORDER ? tw[16 * r + k2] : tw[(4 * k2 * r) & (N - 1)]);
}
template <bool INV>
__device__ __forceinline__ cf tw_pass3(const cf* __restrict__ tw, int jp, int r)
{
    return conj_if<INV>(NSH_FFT_TW_READORDER ? tw[T2N + 256 * (r - 1) + jp] : tw[(r * jp) & (N - 1)]);
}

// Transform of one frame held as v[m] = x[lane + 64 m]; on return v[m] = X[lane + 64 m]
// (pass 3 output kept in registers: m = b + 4 r for butterfly b, output r). tw: the staged table.
template <bool INV>
__device__ __forceinline__ void fft_wave(cf (&v)[16], cf* __restrict__ img, const cf* __restrict__ tw)
{
    const int j = threadIdx.x & 63;
    // pass 1: Ns = 1, radix 16 -> dst[16 j + r]
    dft16<INV>(v);
#pragma unroll
    for (int r = 0; r < 16; ++r) img[pad(16 * j + r)] = v[r];
    __builtin_amdgcn_wave_barrier();
    // pass 2: Ns = 16, radix 16: src[j + 64 r], twiddle W_256^{k r} = W_1024^{4 k r} -> dst[(j >> 4) 256 + k + 16 r]
    const int k2 = j & 15;
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = img[pad(j + 64 * r)];
#pragma unroll
    for (int r = 1; r < 16; ++r) v[r] = cmulw(v[r], tw_pass2<INV>(tw, k2, r));
    dft16<INV>(v);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) img[pad((j >> 4) * 256 + k2 + 16 * r)] = v[r];
    __builtin_amdgcn_wave_barrier();
    // pass 3: Ns = 256, radix 4; butterfly b of this lane: j' = j + 64 b, src[j' + 256 r],
    // twiddle W_1024^{j' r}, output index j' + 256 r  -> v[b + 4 r]
    cf o[16];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int jp = j + 64 * b;
        cf a0 = img[pad(jp)], a1 = img[pad(jp + 256)], a2 = img[pad(jp + 512)], a3 = img[pad(jp + 768)];
        a1 = cmulw(a1, tw_pass3<INV>(tw, jp, 1));
        a2 = cmulw(a2, tw_pass3<INV>(tw, jp, 2));
        a3 = cmulw(a3, tw_pass3<INV>(tw, jp, 3));
        dft4<INV>(a0, a1, a2, a3);
        o[b] = a0;
        o[b + 4] = a1;
        o[b + 8] = a2;
        o[b + 12] = a3;
    }
    __builtin_amdgcn_wave_barrier(); // the image is rewritten by this wave's next transform
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = o[m];
}

// Frame f of a stream of nframes frames by buffer loads/stores over that frame alone: a frame
// past the end reads zeros and drops its stores, so the loop issues the same memory
// instructions every iteration (no conditional prefetch) and the compiler's vmcnt waits stay
// exact -- the next frame's loads remain in flight across this frame's transform and stores.
__device__ __forceinline__ void load_frame16(cf (&v)[16], const float2* __restrict__ in, int64_t f, int64_t nframes)
{
    const int j = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r = nsh::chunk_rsrc<N>(in, f, nframes * N);
#pragma unroll
    for (int m = 0; m < 16; ++m)
        v[m] = __builtin_bit_cast(cf, __builtin_amdgcn_raw_buffer_load_b64(r, (j + 64 * m) * 8, 0, nsh::AUX_LD));
}
__device__ __forceinline__ void store_frame16(const cf (&v)[16], float2* __restrict__ out, int64_t f, int64_t nframes)
{
    const int j = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t r = nsh::chunk_rsrc<N>(out, f, nframes * N);
#pragma unroll
    for (int m = 0; m < 16; ++m) nsh::buf_store_f2(r, (j + 64 * m) * 8, v[m]);
}

constexpr int FPW = NT / 64; // frames (waves) per workgroup

template <bool INV>
__global__ __launch_bounds__(NT) void k_fft1024(const float2* __restrict__ in, float2* __restrict__ out, int64_t nframes,
                                                const float2* __restrict__ tw_g)
{
    __shared__ cf tw[TWN];
    __shared__ cf img_all[FPW * WLDS];
    stage_twiddles(tw, tw_g, threadIdx.x, NT);
    __syncthreads();
    cf* img = img_all + (threadIdx.x >> 6) * WLDS;
    const int64_t stride = (int64_t)gridDim.x * FPW;
    int64_t f = (int64_t)blockIdx.x * FPW + (threadIdx.x >> 6);
    if (f >= nframes) return;
    cf v[16], nx[16];
    load_frame16(v, in, f, nframes);
    for (; f < nframes; f += stride) {
        load_frame16(nx, in, f + stride, nframes);
        fft_wave<INV>(v, img, tw);
        store_frame16(v, out, f, nframes);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = nx[m];
    }
}

// No register prefetch of the next frame here (unlike k_fft1024): without it and with the
// weights in LDS the kernel fits 168 VGPRs, i.e. 3 workgroups (12 waves) per CU, and that
// occupancy hides the load latency better: 816 vs 858 us per 2^28 samples
// (tools/probe/fft_ab.py history in DESIGN.md section 4).
#ifndef NSH_CHAN_FPW
#define NSH_CHAN_FPW 4
#endif
constexpr int CFPW = NSH_CHAN_FPW; // channelizer frames (waves) per workgroup
// probe knobs (round 6): the next frame prefetched into registers as in k_fft1024, and the launch
// bounds' minimum workgroups per CU (2 lets the compiler take up to 256 VGPRs: 2 waves per SIMD)
#ifndef NSH_CHAN_PREFETCH
#define NSH_CHAN_PREFETCH 0
#endif
#ifndef NSH_CHAN_MINWG
#define NSH_CHAN_MINWG 2
#endif
template <int FW>
__global__ __launch_bounds__(64 * FW, FW == 4 ? NSH_CHAN_MINWG : 1) void k_chan1024(const float2* __restrict__ in, float2* __restrict__ out, int64_t nframes,
                                                    const float2* __restrict__ tw_g, const float2* __restrict__ w)
{
    __shared__ cf tw[TWN];
    __shared__ cf wl[N];
    __shared__ cf img_all[FW * WLDS];
    stage_twiddles(tw, tw_g, threadIdx.x, 64 * FW);
    for (int t = threadIdx.x; t < N; t += 64 * FW) wl[t] = cf{ w[t].x, w[t].y };
    __syncthreads();
    cf* img = img_all + (threadIdx.x >> 6) * WLDS;
    const int j = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * FW;
    cf v[16];
#if NSH_CHAN_PREFETCH
    int64_t f = (int64_t)blockIdx.x * FW + (threadIdx.x >> 6);
    if (f >= nframes) return;
    cf nx[16];
    load_frame16(v, in, f, nframes);
    for (; f < nframes; f += stride) {
        load_frame16(nx, in, f + stride, nframes);
        fft_wave<false>(v, img, tw);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = cmul_rn(v[m], wl[j + 64 * m]);
        fft_wave<true>(v, img, tw);
        store_frame16(v, out, f, nframes);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = nx[m];
    }
#else
    for (int64_t f = (int64_t)blockIdx.x * FW + (threadIdx.x >> 6); f < nframes; f += stride) {
        load_frame16(v, in, f, nframes);
        fft_wave<false>(v, img, tw);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = cmul_rn(v[m], wl[j + 64 * m]);
        fft_wave<true>(v, img, tw);
        store_frame16(v, out, f, nframes);
    }
#endif
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

// Workgroups of the grid-stride walk over frames: enough that each walks only a few frame groups.
// With 4096 (16 groups each) the last long-running workgroups left CUs idle at the end of a 2^28
// launch: 16384 workgroups run the channelizer 5 % faster (806 -> 754-774 us, 66.5 -> 69.4-71.2 %),
// 24576 the fft1024 13 % faster (768 -> 670 us = 80 % of 8 TB/s); 65536 (one frame per wave, the
// tables staged per frame) is slower for both (r05zt, r05zu: both orders, bit-identical).
#ifndef NSH_FFT_CAP
#define NSH_FFT_CAP 24576
#endif
#ifndef NSH_CHAN_CAP4
#define NSH_CHAN_CAP4 16384
#endif
#ifndef NSH_CHAN_CAP
#define NSH_CHAN_CAP (65536 / NSH_CHAN_FPW) // probe builds with NSH_CHAN_FPW != 4: the same frames per workgroup step
#endif
unsigned frame_grid(int64_t nframes, int fw, int64_t cap)
{
    const int64_t groups = (nframes + fw - 1) / fw;
    return (unsigned)(groups < cap ? groups : cap);
}

} // namespace

extern "C" {

int nsh_fft1024_c2c(const float* in, float* out, int64_t nframes, int inverse, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (nframes <= 0) return 0;
    if (!in || !out) return nsh::fail_msg("nsh_fft1024_c2c: null pointer");
    if (in == out) return nsh::fail_msg("nsh_fft1024_c2c: in-place not supported");
    int dev = 0;
    NSH_CK(hipGetDevice(&dev));
    const float2* tw = nullptr;
    if (int rc = twiddles(dev, &tw)) return rc;
    if (inverse)
        nsh::launch(k_fft1024<true>, dim3(frame_grid(nframes, FPW, NSH_FFT_CAP)), dim3(NT), 0, nsh::S(stream),
                           (const float2*)in, (float2*)out, nframes, tw);
    else
        nsh::launch(k_fft1024<false>, dim3(frame_grid(nframes, FPW, NSH_FFT_CAP)), dim3(NT), 0, nsh::S(stream),
                           (const float2*)in, (float2*)out, nframes, tw);
    NSH_CK_LAUNCH("nsh_fft1024_c2c");
    return 0;
}

int nsh_channelizer1024(const float* in, float* out, const float* w, int64_t nframes, void* stream)
{
    nsh::launch_events_guard timing_guard; // an armed event pair never outlives this call
    if (nframes <= 0) return 0;
    if (!in || !out || !w) return nsh::fail_msg("nsh_channelizer1024: null pointer");
    if (in == out) return nsh::fail_msg("nsh_channelizer1024: in-place not supported");
    int dev = 0;
    NSH_CK(hipGetDevice(&dev));
    const float2* tw = nullptr;
    if (int rc = twiddles(dev, &tw)) return rc;
    nsh::launch(k_chan1024<CFPW>, dim3(frame_grid(nframes, CFPW, CFPW == 4 ? NSH_CHAN_CAP4 : NSH_CHAN_CAP)), dim3(64 * CFPW), 0, nsh::S(stream),
                       (const float2*)in, (float2*)out, nframes, tw, (const float2*)w);
    NSH_CK_LAUNCH("nsh_channelizer1024");
    return 0;
}

} // extern "C"
