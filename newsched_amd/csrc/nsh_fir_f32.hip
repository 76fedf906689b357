// libnsh_hip.so: fir_filter_ccf in exact fp32 on the matrix cores (NSH_FIR_MFMA_F32, decim 1).
//
// The same blocked Toeplitz GEMM as the split forms (nsh_fir_mfma.hip), on 16-sample blocks
// and the fp32-input v_mfma_f32_16x16x4_f32: no operand split, no scaling, every product and
// sum an fp32 FMA, so the result is the fp32 direct form's up to the order of the sums
// (MI355X_MICROARCH.md: "exact f32 (= fmaf chain, bitwise)" per accumulator chain).
//
//   y[16 beta + j] = sum_{q < QF} sum_{r < 16} h[j - r + 16 q] * x[16 (beta - q) + r]
//
// One MFMA covers 16 rows (8 blocks x {re, im}, row i = 2 b + c) x 16 phases x 4 k. The k index
// of a lane's A and B operand in step s of tap block q is r = 4 g + s (g = lane >> 4), so the
// four steps of a block read one aligned float4 of a sample row (A) and of a tap copy (B).
// K = 16 QF = 144 at 127 taps (QF = 9): 576 FLOP per output sample instead of 508, i.e. a
// ceiling of 157 TF / 576 = 273 GS/s = 55 % of the HBM roofline -- the price of exact fp32
// (the matrix cores' fp32 rate is the vector rate, 1/16 of fp16). C/D rows 4 g .. 4 g + 3 of
// a lane are (re, im) of blocks 2 g and 2 g + 1: the lane stores complex pairs directly.
//
// Access shape as k_fir_mfma12: one 2048-sample chunk per 256-thread workgroup (a wave per
// 512 outputs = 4 tiles of 8 blocks), chunk index remapped per XCD, the 16 (QF - 1)-sample
// halo re-read, nontemporal loads and stores. Samples go to LDS as raw fp32 re / im planes
// (rows of 16 samples at a 64-B pitch, im plane at 32 mod 256 B: conflict-free A reads,
// nsh_fir_f32_tile.hpp). Taps: the reversed taps R[m] = h[P - m]
// (P = 16 QF - 1) as 4 copies shifted by 0..3 floats (a lane's 4 taps of a block are one
// aligned float4 from copy m0 mod 4; copy pitch = 64 mod 256 B: conflict-free), prepared
// on the host and loaded per workgroup (L1/L2 hits).
// Non-finite inputs: the zero-padded K would turn inf x 0 into NaN where the direct form
// sums only real taps, so a chunk whose range holds inf/NaN is computed by the fp32 direct
// form from the same LDS planes (exact IEEE semantics), as in the split kernels.
#include "nsh_common.hpp"

#include <mutex>
#include <set>
#include <utility>
#include <vector>

#include "nsh_fir_f32_tile.hpp"
#include "nsh_fir_plan.hpp"

namespace {

using nsh_f32t::f32x4;
typedef float nf4 __attribute__((ext_vector_type(4)));
using nsh::AUX_NT;

template <int QF>
struct geomf32 : nsh_f32t::geom<QF - 1, QF> {
    using T = nsh_f32t::geom<QF - 1, QF>;
    static constexpr int NT = 256;
    static constexpr int HP = T::H / 2;                           // halo sample pairs
    static constexpr int BUF = 2 * T::PLANE;
    static constexpr int SLOTS = T::BYTES;                        // u32 max[4]
    static constexpr int LDS = SLOTS + 16;
    static_assert(HP <= NT && T::IMG_UNITS <= 2 * NT, "one halo pair / two image units per thread");
};

// wave-wide max, uniform: DPP within rows, readlane across them (as nsh_fir_mfma.hip)
__device__ __forceinline__ unsigned wave_max_u(unsigned v)
{
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));
    const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return max(max(a, b), max(c, d));
}
// largest |x| bit pattern of a float4 (a NaN gives bits >= 0x7f800000)
__device__ __forceinline__ unsigned max_mag4(const float4& v)
{
    const float m = __builtin_elementwise_maximum(__builtin_elementwise_maximum(__builtin_fabsf(v.x), __builtin_fabsf(v.y)),
                                                  __builtin_elementwise_maximum(__builtin_fabsf(v.z), __builtin_fabsf(v.w)));
    return __float_as_uint(m);
}

template <int QF>
__global__ __launch_bounds__(256) void k_fir_f32mfma(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist_in,
                                                     float2* __restrict__ hist_out,
                                                     float2* __restrict__ out,
                                                     const float4* __restrict__ timg, // [4][TWF] floats
                                                     const float* __restrict__ taps,
                                                     int L,
                                                     int64_t n_out,
                                                     int64_t per_x)
{
    using G = geomf32<QF>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned* slot = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out;
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t ch = (int64_t)(blockIdx.x & 7) * per_x + (blockIdx.x >> 3);
    if (ch >= nchunks) return; // whole workgroup, before any barrier

    // the chunk (lane: samples 2(tid + 256 u), +1), its halo, the tap image: all issued first
    float4 v[4];
    {
        const __amdgpu_buffer_rsrc_t r = nsh::chunk_rsrc<2048>(in, ch, n_in);
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = nsh::buf_load_f4(r, (tid + G::NT * u) * 16);
    }
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    {
        __amdgpu_buffer_rsrc_t hr;
        int off0, off1;
        if (ch > 0) {
            hr = nsh::chunk_rsrc<G::H>(in + ch * G::CHUNK - G::H, 0, G::H);
            off0 = 16 * tid;
            off1 = off0 + 8;
        } else {
            hr = nsh::chunk_rsrc<1 << 20>(hist_in, 0, hist_in ? L - 1 : 0);
            const int e = 2 * tid - G::H + (L - 1);
            off0 = e >= 0 ? 8 * e : 1 << 30; // past num_records: zeros
            off1 = e + 1 >= 0 ? 8 * (e + 1) : 1 << 30;
        }
        if (tid < G::HP) {
            const nsh::buf_f2 a = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off0, 0, 0));
            const nsh::buf_f2 b = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off1, 0, 0));
            hv = make_float4(a.x, a.y, b.x, b.y);
        }
    }
    float4 ti[2];
    nsh_f32t::load_taps<G>(timg, ti, tid, G::NT);

    // samples -> re / im planes (local sample s = halo first), the tap image -> its copies
    if (tid < G::HP) nsh_f32t::put<G>(lds, hv, 2 * tid);
#pragma unroll
    for (int u = 0; u < 4; ++u) nsh_f32t::put<G>(lds, v[u], G::H + 2 * (tid + G::NT * u));
    nsh_f32t::put_taps<G>(lds, ti, tid, G::NT);
    {
        unsigned m = max_mag4(hv);
#pragma unroll
        for (int u = 0; u < 4; ++u) m = max(m, max_mag4(v[u]));
        m = wave_max_u(m);
        if (lane == 0) slot[wave] = m;
    }
    nsh::lds_barrier();
    const bool exact = max(max(slot[0], slot[1]), max(slot[2], slot[3])) >= 0x7f800000u; // inf / NaN in range

    f32x4 acc[4];
    if (!exact) {
        nsh_f32t::tile<G, QF>(lds, wave, lane, acc);
    } else {
        // fp32 direct form (taps in order, fmaf) for the lane's 8 outputs, from the planes
        const int i = lane & 15, g = lane >> 4;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int n = G::H + 16 * (32 * wave + 8 * t + 2 * g + u) + i;
                float re = 0.f, im = 0.f;
                for (int k = 0; k < L; ++k) {
                    const int s = n - k;
                    const int off = (s >> 4) * G::PITCH + (s & 15) * 4;
                    re = fmaf(taps[k], *reinterpret_cast<const float*>(lds + off), re);
                    im = fmaf(taps[k], *reinterpret_cast<const float*>(lds + G::PLANE + off), im);
                }
                acc[t][2 * u] = re;
                acc[t][2 * u + 1] = im;
            }
    }
    nsh_f32t::store(nsh::chunk_rsrc<2048>(out, ch, n_out), acc, wave, lane);
    if (ch == 0) // the last L-1 inputs for the next call
        for (int j = tid; j < L - 1; j += G::NT) {
            const int64_t gi = n_in - (L - 1) + j;
            hist_out[j] = gi >= 0 ? in[gi] : (hist_in ? hist_in[gi + (L - 1)] : make_float2(0.f, 0.f));
        }
}

hipError_t set_lds_attr_f32(const void* fn, int bytes, int dev)
{
    static std::mutex m;
    static std::set<std::pair<const void*, int>> done;
    std::lock_guard<std::mutex> g(m);
    if (done.count({ fn, dev })) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert({ fn, dev });
    return e;
}

template <int QF>
int launch_f32(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geomf32<QF>;
    NSH_CK(set_lds_attr_f32((const void*)k_fir_f32mfma<QF>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per_x = (nchunks + 7) / 8;
    const int64_t grid = per_x * 8;
    if (grid > 0x7fffffff) return nsh::fail_msg("nsh_fir_ccf(mfma f32): stream too long for one launch");
    nsh::launch((k_fir_f32mfma<QF>), dim3((unsigned)grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const float4*)p->tf32_dev, (const float*)p->taps_dev, p->L, n_out, per_x);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma f32)");
    return 0;
}

} // namespace

int nsh_fir_f32_qf(int L) { return (L + 15 + 15) / 16; }

bool nsh_fir_f32_supported(const nsh_fir_plan* p)
{
    if (p->D != 1) return false;
    for (float t : p->taps_host)
        if (!(t == t) || t - t != 0.f) return false;
    const int qf = nsh_fir_f32_qf(p->L);
    return qf >= 1 && qf <= 17;
}

int nsh_fir_f32_prepare(nsh_fir_plan* p)
{
    const int QF = nsh_fir_f32_qf(p->L);
    const int TWF = 16 * QF + 16, P = 16 * QF - 1;
    std::vector<float> img((size_t)4 * TWF, 0.f);
    for (int d = 0; d < 4; ++d)
        for (int k = 0; k < TWF; ++k) {
            const int t = P - (k + d);
            img[(size_t)d * TWF + k] = (t >= 0 && t < p->L) ? p->taps_host[t] : 0.f;
        }
    p->QF = QF;
    NSH_CK(hipMalloc(&p->tf32_dev, img.size() * sizeof(float)));
    NSH_CK(hipMemcpy(p->tf32_dev, img.data(), img.size() * sizeof(float), hipMemcpyHostToDevice));
    p->kernel = "k_fir_f32mfma<" + std::to_string(QF) + ">";
    return 0;
}

int nsh_fir_f32_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                    int64_t n_out, hipStream_t s)
{
    switch (p->QF) {
    case 1: return launch_f32<1>(p, in, hist_in, hist_out, out, n_out, s);
    case 2: return launch_f32<2>(p, in, hist_in, hist_out, out, n_out, s);
    case 3: return launch_f32<3>(p, in, hist_in, hist_out, out, n_out, s);
    case 4: return launch_f32<4>(p, in, hist_in, hist_out, out, n_out, s);
    case 5: return launch_f32<5>(p, in, hist_in, hist_out, out, n_out, s);
    case 6: return launch_f32<6>(p, in, hist_in, hist_out, out, n_out, s);
    case 7: return launch_f32<7>(p, in, hist_in, hist_out, out, n_out, s);
    case 8: return launch_f32<8>(p, in, hist_in, hist_out, out, n_out, s);
    case 9: return launch_f32<9>(p, in, hist_in, hist_out, out, n_out, s);
    case 10: return launch_f32<10>(p, in, hist_in, hist_out, out, n_out, s);
    case 11: return launch_f32<11>(p, in, hist_in, hist_out, out, n_out, s);
    case 12: return launch_f32<12>(p, in, hist_in, hist_out, out, n_out, s);
    case 13: return launch_f32<13>(p, in, hist_in, hist_out, out, n_out, s);
    case 14: return launch_f32<14>(p, in, hist_in, hist_out, out, n_out, s);
    case 15: return launch_f32<15>(p, in, hist_in, hist_out, out, n_out, s);
    case 16: return launch_f32<16>(p, in, hist_in, hist_out, out, n_out, s);
    case 17: return launch_f32<17>(p, in, hist_in, hist_out, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma f32): unsupported tap count");
    }
}
