// Helpers of the FIR matrix-core kernels (nsh_fir_mfma.hip: k_fir_mfma12 for decim 1 and
// k_fir_mfma11 for decim 2 / 4). Device helpers only, in an anonymous namespace.
#pragma once
#include "nsh_common.hpp"
#include "nsh_fir_plan.hpp"

#include <mutex>
#include <set>
#include <utility>

namespace {


// CUs of the plan's device (queried once, at plan creation: a plan is read-only afterwards and
// may be shared by concurrent launches)
int plan_cus(const nsh_fir_plan* p) { return p->n_cu > 0 ? p->n_cu : 256; }

// The dynamic-LDS limit of a kernel, set once per (kernel, device): hipFuncSetAttribute acts on
// the current device, so a process-wide flag would leave a second device's launches unset.
hipError_t set_lds_attr(const void* fn, int bytes, int dev)
{
    static std::mutex m;
    static std::set<std::pair<const void*, int>> done;
    std::lock_guard<std::mutex> g(m);
    if (done.count({ fn, dev })) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert({ fn, dev });
    return e;
}

using nsh::AUX_NT;
using nsh::buf_load_f4;
using nsh::buf_store_f2;
using nsh::chunk_rsrc;
using nsh::u32x2;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef float nf2 __attribute__((ext_vector_type(2)));

constexpr int TILE = 512;   // outputs per wave per chunk
constexpr int QMAX = 6;     // L <= 161

__device__ __forceinline__ float2 virt(const float2* __restrict__ in, const float2* __restrict__ hist, int64_t g, int64_t n_in, int L)
{
    if (g >= 0) return g < n_in ? in[g] : make_float2(0.f, 0.f);
    if (g >= -(int64_t)(L - 1)) return hist ? hist[g + (L - 1)] : make_float2(0.f, 0.f); // null: zeros
    return make_float2(0.f, 0.f);
}



// ---- fp16x2: per-chunk scaled split, three products (default for decim 1) -------------------
// Same Toeplitz GEMM and LDS row layout as v2, on v_mfma_f32_32x32x16_f16.
// fp16 keeps 11 significant bits, so a two-term split x = x0 + x1 (both RNE) keeps 22 and
// three products x0h0 + x0h1 + x1h0 suffice (dropped x1h1 <= 2^-22 |xh|), where bf16 needs
// three terms and six products: half the matrix work, which is what bounds v2 (DESIGN.md
// section 4). fp16's narrow exponent range is handled by power-of-two scaling, which is
// exact:
//  * taps: scaled once on the host so max |h| * 2^sh lies in [2^14, 2^15);
//  * samples: per 2048-sample chunk, 2^s with s from the largest magnitude in the chunk and
//    in its predecessor (which holds the chunk's halo), so every scaled sample is < 2^15
//    (no fp16 overflow) and outputs are unscaled with one ldexp (exact unless subnormal).
// Per sample the split is then exact to 2^-22 relative, or 2^-39 of the chunk maximum for
// samples far below it (fp16 subnormal low term) -- below the fp32 direct form's own
// rounding error. A chunk holding a non-finite value, or a nonzero sample more than 2^28
// below the chunk maximum (its high term would be fp16-subnormal), is computed instead by
// the fp32 direct form inside the same kernel (exact fp32 semantics, including inf/NaN).
// The scale of chunk c+1 is agreed across the workgroup on the barrier of step c-1 (a wave
// maximum per slot in LDS); because the scale differs between chunks, the halo of chunk
// c+1 is re-split from the raw fp32 tail of chunk c kept in an LDS stash, not copied.
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef float f32x2 __attribute__((ext_vector_type(2)));
// fp16x2 split of the pair (a, b) * 2^sc: hi = RNE fp16 of each, lo = RNE fp16 of the exact
// residuals. As packed vectors: one v_cvt_pk_f16_f32 per plane, the residual as one packed
// subtract (the scalar form converted every value twice).
__device__ __forceinline__ void split_pair16(float a, float b, int sc, unsigned& hi, unsigned& lo)
{
    const f32x2 x = f32x2{ __builtin_ldexpf(a, sc), __builtin_ldexpf(b, sc) };
    const f16x2 h = __builtin_convertvector(x, f16x2);
    const f32x2 r = x - __builtin_convertvector(h, f32x2);
    hi = __builtin_bit_cast(unsigned, h);
    lo = __builtin_bit_cast(unsigned, __builtin_convertvector(r, f16x2));
}

template <int Q>
struct geom8 {
    static constexpr int NT = 256;
    static constexpr int CHUNK = 2048;
    static constexpr int S = 2 * Q;
    static constexpr int H = 32 * (Q - 1);
    static constexpr int HP = H / 2;                          // halo sample pairs
    static constexpr int NB = (CHUNK + H) / 32;
    static constexpr int PLANE = (NB * 80 + 255) / 256 * 256;
    static constexpr int BUF = 4 * PLANE;                     // re0 re1 im0 im1
    static constexpr int STASH = HP * 16;                     // raw fp32 tail of one chunk
    static constexpr int SLOTS = 2 * BUF + 2 * STASH;          // u32 max[2][4], flag[2][4]
    static constexpr int LDS = SLOTS + 64;                     // u32 [2][4] x 2 (v8: max, exact; v9: max, mnz)
    static constexpr int VPT = 4;
    static_assert(HP <= NT, "halo pairs: one per thread");
};

__device__ __forceinline__ unsigned mag(float x) { return __float_as_uint(x) & 0x7fffffffu; }
// largest magnitude as a bit pattern: NaN-propagating v_maximum3_f32 with |.| operand modifiers
// (a NaN anywhere gives a NaN, i.e. bits >= 0x7f800000, as the integer form did)
__device__ __forceinline__ float max_abs(float a, float b) { return __builtin_elementwise_maximum(__builtin_fabsf(a), __builtin_fabsf(b)); }
__device__ __forceinline__ float max_abs4(const float4& v) { return __builtin_elementwise_maximum(max_abs(v.x, v.y), max_abs(v.z, v.w)); }
__device__ __forceinline__ unsigned max_mag(const float4& v) { return __float_as_uint(max_abs4(v)); }
// scale exponent: max magnitude (bit pattern) * 2^s in [2^14, 2^15) (zero/subnormal: 2^141)
__device__ __forceinline__ int scale_of(unsigned maxbits) { return 141 - (int)(maxbits >> 23); }
// Wave-wide max / min, uniform result: DPP within each 16-lane row (quad_perm xor 1, xor 2,
// row_ror 4, 8: VALU, no LDS) then the four row results by v_readlane. The __shfl_xor form
// was six dependent ds_bpermute round trips through the LDS unit per reduction.
template <bool MAX>
__device__ __forceinline__ unsigned wave_red(unsigned v)
{
    constexpr int id = MAX ? 0 : -1;
    auto op = [](unsigned a, unsigned b) { return MAX ? max(a, b) : min(a, b); };
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(id, (int)v, 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(id, (int)v, 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(id, (int)v, 0x124, 0xf, 0xf, false)); // row_ror:4
    v = op(v, (unsigned)__builtin_amdgcn_update_dpp(id, (int)v, 0x128, 0xf, 0xf, false)); // row_ror:8
    const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return op(op(a, b), op(c, d));
}
__device__ __forceinline__ unsigned wave_max(unsigned v) { return wave_red<true>(v); }
__device__ __forceinline__ unsigned wave_min(unsigned v) { return wave_red<false>(v); }
// min over components of (magnitude bits - 1): zero maps to 0xffffffff, so the chunk minimum
// is (smallest nonzero magnitude - 1), or ~0u for an all-zero chunk
// smallest nonzero magnitude, coded as 2 |x|_bits - 1 (one v_lshl_add per value; zero -> ~0u)
__device__ __forceinline__ unsigned nz_code(float x) { return (__float_as_uint(x) << 1) - 1u; }
__device__ __forceinline__ unsigned min_nz1(const float4& v)
{
    return min(min(nz_code(v.x), nz_code(v.y)), min(nz_code(v.z), nz_code(v.w)));
}
// The exact-path rule over a whole chunk: non-finite iff its largest magnitude is; a nonzero sample
// scales below fp16's normal range iff its smallest nonzero one does (ldexp is exact, monotonic)
__device__ __forceinline__ bool chunk_needs_exact(unsigned maxbits, unsigned mnz1, int s)
{
    if (maxbits >= 0x7f800000u) return true;
    if (mnz1 == ~0u) return false; // all zero
    return __builtin_ldexpf(__uint_as_float((mnz1 >> 1) + 1u), s) < 6.103515625e-05f; // 2^-14
}

// chunk ch -> registers: lane t holds samples (2t, 2t+1) + 512 u, u < 4
__device__ __forceinline__ void load_chunk9(float4 (&v)[4], const float2* __restrict__ in, int64_t ch, int64_t n_in)
{
    const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(in, ch, n_in);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf_load_f4(r, (threadIdx.x + 256 * u) * 16);
}

__device__ __forceinline__ float2 f4_sample(const float4& v, int which)
{
    return which ? make_float2(v.z, v.w) : make_float2(v.x, v.y);
}

// The exact path on a raw fp32 chunk in LDS (local sample j at float2 index j, halo first):
// the lane's 8 outputs by the fp32 direct form (taps in order, fused multiply-add per component).
// The 8 outputs are two groups of four, 32 samples apart (blocks (reg & 3) + 8 (reg >> 2) + 4 h):
// an input sample j0 + q feeds output b of its group through tap k = 32 b - q, so each sample is
// read from LDS once per group (L + 96 reads instead of 4 L). q = 32 c - r runs downward, so every
// output still takes its taps in the order k = 0, 1, ..., L - 1 (bit-identical to one output at a
// time). (c, r, b) are unrolled, so every tap index k = 32 (b - c) + r is a compile-time constant:
// the tap loads are unconditional scalar loads the compiler batches ahead of use, and only taps of
// the last 32-block (k > 32 (Q - 2); Q = (L + 30) / 32 + 1 makes every earlier k < L) test k < L.
// re and im go through one v_pk_fma_f32.
// The same input reuse for NG outputs SP raw samples apart (output b at raw[j0 + SP b]): taps of
// index k > HMAX are zero (L - 1 <= HMAX), and every k <= KSAFE is below L.
template <int NG, int SP, int HMAX, int KSAFE>
__device__ __forceinline__ void direct_group(const nf2* raw, int j0, const float* __restrict__ taps, int L, nf2 (&acc)[NG])
{
#pragma unroll
    for (int b = 0; b < NG; ++b) acc[b] = nf2{ 0.f, 0.f };
#pragma unroll
    for (int i = 0; i <= SP * (NG - 1) + HMAX; ++i) {
        const int q = SP * (NG - 1) - i;
        const nf2 x = raw[j0 + q];
#pragma unroll
        for (int b = 0; b < NG; ++b) {
            const int k = SP * b - q;
            if (k < 0 || k > HMAX) continue;
            const float t = taps[k < L ? k : L - 1];
            if (k > KSAFE && k >= L) continue;
            acc[b] = __builtin_elementwise_fma(nf2{ t, t }, x, acc[b]);
        }
    }
}

template <int Q>
__device__ __forceinline__ void direct_tile9(const unsigned char* lds, const float* __restrict__ taps, int L, int wave, int h,
                                             int phase, nf2 (&o)[8])
{
    using G = geom8<Q>;
    const nf2* raw = reinterpret_cast<const nf2*>(lds);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const int j0 = G::H + wave * TILE + 32 * (8 * g + 4 * h) + phase;
        nf2 acc[4] = { nf2{ 0.f, 0.f }, nf2{ 0.f, 0.f }, nf2{ 0.f, 0.f }, nf2{ 0.f, 0.f } };
#pragma unroll
        for (int c = 3; c >= -(Q - 1); --c) {
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const int q = 32 * c - r;
                if (q < -G::H) break;  // L - 1 <= H: no tap reaches further back
                const nf2 x = raw[j0 + q];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int k = 32 * (b - c) + r;
                    if (k < 0 || k > G::H) continue;
                    const float t = taps[k < L ? k : L - 1];
                    if (k > 32 * (Q - 2) && k >= L) continue;
                    acc[b] = __builtin_elementwise_fma(nf2{ t, t }, x, acc[b]);
                }
            }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) o[4 * g + b] = acc[b];
    }
}

// ---- k_fir_mfma11: decimating polyphase FIR (D = 2, 4) on the fp16x2 split -----------------
// k_fir_mfma7's polyphase Toeplitz form (phase streams z_0[i] = x[D i], z_r[i] = x[D i + D - r],
// taps h'_0[j] = h[D j], h'_r[j] = h[D (j - 1) + r], 16-sample blocks, 16x16x32 + 16x16x16 tail)
// with k_fir_mfma9's numerics and pipeline: two fp16 planes per component and three products
// instead of three bf16 planes and six, per-chunk power-of-two scale, exact chunks staged raw
// in LDS and filtered by the fp32 direct form, buffer loads/stores, LDS-only barriers. The halo
// (the last D*H input samples of the previous chunk) is kept raw in an LDS stash and re-split
// at each chunk's scale.
#ifndef NSH_DECIM2_SHARED // A/B switch: D = 2 on the shared-input exact path (one pair at a time)
#define NSH_DECIM2_SHARED 0
#endif
#ifndef NSH_V13_CLOAD
// k_fir_mfma13: each chunk-load instruction reads 1 KiB contiguous (nontemporal), lane pairs exchange
// their samples by DPP before the split stores; 0 = a thread's D float4 side by side (each
// instruction spread over D KiB, default cache policy). D = 4, bit-identical: faster on three boxes
// of four (72.5 vs 70.1 %, r05ze; ~1 % in four two-library A/Bs each on two more, r05zzd), 1.3 %
// slower on one (r05zg)
#define NSH_V13_CLOAD 1
#endif
template <int D, int QH>
struct geom11 {
    static constexpr int NT = 256;
    static constexpr int CHUNK_IN = 2048;
    static constexpr int CHUNK = CHUNK_IN / D;
    static constexpr int TILES = 4 / D;
    static constexpr int WAVE_OUT = TILES * 128;
    static constexpr int KS = QH / 2;
    static constexpr int TAIL = QH % 2;
    static constexpr int H = 16 * (QH - 1);                    // halo samples per phase
    static constexpr int HR = QH - 1;
    static constexpr int NB = (CHUNK + H) / 16;
    static constexpr int PLANE = NB * 32;
    static constexpr int IM_OFF = (2 * PLANE + 255) / 256 * 256 + 128;
    // phase planes PH apart; k_fir_mfma13's split stores (NSH_V13_CLOAD) write all D phases in one
    // instruction, 32 / D pairs each per 32-lane group: PH = 32 * (4 / D) mod 128 B puts them on
    // disjoint banks
    static constexpr int PH = (IM_OFF + 2 * PLANE + 255) / 256 * 256 + (NSH_V13_CLOAD ? 128 / D : 0);
    static constexpr int BUF = (D * PH + 255) / 256 * 256;
    static constexpr int HP = D * H / 2;                      // halo float4 (2 input samples each)
    static constexpr int STASH = HP * 16;
    static constexpr int SLOTS = 2 * BUF + 2 * STASH;
    static constexpr int LDS = SLOTS + 64;                     // u32 max[2][4], mnz[2][4]
    static constexpr int UNITS = 4 / D;                        // units of 2D samples per thread
    static constexpr int PER_PHASE = 2 * KS * 64 * 8 + 2 * 64 * 4; // fp16 tap elements
    static_assert(D == 2 || D == 4, "D");
    static_assert((HP + 1024) * 16 <= BUF, "a raw fp32 chunk + halo fits one plane buffer");
    static_assert(HP <= NT && H / 2 <= NT, "halo: one float4 per thread");
};

template <class G>
__device__ __forceinline__ void store_pair_g(unsigned char* buf, int r, int s, float a_re, float b_re, float a_im,
                                             float b_im, int sc)
{
    unsigned char* ph = buf + r * G::PH;
    const int off = (s >> 4) * 32 + (s & 15) * 2;
    unsigned rh, rl, ih, il;
    split_pair16(a_re, b_re, sc, rh, rl);
    split_pair16(a_im, b_im, sc, ih, il);
    *reinterpret_cast<unsigned*>(ph + off) = rh;
    *reinterpret_cast<unsigned*>(ph + G::PLANE + off) = rl;
    *reinterpret_cast<unsigned*>(ph + G::IM_OFF + off) = ih;
    *reinterpret_cast<unsigned*>(ph + G::IM_OFF + G::PLANE + off) = il;
}
// o = s * 2^u per (re, im) pair: one packed multiply when 2^u is a normal float (it rounds as
// ldexp does), else ldexp
template <int M>
__device__ __forceinline__ void unscale_tile(const nf2 (&s)[M], int u, nf2 (&o)[M])
{
    if (u >= -126 && u <= 127) {
        const float f = __builtin_bit_cast(float, (u + 127) << 23);
#pragma unroll
        for (int i = 0; i < M; ++i) o[i] = s[i] * f;
    } else {
#pragma unroll
        for (int i = 0; i < M; ++i) o[i] = nf2{ __builtin_ldexpf(s[i].x, u), __builtin_ldexpf(s[i].y, u) };
    }
}
template <int D, int QH>
__device__ __forceinline__ void store_pair11(unsigned char* buf, int r, int s, float a_re, float b_re, float a_im,
                                             float b_im, int sc)
{
    store_pair_g<geom11<D, QH>>(buf, r, s, a_re, b_re, a_im, b_im, sc);
}


int decim_qh(const nsh_fir_plan* p) { return ((p->L + p->D - 1) / p->D + 1 + 15 + 15) / 16; }
bool finite_taps(const nsh_fir_plan* p)
{
    for (float t : p->taps_host)
        if (!(t == t) || t - t != 0.f) return false;
    return true;
}

} // namespace
