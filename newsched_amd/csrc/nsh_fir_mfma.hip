// libnsh_hip.so: fir_filter_ccf as a Toeplitz GEMM on the bf16 matrix cores (decim 1).
//
// Blocked form. Split the output stream into 32-sample blocks; output n = 32*beta + i:
//     y[32 beta + i] = sum_{q<Q} sum_{r<32} h[i - r + 32 q] * x[32 (beta - q) + r]
// i.e. C[rho][i] = sum_k A[rho][k] B[k][i] with k = 32 q + r (K = 32 Q),
//     A[rho][k] = x_c[32 (beta - q) + r]    rho = (block beta, component c)  -- the stream
//     B[k][i]   = h[i - r + 32 q]           (zero outside [0, L))           -- the taps
// One v_mfma_f32_32x32x16_bf16 covers 32 rows (16 blocks x {re, im}) x 32 phases x 16 k;
// a wave owns a 512-sample tile and runs 2Q k-steps. Q = 5 for L = 127 (K = 160: 26 %
// zero padding). Cost: 3840 bf16 FLOP per output sample, i.e. 51 us of dense MFMA issue
// per 2^25 samples at 2.4 GHz (60 us at the 2.05 GHz the chip holds under this load), against
// 91 us for the HBM stream at the measured copy rate: the matrix cores are not free here,
// and overlapping them with the stream is what the v2 pipeline below is about.
//
// Precision: fp32 emulated by a 3-term bf16 split of both operands (x = x1 + x2 + x3 and
// h = h1 + h2 + h3, each split exact for finite normal fp32) and the six products with
// term-order sum <= 4 (x1h1 | x1h2 x2h1 x1h3 x2h2 x3h1), accumulated in fp32 by the MFMA;
// the leading product and the correction terms use separate accumulators. Dropped terms
// are < 2^-24 relative; measured error is at the fp32 direct-form level (tests/).
// bf16 keeps the fp32 exponent range, so no input scaling is needed. Non-finite inputs
// are not supported by this form (use NSH_FIR_DIRECT).
//
// Data movement (v2, the NSH_FIR_MFMA kernel; the 16-sample form v5 and the decimating
// form v7 follow below): a 256-thread workgroup
// (2 per CU) walks a contiguous range of 2048-output chunks. Each chunk's 2048 samples are
// loaded with 16-byte nontemporal global loads into registers two chunks ahead, split, and
// written as six bf16 planes (re/im x 3 terms) to one of two LDS buffers while the MFMAs
// read the other; the 32(Q-1)-sample halo is the previous chunk's tail, copied LDS -> LDS.
// Every 32-sample row is padded to
// 80 B so the per-lane ds_read_b128 A-fragment reads are bank-conflict free (lanes of one
// 16-lane group read 16 distinct 16-B slots: 5*beta mod 16 is a bijection). The taps'
// B fragments (3 terms x 2Q k-steps, prepared on the host in lane order) stay in VGPRs for
// the whole launch. Outputs leave the accumulators as (re, im) float2 pairs: lanes 0-31
// of a store cover 32 consecutive samples (256 contiguous bytes).
#include "nsh_common.hpp"

#include <algorithm>
#include <mutex>
#include <set>
#include <utility>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nsh_fir_plan.hpp"

// Ablation hooks for tools/probe/fir_ablate.sh only (bit mask; 0 in every product build):
// 1 = no MFMA, 2 = no global loads, 4 = no bf16 split, 8 = no global stores; timing-only
// (wrong results): 16 = half the MFMAs, 32 = int8 MFMA instruction count, 64 = the same
// FLOPs as 16x16x32 MFMAs, 128 = A fragments read once and reused.
#ifndef NSH_FIR_ABLATE
#define NSH_FIR_ABLATE 0
#endif

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



template <int Q, int NW, int PLANE_>
__device__ __forceinline__ void compute_tile(const unsigned char* lds,
                                             const bf16x8 (&B0)[2 * Q],
                                             const bf16x8 (&B1)[2 * Q],
                                             const bf16x8 (&B2)[2 * Q],
                                             int a_base,
                                             int64_t n_tile,
                                             int h,
                                             int phase,
                                             int64_t n_out,
                                             float2* __restrict__ out)
{
    constexpr int S_ = 2 * Q;
    f32x16 acc_hi = {};
    f32x16 acc_lo = {};
#if NSH_FIR_ABLATE & 128 // timing only: A fragments read for q = 0 and reused for every q
    bf16x8 Ar[2][3];
#endif
#pragma unroll
    for (int st = 0; st < S_; ++st) {
        const int q = st >> 1;
        const int off = a_base - q * 80 + 32 * (st & 1);
#if NSH_FIR_ABLATE & 128
        if (q == 0) {
            Ar[st & 1][0] = *reinterpret_cast<const bf16x8*>(lds + off);
            Ar[st & 1][1] = *reinterpret_cast<const bf16x8*>(lds + off + PLANE_);
            Ar[st & 1][2] = *reinterpret_cast<const bf16x8*>(lds + off + 2 * PLANE_);
        }
        const bf16x8 A0 = Ar[st & 1][0], A1 = Ar[st & 1][1], A2 = Ar[st & 1][2];
#else
        const bf16x8 A0 = *reinterpret_cast<const bf16x8*>(lds + off);
        const bf16x8 A1 = *reinterpret_cast<const bf16x8*>(lds + off + PLANE_);
        const bf16x8 A2 = *reinterpret_cast<const bf16x8*>(lds + off + 2 * PLANE_);
#endif
#if NSH_FIR_ABLATE & 1
        acc_hi[st & 15] += (float)A0[0] + (float)A1[1] + (float)A2[2] + (float)B0[st][0] + (float)B1[st][1] + (float)B2[st][2];
        continue;
#endif
#if NSH_FIR_ABLATE & 16 // timing only: half the matrix work
        acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0[st], acc_hi, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2, B2[st], acc_lo, 0, 0, 0);
        continue;
#endif
#if NSH_FIR_ABLATE & 64 // timing only: the same FLOPs as 2 x v_mfma_f32_16x16x32_bf16 per product
        {
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
            f32x4 c0 = { acc_hi[0], acc_hi[1], acc_hi[2], acc_hi[3] }, c1 = { acc_lo[0], acc_lo[1], acc_lo[2], acc_lo[3] };
#pragma unroll
            for (int rep = 0; rep < 2; ++rep) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B0[st], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B1[st], c1, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B0[st], c1, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B2[st], c1, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B1[st], c1, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2, B0[st], c1, 0, 0, 0);
            }
            for (int t = 0; t < 4; ++t) {
                acc_hi[t] = c0[t];
                acc_lo[t] = c1[t];
            }
        }
        continue;
#endif
#if NSH_FIR_ABLATE & 32 // timing only: the int8 instruction count (6 x i32_32x32x32_i8 per 2 k-steps)
        if (st & 1) {
            typedef int i32x4 __attribute__((ext_vector_type(4)));
            typedef int i32x16 __attribute__((ext_vector_type(16)));
            const i32x4 a0 = __builtin_bit_cast(i32x4, A0), a1 = __builtin_bit_cast(i32x4, A1), a2 = __builtin_bit_cast(i32x4, A2);
            const i32x4 b0 = __builtin_bit_cast(i32x4, B0[st]), b1 = __builtin_bit_cast(i32x4, B1[st]), b2 = __builtin_bit_cast(i32x4, B2[st]);
            i32x16 ih = __builtin_bit_cast(i32x16, acc_hi), il = __builtin_bit_cast(i32x16, acc_lo);
            ih = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, ih, 0, 0, 0);
            il = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, il, 0, 0, 0);
            il = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, il, 0, 0, 0);
            ih = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b2, ih, 0, 0, 0);
            il = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, il, 0, 0, 0);
            ih = __builtin_amdgcn_mfma_i32_32x32x32_i8(a2, b0, ih, 0, 0, 0);
            acc_hi = __builtin_bit_cast(f32x16, ih);
            acc_lo = __builtin_bit_cast(f32x16, il);
        }
        continue;
#endif
        acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0[st], acc_hi, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B2[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2, B0[st], acc_lo, 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 8; ++reg) {
        const int blk = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int64_t n = n_tile + 32 * blk + phase;
        const float re = acc_hi[reg] + acc_lo[reg];
        const float im = acc_hi[reg + 8] + acc_lo[reg + 8];
#if NSH_FIR_ABLATE & 8
        if (re == 1.2345e-30f && n < n_out) {
#else
        if (n < n_out) {
#endif
            nf2 o = { re, im };
            __builtin_nontemporal_store(o, reinterpret_cast<nf2*>(out + n));
        }
    }
}

// ---- v2: software-pipelined form --------------------------------------------------------
// * split by truncation: x1 = x & 0xffff0000, x2 = (x - x1) & 0xffff0000, x3 = x - x1 - x2;
//   both subtractions are exact and x3 has <= 8 significant bits, so x = x1 + x2 + x3 holds
//   exactly (as for the rounding split); bf16 pairs are packed with one v_perm_b32.
// * two LDS plane buffers: chunk c+1 is split into buffer (i+1)&1 in the same basic block
//   as chunk c's MFMAs from buffer i&1, so the VALU split co-issues with the matrix pipe;
//   one barrier per chunk.
// * the 32(Q-1)-sample halo of chunk c+1 is the tail of chunk c: copied LDS -> LDS, so
//   HBM reads each input sample once (only a workgroup's first chunk loads its halo).
template <int Q>
struct geom2 {
    static constexpr int NT = 256;
    static constexpr int CHUNK = 2048;
    static constexpr int S = 2 * Q;
    static constexpr int H = 32 * (Q - 1);
    static constexpr int HR = Q - 1;                          // halo rows (32 samples each)
    static constexpr int NB = (CHUNK + H) / 32;               // rows per buffer
    static constexpr int PLANE = (NB * 80 + 255) / 256 * 256;
    static constexpr int BUF = 6 * PLANE;
    static constexpr int LDS = 2 * BUF;
    static constexpr int VPT = CHUNK / 2 / NT;                // 4 float4 per thread (main part)
};

__device__ __forceinline__ unsigned hi16pair(float a, float b)
{
    // upper halves of a (low 16 bits of result) and b (high 16 bits): one v_perm_b32
    return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
__device__ __forceinline__ float trunc_bf(float x) { return __uint_as_float(__float_as_uint(x) & 0xffff0000u); }

// Split two consecutive samples (a, b) of one component into three packed bf16 pairs.
__device__ __forceinline__ void split_pair(float a, float b, unsigned& p1, unsigned& p2, unsigned& p3)
{
    const float a1 = trunc_bf(a), b1 = trunc_bf(b);
    const float ar = a - a1, br = b - b1;
    const float a2 = trunc_bf(ar), b2 = trunc_bf(br);
    const float a3 = ar - a2, b3 = br - b2;
    p1 = hi16pair(a1, b1);
    p2 = hi16pair(a2, b2);
    p3 = hi16pair(a3, b3);
}

// Global -> registers: the 2048 non-halo samples of chunk ch (local samples H .. H+2047).
template <int Q>
__device__ __forceinline__ void load_main(float4 (&v)[geom2<Q>::VPT], const float2* __restrict__ in,
                                          const float2* __restrict__ hist, int64_t ch, int64_t n_in, int L,
                                          bool in_aligned)
{
    using G = geom2<Q>;
    const int64_t g0 = ch * G::CHUNK;
#if NSH_FIR_ABLATE & 2
    for (int u = 0; u < G::VPT; ++u) v[u] = make_float4((float)g0, (float)u, (float)threadIdx.x, 1.f);
    return;
#endif
    if (in_aligned && g0 + G::CHUNK <= n_in) {
        const nf4* src = reinterpret_cast<const nf4*>(in + g0);
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const nf4 t = __builtin_nontemporal_load(src + threadIdx.x + G::NT * u);
            v[u] = make_float4(t.x, t.y, t.z, t.w);
        }
    } else {
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const int vi = threadIdx.x + G::NT * u;
            const float2 a = virt(in, hist, g0 + 2 * vi, n_in, L);
            const float2 b = virt(in, hist, g0 + 2 * vi + 1, n_in, L);
            v[u] = make_float4(a.x, a.y, b.x, b.y);
        }
    }
}

// Registers -> six bf16 planes of one buffer (rows HR.. of the buffer).
template <int Q>
__device__ __forceinline__ void store_main(const float4 (&v)[geom2<Q>::VPT], unsigned char* buf)
{
    using G = geom2<Q>;
#pragma unroll
    for (int u = 0; u < G::VPT; ++u) {
        const int s = G::H + 2 * (threadIdx.x + G::NT * u); // even local sample
        const int off = (s >> 5) * 80 + (s & 31) * 2;
        unsigned r1, r2, r3, i1, i2, i3;
#if NSH_FIR_ABLATE & 4
        r1 = r2 = r3 = __float_as_uint(v[u].x);
        i1 = i2 = i3 = __float_as_uint(v[u].y);
#else
        split_pair(v[u].x, v[u].z, r1, r2, r3);
        split_pair(v[u].y, v[u].w, i1, i2, i3);
#endif
        *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = r1;
        *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = r2;
        *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = r3;
        *reinterpret_cast<unsigned*>(buf + 3 * G::PLANE + off) = i1;
        *reinterpret_cast<unsigned*>(buf + 4 * G::PLANE + off) = i2;
        *reinterpret_cast<unsigned*>(buf + 5 * G::PLANE + off) = i3;
    }
}

// Halo rows of the next buffer = last HR rows of the current one (6 planes x HR x 64 B).
template <int Q>
__device__ __forceinline__ void copy_halo(const unsigned char* cur, unsigned char* nxt)
{
    using G = geom2<Q>;
    constexpr int PIECES = 6 * G::HR * 4; // 16-B pieces (64 data bytes per row)
    if constexpr (PIECES > 0) {
        for (int t = threadIdx.x; t < PIECES; t += G::NT) {
            const int plane = t / (G::HR * 4);
            const int rem = t % (G::HR * 4);
            const int row = rem >> 2, q16 = rem & 3;
            const uint4 d = *reinterpret_cast<const uint4*>(cur + plane * G::PLANE + (G::NB - G::HR + row) * 80 + q16 * 16);
            *reinterpret_cast<uint4*>(nxt + plane * G::PLANE + row * 80 + q16 * 16) = d;
        }
    }
}

// First chunk of a workgroup: its halo comes from global memory / history.
template <int Q>
__device__ __forceinline__ void load_store_halo(unsigned char* buf, const float2* __restrict__ in,
                                                const float2* __restrict__ hist, int64_t ch, int64_t n_in, int L)
{
    using G = geom2<Q>;
    if constexpr (G::H > 0) {
        const int64_t g0 = ch * G::CHUNK - G::H;
        for (int p = threadIdx.x; p < G::H / 2; p += G::NT) {
            const float2 a = virt(in, hist, g0 + 2 * p, n_in, L);
            const float2 b = virt(in, hist, g0 + 2 * p + 1, n_in, L);
            const int s = 2 * p;
            const int off = (s >> 5) * 80 + (s & 31) * 2;
            unsigned r1, r2, r3, i1, i2, i3;
            split_pair(a.x, b.x, r1, r2, r3);
            split_pair(a.y, b.y, i1, i2, i3);
            *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = r1;
            *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = r2;
            *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = r3;
            *reinterpret_cast<unsigned*>(buf + 3 * G::PLANE + off) = i1;
            *reinterpret_cast<unsigned*>(buf + 4 * G::PLANE + off) = i2;
            *reinterpret_cast<unsigned*>(buf + 5 * G::PLANE + off) = i3;
        }
    }
}

template <int Q, int DEPTH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma2(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist_in,
                                                     float2* __restrict__ hist_out,
                                                     float2* __restrict__ out,
                                                     const bf16x8* __restrict__ frag, // [3][S][64]
                                                     int L,
                                                     int64_t n_out,
                                                     int in_aligned)
{
    using G = geom2<Q>;
    constexpr int S = G::S;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    bf16x8 B0[S], B1[S], B2[S];
#pragma unroll
    for (int st = 0; st < S; ++st) {
        B0[st] = frag[(0 * S + st) * 64 + lane];
        B1[st] = frag[(1 * S + st) * 64 + lane];
        B2[st] = frag[(2 * S + st) * 64 + lane];
    }

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;

    const int rho = lane & 31;
    const int b = rho & 15;
    const int c = rho >> 4;
    const int h = lane >> 5;
    const int a_base = c * 3 * G::PLANE + ((Q - 1) + 16 * wave + b) * 80 + 16 * h;
    const int phase = lane & 31;
    const bool al = in_aligned != 0;

    auto clamp = [&](int64_t x) { return x <= c_last ? x : c_last; };
    // prologue: chunk c_begin -> buffer 0 (halo from global); chunks up to c_begin+DEPTH in flight
    float4 va[G::VPT], vb[G::VPT], vc[G::VPT];
    load_store_halo<Q>(lds, in, hist_in, c_begin, n_in, L);
    load_main<Q>(va, in, hist_in, c_begin, n_in, L, al);
    store_main<Q>(va, lds);
    load_main<Q>(va, in, hist_in, clamp(c_begin + 1), n_in, L, al);
    if constexpr (DEPTH > 1) load_main<Q>(vb, in, hist_in, clamp(c_begin + 2), n_in, L, al);
    __syncthreads();

    // step ch: `nxt` holds chunk ch+1 (split into the other buffer now), `ld` receives
    // chunk ch+1+DEPTH (clamped: the tail re-reads its last chunk from L2).
    auto step = [&](float4 (&nxt)[G::VPT], float4 (&ld)[G::VPT], int64_t ch) {
        unsigned char* cur = lds + ((ch - c_begin) & 1) * G::BUF;
        unsigned char* nbuf = lds + (((ch - c_begin) & 1) ^ 1) * G::BUF;
        load_main<Q>(ld, in, hist_in, clamp(ch + 1 + DEPTH), n_in, L, al);
        copy_halo<Q>(cur, nbuf);
        store_main<Q>(nxt, nbuf); // split chunk ch+1 while chunk ch runs on the matrix cores
        compute_tile<Q, 4, G::PLANE>(cur, B0, B1, B2, a_base, ch * G::CHUNK + (int64_t)wave * TILE, h, phase, n_out, out);
        __syncthreads();
    };
    int64_t ch = c_begin;
    if constexpr (DEPTH == 1) {
        for (; ch + 1 <= c_last; ch += 2) {
            step(va, vb, ch);
            step(vb, va, ch + 1);
        }
        if (ch <= c_last) step(va, vb, ch);
    } else {
        for (; ch + 2 <= c_last; ch += 3) {
            step(va, vc, ch);
            step(vb, va, ch + 1);
            step(vc, vb, ch + 2);
        }
        if (ch <= c_last) step(va, vc, ch++);
        if (ch <= c_last) step(vb, va, ch);
    }
}

// ---- v5: 16-phase blocks on v_mfma_f32_16x16x32_bf16 -------------------------------------
// Same Toeplitz GEMM with 16-sample blocks: y[16b + i] = sum_q sum_{r<16} h[i - r + 16q] x[16(b-q) + r],
// q < QH = ceil((L + 15) / 16) (9 for L = 127), K = 16 QH padded to the 32 of one k-step.
// Under this kernel's power-limited clock the 16x16x32 form issues the same FLOPs faster
// (ablation mask 64: -5 % min, -10 % median vs 32x32x16), the tap fragments need half the
// VGPRs (3 x KS x 4) and the LDS rows need no padding:
//   * rows of 16 samples = 32 B per bf16 plane, packed; A-fragment row rho = l & 15 is
//     (component c = rho & 1, block b = rho >> 1), k-group g = l >> 4 reads 16 B of row
//     (b - q), q = 2s + (g >> 1); with the im planes at an offset = 128 mod 256 B every
//     16-lane ds_read_b128 group covers 16 distinct 16-B slots (searched exhaustively);
//   * C row 4g + reg = (c = reg & 1, b = 2g + (reg >> 1)): re and im of a block land in
//     the same lane (regs 0/1 and 2/3), stored as float2 without lane exchanges.
// A wave owns 512 outputs = 4 row-tiles of 8 blocks; tap fragments are shared by the tiles.
template <int QH>
struct geom5 {
    static constexpr int NT = 256;
    static constexpr int CHUNK = 2048;
    static constexpr int KS = QH / 2;                          // full k-steps of 32 (16x16x32)
    static constexpr int TAIL = QH % 2;                        // one k-step of 16 (16x16x16)
    static constexpr int H = 16 * (QH - 1);                    // halo samples
    static constexpr int HR = QH - 1;                          // halo rows
    static constexpr int NB = (CHUNK + H) / 16;                // rows per buffer
    static constexpr int PLANE = NB * 32;
    static constexpr int IM_OFF = (3 * PLANE + 255) / 256 * 256 + 128;
    static constexpr int BUF = (IM_OFF + 3 * PLANE + 255) / 256 * 256;
    static constexpr int LDS = 2 * BUF;
    static constexpr int VPT = CHUNK / 2 / NT;                 // 4 float4 per thread
    static constexpr int TILES = 4;                            // row-tiles per wave
};

template <int QH>
__device__ __forceinline__ void v5_store_pair(unsigned char* buf, int s, float a_re, float b_re, float a_im,
                                              float b_im)
{
    using G = geom5<QH>;
    const int off = (s >> 4) * 32 + (s & 15) * 2;
    unsigned r1, r2, r3, i1, i2, i3;
#if NSH_FIR_ABLATE & 4
    r1 = r2 = r3 = __float_as_uint(a_re);
    i1 = i2 = i3 = __float_as_uint(a_im);
#else
    split_pair(a_re, b_re, r1, r2, r3);
    split_pair(a_im, b_im, i1, i2, i3);
#endif
    *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = r1;
    *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = r2;
    *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = r3;
    *reinterpret_cast<unsigned*>(buf + G::IM_OFF + 0 * G::PLANE + off) = i1;
    *reinterpret_cast<unsigned*>(buf + G::IM_OFF + 1 * G::PLANE + off) = i2;
    *reinterpret_cast<unsigned*>(buf + G::IM_OFF + 2 * G::PLANE + off) = i3;
}

template <int QH>
__device__ __forceinline__ void v5_load_main(float4 (&v)[geom5<QH>::VPT], const float2* __restrict__ in,
                                             const float2* __restrict__ hist, int64_t ch, int64_t n_in, int L,
                                             bool in_aligned)
{
    using G = geom5<QH>;
    const int64_t g0 = ch * G::CHUNK;
#if NSH_FIR_ABLATE & 2
    for (int u = 0; u < G::VPT; ++u) v[u] = make_float4((float)g0, (float)u, (float)threadIdx.x, 1.f);
    return;
#endif
    if (in_aligned && g0 + G::CHUNK <= n_in) {
        const nf4* src = reinterpret_cast<const nf4*>(in + g0);
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const nf4 t = __builtin_nontemporal_load(src + threadIdx.x + G::NT * u);
            v[u] = make_float4(t.x, t.y, t.z, t.w);
        }
    } else {
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const int vi = threadIdx.x + G::NT * u;
            const float2 a = virt(in, hist, g0 + 2 * vi, n_in, L);
            const float2 b = virt(in, hist, g0 + 2 * vi + 1, n_in, L);
            v[u] = make_float4(a.x, a.y, b.x, b.y);
        }
    }
}

template <int QH>
__device__ __forceinline__ void v5_store_main(const float4 (&v)[geom5<QH>::VPT], unsigned char* buf)
{
    using G = geom5<QH>;
#pragma unroll
    for (int u = 0; u < G::VPT; ++u)
        v5_store_pair<QH>(buf, G::H + 2 * (threadIdx.x + G::NT * u), v[u].x, v[u].z, v[u].y, v[u].w);
}

template <int QH>
__device__ __forceinline__ void v5_copy_halo(const unsigned char* cur, unsigned char* nxt)
{
    using G = geom5<QH>;
    constexpr int PIECES = 6 * G::HR * 2; // 16-B pieces (32 B per row)
    if constexpr (PIECES > 0) {
        for (int t = threadIdx.x; t < PIECES; t += G::NT) {
            const int plane = t / (G::HR * 2);
            const int rem = t % (G::HR * 2);
            const int pbase = (plane < 3 ? 0 : G::IM_OFF) + (plane % 3) * G::PLANE;
            const uint4 d = *reinterpret_cast<const uint4*>(cur + pbase + (G::NB - G::HR) * 32 + rem * 16);
            *reinterpret_cast<uint4*>(nxt + pbase + rem * 16) = d;
        }
    }
}

template <int QH>
__device__ __forceinline__ void v5_load_store_halo(unsigned char* buf, const float2* __restrict__ in,
                                                   const float2* __restrict__ hist, int64_t ch, int64_t n_in, int L)
{
    using G = geom5<QH>;
    if constexpr (G::H > 0) {
        const int64_t g0 = ch * G::CHUNK - G::H;
        for (int p = threadIdx.x; p < G::H / 2; p += G::NT) {
            const float2 a = virt(in, hist, g0 + 2 * p, n_in, L);
            const float2 b = virt(in, hist, g0 + 2 * p + 1, n_in, L);
            v5_store_pair<QH>(buf, 2 * p, a.x, b.x, a.y, b.y);
        }
    }
}

// The wave's 4 row-tiles x (KS k-steps of 32 + an optional tail of 16).
template <int QH>
__device__ __forceinline__ void v5_compute(const unsigned char* lds, const bf16x8 (&B0)[geom5<QH>::KS + 1],
                                           const bf16x8 (&B1)[geom5<QH>::KS + 1], const bf16x8 (&B2)[geom5<QH>::KS + 1],
                                           const bf16x4 (&T)[3], int64_t n_tile, int64_t n_out,
                                           float2* __restrict__ out)
{
    using G = geom5<QH>;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int rho = lane & 15;
    const int c = rho & 1, b = rho >> 1;
    const int g = lane >> 4;
    const int phase = lane & 15;
    const int row_base = c * G::IM_OFF + (G::HR + wave * 32 + b) * 32; // this lane's block row, q = 0
    f32x4 hi[G::TILES], lo[G::TILES];
#pragma unroll
    for (int t = 0; t < G::TILES; ++t) {
        hi[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        lo[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
    }
#pragma unroll
    for (int st = 0; st < G::KS; ++st) {
        const int q = 2 * st + (g >> 1);
#pragma unroll
        for (int t = 0; t < G::TILES; ++t) {
            const int off = row_base + t * 8 * 32 - q * 32 + (g & 1) * 16;
            const bf16x8 A0 = *reinterpret_cast<const bf16x8*>(lds + off);
            const bf16x8 A1 = *reinterpret_cast<const bf16x8*>(lds + off + G::PLANE);
            const bf16x8 A2 = *reinterpret_cast<const bf16x8*>(lds + off + 2 * G::PLANE);
#if NSH_FIR_ABLATE & 1
            hi[t][0] += (float)A0[0] + (float)A1[1] + (float)A2[2] + (float)B0[st][0] + (float)B1[st][1] + (float)B2[st][2];
            continue;
#endif
            hi[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B0[st], hi[t], 0, 0, 0);
            lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B1[st], lo[t], 0, 0, 0);
            lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B0[st], lo[t], 0, 0, 0);
            lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B2[st], lo[t], 0, 0, 0);
            lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B1[st], lo[t], 0, 0, 0);
            lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2, B0[st], lo[t], 0, 0, 0);
        }
    }
    // The K tail accumulates into its own registers: an accumulator handed directly from a
    // 16x16x32 MFMA to a dependent 16x16x16 one is read before its upper rows are written
    // when nothing is scheduled in between (measured: regs 2-3 stale, ~1e-6 errors), so the
    // two opcodes never share an accumulation chain.
    f32x4 hi_t[G::TILES], lo_t[G::TILES];
#pragma unroll
    for (int t = 0; t < G::TILES; ++t) {
        hi_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        lo_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
    }
    if constexpr (G::TAIL) {
        // q = QH - 1 alone: v_mfma_f32_16x16x16_bf16, lane l holds A[l & 15][k = 4(l >> 4) + j]
#pragma unroll
        for (int t = 0; t < G::TILES; ++t) {
            const int off = row_base + t * 8 * 32 - (QH - 1) * 32 + g * 8;
            const bf16x4 A0 = *reinterpret_cast<const bf16x4*>(lds + off);
            const bf16x4 A1 = *reinterpret_cast<const bf16x4*>(lds + off + G::PLANE);
            const bf16x4 A2 = *reinterpret_cast<const bf16x4*>(lds + off + 2 * G::PLANE);
#if NSH_FIR_ABLATE & 1
            hi[t][1] += (float)A0[0] + (float)A1[1] + (float)A2[2] + (float)T[0][0] + (float)T[1][1] + (float)T[2][2];
            continue;
#endif
            hi_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[0], hi_t[t], 0, 0, 0);
            lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[1], lo_t[t], 0, 0, 0);
            lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A1, T[0], lo_t[t], 0, 0, 0);
            lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[2], lo_t[t], 0, 0, 0);
            lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A1, T[1], lo_t[t], 0, 0, 0);
            lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A2, T[0], lo_t[t], 0, 0, 0);
        }
    }
#pragma unroll
    for (int t = 0; t < G::TILES; ++t) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int blk = t * 8 + 2 * g + half;
            const int64_t n = n_tile + (int64_t)wave * TILE + blk * 16 + phase;
            const float re = (hi[t][2 * half] + hi_t[t][2 * half]) + (lo[t][2 * half] + lo_t[t][2 * half]);
            const float im = (hi[t][2 * half + 1] + hi_t[t][2 * half + 1]) + (lo[t][2 * half + 1] + lo_t[t][2 * half + 1]);
#if NSH_FIR_ABLATE & 8
            if (re == 1.2345e-30f && n < n_out) {
#else
            if (n < n_out) {
#endif
                nf2 o = { re, im };
                __builtin_nontemporal_store(o, reinterpret_cast<nf2*>(out + n));
            }
        }
    }
}

template <int QH, int DEPTH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma5(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist_in,
                                                     float2* __restrict__ hist_out,
                                                     float2* __restrict__ out,
                                                     const bf16x8* __restrict__ frag, // [3][KS][64] + tail [3][64] x4
                                                     int L,
                                                     int64_t n_out,
                                                     int in_aligned)
{
    using G = geom5<QH>;
    constexpr int KS = G::KS;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int64_t n_in = n_out;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    bf16x8 B0[KS + 1], B1[KS + 1], B2[KS + 1]; // +1: keeps the arrays non-empty for QH = 1
#pragma unroll
    for (int st = 0; st < KS; ++st) {
        B0[st] = frag[(0 * KS + st) * 64 + lane];
        B1[st] = frag[(1 * KS + st) * 64 + lane];
        B2[st] = frag[(2 * KS + st) * 64 + lane];
    }
    bf16x4 T[3] = {};
    if constexpr (G::TAIL) {
        const bf16x4* tf = reinterpret_cast<const bf16x4*>(frag + 3 * KS * 64);
#pragma unroll
        for (int k = 0; k < 3; ++k) T[k] = tf[k * 64 + lane];
    }

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;
    const bool al = in_aligned != 0;
    auto clamp = [&](int64_t x) { return x <= c_last ? x : c_last; };

    float4 va[G::VPT], vb[G::VPT], vc[G::VPT];
    v5_load_store_halo<QH>(lds, in, hist_in, c_begin, n_in, L);
    v5_load_main<QH>(va, in, hist_in, c_begin, n_in, L, al);
    v5_store_main<QH>(va, lds);
    v5_load_main<QH>(va, in, hist_in, clamp(c_begin + 1), n_in, L, al);
    if constexpr (DEPTH > 1) v5_load_main<QH>(vb, in, hist_in, clamp(c_begin + 2), n_in, L, al);
    __syncthreads();

    auto step = [&](float4 (&nxt)[G::VPT], float4 (&ld)[G::VPT], int64_t ch) {
        unsigned char* cur = lds + ((ch - c_begin) & 1) * G::BUF;
        unsigned char* nbuf = lds + (((ch - c_begin) & 1) ^ 1) * G::BUF;
        v5_load_main<QH>(ld, in, hist_in, clamp(ch + 1 + DEPTH), n_in, L, al);
        v5_copy_halo<QH>(cur, nbuf);
        v5_store_main<QH>(nxt, nbuf);
        v5_compute<QH>(cur, B0, B1, B2, T, ch * G::CHUNK, n_out, out);
        __syncthreads();
    };
    int64_t ch = c_begin;
    if constexpr (DEPTH == 1) {
        for (; ch + 1 <= c_last; ch += 2) {
            step(va, vb, ch);
            step(vb, va, ch + 1);
        }
        if (ch <= c_last) step(va, vb, ch);
    } else {
        for (; ch + 2 <= c_last; ch += 3) {
            step(va, vc, ch);
            step(vb, va, ch + 1);
            step(vc, vb, ch + 2);
        }
        if (ch <= c_last) step(va, vc, ch++);
        if (ch <= c_last) step(vb, va, ch);
    }
}

template <int QH, int DEPTH>
int launch_v5(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
              hipStream_t s, int wg_per_cu)
{
    using G = geom5<QH>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma5<QH, DEPTH>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int64_t max_grid = (int64_t)n_cu * wg_per_cu;
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    const int aligned = ((uintptr_t)in % 16 == 0) ? 1 : 0;
    hipLaunchKernelGGL((k_fir_mfma5<QH, DEPTH>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const bf16x8*)p->frag16_dev, p->L, n_out, aligned);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma5)");
    return 0;
}

template <int QH>
int launch_qh(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
              hipStream_t s)
{
    switch (p->variant) {
    case 20: return launch_v5<QH, 2>(p, in, hin, hout, out, n_out, s, 2);
    case 22: return launch_v5<QH, 1>(p, in, hin, hout, out, n_out, s, 2);
    default: return launch_v5<QH, 1>(p, in, hin, hout, out, n_out, s, 3); // 163 VGPRs: 3 waves/SIMD
    }
}

// ---- v7: decimating FIR (D = 2, 4) as a polyphase Toeplitz GEMM -------------------------------
// y[m] = sum_k h[k] x[D m - k]; with k = D j + r and the phase streams
//     z_0[i] = x[D i],   z_r[i] = x[D i + D - r]  (r >= 1),
//     h'_0[j] = h[D j],  h'_r[j] = h[D (j - 1) + r]  (j >= 1; h'_r[0] = 0),
// y[m] = sum_r sum_j h'_r[j] z_r[m - j]: D ordinary FIRs at the output rate on the
// deinterleaved input, summed in the same accumulators. Each phase is laid out and
// multiplied exactly as the 16-sample form above (v5). A chunk = 2048 input samples =
// 2048/D outputs; a thread's 2D consecutive samples give one aligned bf16 pair per phase, so
// the split still writes packed 32-bit words. Per output the matrix work is about the
// decim-1 form's (K = 16 QH per phase, QH = ceil((ceil(L/D) + 16) / 16)), per input sample 1/D.
template <int D, int QH>
struct geom7 {
    static constexpr int NT = 256;
    static constexpr int CHUNK_IN = 2048;
    static constexpr int CHUNK = CHUNK_IN / D;                 // outputs per chunk
    static constexpr int TILES = 4 / D;                        // row-tiles (8 blocks of 16) per wave
    static constexpr int WAVE_OUT = TILES * 128;
    static constexpr int KS = QH / 2;
    static constexpr int TAIL = QH % 2;
    static constexpr int H = 16 * (QH - 1);                    // halo samples per phase
    static constexpr int HR = QH - 1;
    static constexpr int NB = (CHUNK + H) / 16;                // rows per phase
    static constexpr int PLANE = NB * 32;
    static constexpr int IM_OFF = (3 * PLANE + 255) / 256 * 256 + 128;
    static constexpr int PH = (IM_OFF + 3 * PLANE + 255) / 256 * 256; // one phase's planes
    static constexpr int BUF = D * PH;
    static constexpr int LDS = 2 * BUF;
    static constexpr int VPT = CHUNK_IN / 2 / NT;              // 4 float4 per thread
    static constexpr int UNITS = VPT * 2 / (2 * D);            // groups of 2D samples per thread
    static_assert(D == 2 || D == 4, "D");
    static_assert(VPT == 4, "register arrays below are declared [4]");
};

template <int D, int QH>
__device__ __forceinline__ void v7_store_pair(unsigned char* buf, int r, int s, float a_re, float b_re, float a_im,
                                              float b_im)
{
    using G = geom7<D, QH>;
    unsigned char* ph = buf + r * G::PH;
    const int off = (s >> 4) * 32 + (s & 15) * 2;
    unsigned r1, r2, r3, i1, i2, i3;
    split_pair(a_re, b_re, r1, r2, r3);
    split_pair(a_im, b_im, i1, i2, i3);
    *reinterpret_cast<unsigned*>(ph + 0 * G::PLANE + off) = r1;
    *reinterpret_cast<unsigned*>(ph + 1 * G::PLANE + off) = r2;
    *reinterpret_cast<unsigned*>(ph + 2 * G::PLANE + off) = r3;
    *reinterpret_cast<unsigned*>(ph + G::IM_OFF + 0 * G::PLANE + off) = i1;
    *reinterpret_cast<unsigned*>(ph + G::IM_OFF + 1 * G::PLANE + off) = i2;
    *reinterpret_cast<unsigned*>(ph + G::IM_OFF + 2 * G::PLANE + off) = i3;
}

// Registers: thread t holds input samples [2D (t + 256 u'), 2D (t + 256 u') + 2D) of the
// chunk, u' < UNITS, as D float4 each (2 samples per float4). Buffer loads (chunk_rsrc): the
// streaming loop's form.
template <int D, int QH>
__device__ __forceinline__ void v7_load_buf(float4 (&v)[4], const float2* __restrict__ in, int64_t ch, int64_t n_in)
{
    using G = geom7<D, QH>;
    const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK_IN>(in, ch, n_in);
#pragma unroll
    for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
        for (int f = 0; f < D; ++f) v[u * D + f] = buf_load_f4(r, ((threadIdx.x + G::NT * u) * D + f) * 16);
}
__device__ __forceinline__ float2 f4_sample(const float4& v, int which)
{
    return which ? make_float2(v.z, v.w) : make_float2(v.x, v.y);
}

// Split + deinterleave into the phase planes (rows HR.. of each phase).
template <int D, int QH>
__device__ __forceinline__ void v7_store_main(const float4 (&v)[4], unsigned char* buf)
{
    using G = geom7<D, QH>;
#pragma unroll
    for (int u = 0; u < G::UNITS; ++u) {
        const int i0 = 2 * (threadIdx.x + G::NT * u); // phase-stream index of this unit's first pair
#pragma unroll
        for (int r = 0; r < D; ++r) {
            // z_r[i] = x[D i + s_r]: local samples D i0 + s_r and D (i0 + 1) + s_r
            const int sr = r == 0 ? 0 : D - r;
            const int la = sr, lb = D + sr; // within the unit's 2D samples
            const float2 a = f4_sample(v[u * D + la / 2], la & 1);
            const float2 b = f4_sample(v[u * D + lb / 2], lb & 1);
            v7_store_pair<D, QH>(buf, r, G::H + i0, a.x, b.x, a.y, b.y);
        }
    }
}

template <int D, int QH>
__device__ __forceinline__ void v7_copy_halo(const unsigned char* cur, unsigned char* nxt)
{
    using G = geom7<D, QH>;
    constexpr int PER_PHASE = 6 * G::HR * 2;
    constexpr int PIECES = D * PER_PHASE;
    if constexpr (G::HR > 0) {
        for (int t = threadIdx.x; t < PIECES; t += G::NT) {
            const int r = t / PER_PHASE;
            const int tt = t % PER_PHASE;
            const int plane = tt / (G::HR * 2);
            const int rem = tt % (G::HR * 2);
            const int pbase = r * G::PH + (plane < 3 ? 0 : G::IM_OFF) + (plane % 3) * G::PLANE;
            const uint4 d = *reinterpret_cast<const uint4*>(cur + pbase + (G::NB - G::HR) * 32 + rem * 16);
            *reinterpret_cast<uint4*>(nxt + pbase + rem * 16) = d;
        }
    }
}

// Halo rows of the first chunk from global memory / history: z_r[i], i in [-H, 0) relative
// to the chunk's first output.
template <int D, int QH>
__device__ __forceinline__ void v7_load_store_halo(unsigned char* buf, const float2* __restrict__ in,
                                                   const float2* __restrict__ hist, int64_t ch, int64_t n_in, int L)
{
    using G = geom7<D, QH>;
    if constexpr (G::H > 0) {
        const int64_t m0 = ch * G::CHUNK; // first output of the chunk
        for (int t = threadIdx.x; t < D * (G::H / 2); t += G::NT) {
            const int r = t / (G::H / 2);
            const int pi = t % (G::H / 2);
            const int sr = r == 0 ? 0 : D - r;
            const int64_t i = m0 - G::H + 2 * pi;
            const float2 a = virt(in, hist, D * i + sr, n_in, L);
            const float2 b = virt(in, hist, D * (i + 1) + sr, n_in, L);
            v7_store_pair<D, QH>(buf, r, 2 * pi, a.x, b.x, a.y, b.y);
        }
    }
}

template <int D, int QH>
__device__ __forceinline__ void v7_compute(const unsigned char* lds, const bf16x8 (&B)[D][3][QH / 2 + 1],
                                           const bf16x4 (&T)[D][3], int64_t ch, int64_t n_out,
                                           float2* __restrict__ out)
{
    using G = geom7<D, QH>;
    const __amdgpu_buffer_rsrc_t ro = chunk_rsrc<G::CHUNK>(out, ch, n_out);
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int rho = lane & 15;
    const int c = rho & 1, b = rho >> 1;
    const int g = lane >> 4;
    const int phase = lane & 15;
    const int row_base = c * G::IM_OFF + (G::HR + wave * (G::WAVE_OUT / 16) + b) * 32;
    f32x4 hi[G::TILES], lo[G::TILES], hi_t[G::TILES], lo_t[G::TILES]; // _t: K tail (see v5_compute)
#pragma unroll
    for (int t = 0; t < G::TILES; ++t) {
        hi[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        lo[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        hi_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        lo_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
    }
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const unsigned char* ph = lds + r * G::PH;
#pragma unroll
        for (int st = 0; st < G::KS; ++st) {
            const int q = 2 * st + (g >> 1);
#pragma unroll
            for (int t = 0; t < G::TILES; ++t) {
                const int off = row_base + t * 8 * 32 - q * 32 + (g & 1) * 16;
                const bf16x8 A0 = *reinterpret_cast<const bf16x8*>(ph + off);
                const bf16x8 A1 = *reinterpret_cast<const bf16x8*>(ph + off + G::PLANE);
                const bf16x8 A2 = *reinterpret_cast<const bf16x8*>(ph + off + 2 * G::PLANE);
                hi[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B[r][0][st], hi[t], 0, 0, 0);
                lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B[r][1][st], lo[t], 0, 0, 0);
                lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B[r][0][st], lo[t], 0, 0, 0);
                lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B[r][2][st], lo[t], 0, 0, 0);
                lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B[r][1][st], lo[t], 0, 0, 0);
                lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2, B[r][0][st], lo[t], 0, 0, 0);
            }
        }
        if constexpr (G::TAIL) {
#pragma unroll
            for (int t = 0; t < G::TILES; ++t) {
                const int off = row_base + t * 8 * 32 - (QH - 1) * 32 + g * 8;
                const bf16x4 A0 = *reinterpret_cast<const bf16x4*>(ph + off);
                const bf16x4 A1 = *reinterpret_cast<const bf16x4*>(ph + off + G::PLANE);
                const bf16x4 A2 = *reinterpret_cast<const bf16x4*>(ph + off + 2 * G::PLANE);
                hi_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[r][0], hi_t[t], 0, 0, 0);
                lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[r][1], lo_t[t], 0, 0, 0);
                lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A1, T[r][0], lo_t[t], 0, 0, 0);
                lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A0, T[r][2], lo_t[t], 0, 0, 0);
                lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A1, T[r][1], lo_t[t], 0, 0, 0);
                lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(A2, T[r][0], lo_t[t], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < G::TILES; ++t) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int blk = t * 8 + 2 * g + half;
            nf2 o = { (hi[t][2 * half] + hi_t[t][2 * half]) + (lo[t][2 * half] + lo_t[t][2 * half]),
                      (hi[t][2 * half + 1] + hi_t[t][2 * half + 1]) + (lo[t][2 * half + 1] + lo_t[t][2 * half + 1]) };
            buf_store_f2(ro, (wave * G::WAVE_OUT + blk * 16 + phase) * 8, o);
        }
    }
}

template <int D, int QH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma7(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist_in,
                                                     float2* __restrict__ hist_out,
                                                     float2* __restrict__ out,
                                                     const unsigned short* __restrict__ frag,
                                                     int L,
                                                     int64_t n_out)
{
    using G = geom7<D, QH>;
    constexpr int KS = G::KS;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int64_t n_in = n_out * D;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    // fragments: per phase r: [3][KS][64] bf16x8, then [3][64] bf16x4 tail
    constexpr int PER_PHASE = 3 * KS * 64 * 8 + (G::TAIL ? 3 * 64 * 4 : 0); // bf16 elements
    bf16x8 B[D][3][KS + 1];
    bf16x4 T[D][3] = {};
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const unsigned short* fr = frag + (size_t)r * PER_PHASE;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int st = 0; st < KS; ++st) B[r][k][st] = reinterpret_cast<const bf16x8*>(fr)[(k * KS + st) * 64 + lane];
            if constexpr (G::TAIL) T[r][k] = reinterpret_cast<const bf16x4*>(fr + 3 * KS * 64 * 8)[k * 64 + lane];
        }
    }

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;
    // prefetch index: past the workgroup's range, an empty buffer range (loads return 0 and move
    // no bytes; a re-load of the last chunk would go to HBM again, the loads are nontemporal)
    auto clamp = [&](int64_t x) { return x <= c_last ? x : nchunks; };

    float4 va[G::VPT], vb[G::VPT];
    v7_load_store_halo<D, QH>(lds, in, hist_in, c_begin, n_in, L);
    v7_load_buf<D, QH>(va, in, c_begin, n_in);
    v7_store_main<D, QH>(va, lds);
    v7_load_buf<D, QH>(va, in, clamp(c_begin + 1), n_in);
    nsh::lds_barrier(); // LDS only: keep the chunk ch+2 loads in flight

    auto step = [&](float4 (&nxt)[G::VPT], float4 (&ld)[G::VPT], int64_t ch) {
        unsigned char* cur = lds + ((ch - c_begin) & 1) * G::BUF;
        unsigned char* nbuf = lds + (((ch - c_begin) & 1) ^ 1) * G::BUF;
        v7_load_buf<D, QH>(ld, in, clamp(ch + 2), n_in);
        v7_copy_halo<D, QH>(cur, nbuf);
        v7_store_main<D, QH>(nxt, nbuf);
        v7_compute<D, QH>(cur, B, T, ch, n_out, out);
        nsh::lds_barrier(); // LDS only: keep the chunk ch+2 loads in flight
    };
    int64_t ch = c_begin;
    for (; ch + 1 <= c_last; ch += 2) {
        step(va, vb, ch);
        step(vb, va, ch + 1);
    }
    if (ch <= c_last) step(va, vb, ch);
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
    static_assert(geom2<Q>::VPT == VPT && geom2<Q>::CHUNK == CHUNK, "v8 reuses v2's load_main");
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
// ---- k_fir_mfma9: the fp16x2 kernel with an exactly counted memory pipeline ----------------
// Its first form (k_fir_mfma8, removed; bit-identical outputs) tested each
// sample for the exact path in the split, used __syncthreads() and read the exact path's inputs
// from global memory -- its .s waited vmcnt(0) once per step, i.e. for the prefetch of chunk
// ch+3 issued at the top of that step. Here:
//  * barriers order LDS only (nsh::lds_barrier); __syncthreads() is a fence on global memory too;
//  * every step issues exactly 4 buffer loads (chunk ch+3) and 8 buffer stores per lane on a
//    per-chunk resource: out-of-range lanes read 0 and drop their store, so the stream's
//    partial last chunk needs no branch and the compiler's vmcnt waits count exactly;
//  * the exact path issues no global memory operation: a chunk that needs it is staged in LDS
//    as raw fp32 (instead of fp16 planes) one step ahead, and the direct form reads it there,
//    producing the same 8 outputs per lane the MFMA tile does, stored by the same 8 stores;
//  * the exact-path decision is per chunk, from the chunk maximum (non-finite) and minimum
//    nonzero magnitude (fp16-subnormal after scaling) reduced alongside the scale: a nonzero
//    sample more than 2^28 below the chunk maximum, or a non-finite one, sends the chunk to the
//    fp32 direct form; the halo test covers its whole source chunk (conservative).

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
#if NSH_FIR_ABLATE & 1024 // timing only: no global loads
    for (int u = 0; u < 4; ++u) v[u] = make_float4((float)ch, (float)u, (float)threadIdx.x, 1.f);
    return;
#endif
    const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(in, ch, n_in);
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = buf_load_f4(r, (threadIdx.x + 256 * u) * 16);
}

// split without the per-sample test (k_fir_mfma9 decides per chunk)
template <int Q>
__device__ __forceinline__ void store_pair9(const float4& v, unsigned char* buf, int s, int sc)
{
    using G = geom8<Q>;
    const int off = (s >> 5) * 80 + (s & 31) * 2;
#if NSH_FIR_ABLATE & 512 // timing only: the split's LDS writes without its conversion VALU
    *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = __float_as_uint(v.x);
    *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = __float_as_uint(v.y);
    *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = __float_as_uint(v.z);
    *reinterpret_cast<unsigned*>(buf + 3 * G::PLANE + off) = __float_as_uint(v.w);
    return;
#endif
    unsigned rh, rl, ih, il;
    split_pair16(v.x, v.z, sc, rh, rl);
    split_pair16(v.y, v.w, sc, ih, il);
    *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = rh;
    *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = rl;
    *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = ih;
    *reinterpret_cast<unsigned*>(buf + 3 * G::PLANE + off) = il;
}

// MFMA tile -> the lane's 8 outputs, unscaled (lane holds phase rho of blocks (reg & 3) +
// 8 (reg >> 2) + 4 h: rows 0-7 re, 8-15 im)
template <int Q>
__device__ __forceinline__ void mfma_tile9(const unsigned char* lds, const f16x8 (&B0)[2 * Q], const f16x8 (&B1)[2 * Q],
                                           int a_base, int unscale, nf2 (&o)[8])
{
    using G = geom8<Q>;
    f32x16 acc_hi = {};
    f32x16 acc_lo = {};
#pragma unroll
    for (int st = 0; st < 2 * Q; ++st) {
        const int off = a_base - (st >> 1) * 80 + 32 * (st & 1);
        const f16x8 A0 = *reinterpret_cast<const f16x8*>(lds + off);
        const f16x8 A1 = *reinterpret_cast<const f16x8*>(lds + off + G::PLANE);
#if NSH_FIR_ABLATE & 256 // timing only: A-fragment reads kept, no matrix work
        acc_hi[st & 15] += (float)A0[0] + (float)A1[1];
        continue;
#endif
        acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B0[st], acc_hi, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B1[st], acc_lo, 0, 0, 0);
        acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B0[st], acc_lo, 0, 0, 0);
    }
    const f32x16 sum = acc_hi + acc_lo; // packed adds
    if (unscale >= -126 && unscale <= 127) { // 2^unscale is a normal float: the multiply rounds as ldexp does
        const nf2 f = nf2{ __builtin_bit_cast(float, (unscale + 127) << 23), __builtin_bit_cast(float, (unscale + 127) << 23) };
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ sum[reg], sum[reg + 8] } * f;
    } else {
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ __builtin_ldexpf(sum[reg], unscale), __builtin_ldexpf(sum[reg + 8], unscale) };
    }
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

template <int Q>
__global__ __launch_bounds__(256, 2) void k_fir_mfma9(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist_in,
                                                     float2* __restrict__ hist_out,
                                                     float2* __restrict__ out,
                                                     const f16x8* __restrict__ frag, // [2][S][64]
                                                     const float* __restrict__ taps,
                                                     int L,
                                                     int sh,
                                                     int64_t n_out)
{
    using G = geom8<Q>;
    constexpr int S = G::S;
    static_assert((G::HP + 4 * G::NT) * 16 <= G::BUF, "a raw fp32 chunk + halo fits one plane buffer");
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* stash = reinterpret_cast<float4*>(lds + 2 * G::BUF); // [2][HP] raw fp32 chunk tails
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS); // [2][4]
    unsigned* slot_mnz = slot_max + 8;                                 // [2][4]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    f16x8 B0[S], B1[S];
#pragma unroll
    for (int st = 0; st < S; ++st) {
        B0[st] = frag[(0 * S + st) * 64 + lane];
        B1[st] = frag[(1 * S + st) * 64 + lane];
    }

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;

    const int rho = lane & 31;
    const int b = rho & 15;
    const int c = rho >> 4;
    const int h = lane >> 5;
    const int a_base = c * 2 * G::PLANE + ((Q - 1) + 16 * wave + b) * 80 + 16 * h;
    const int phase = lane & 31;
    const bool tail_owner = tid >= G::NT - G::HP; // holds the chunk's last H samples in v[3]
    // prefetch index: past the workgroup's range, an empty buffer range (loads return 0 and move
    // no bytes; a re-load of the last chunk would go to HBM again, the loads are nontemporal)
    auto clamp = [&](int64_t x) { return x <= c_last ? x : nchunks; };
    // chunk (halo pairs from hv_or_stash, main pairs from v) -> buffer, raw or split
    auto put_chunk = [&](unsigned char* buf, const float4& halo, const float4 (&v)[4], bool raw, int sc) {
        if (raw) {
            float4* r = reinterpret_cast<float4*>(buf);
            if (G::HP > 0 && tid < G::HP) r[tid] = halo;
#pragma unroll
            for (int u = 0; u < 4; ++u) r[G::HP + tid + G::NT * u] = v[u];
        } else {
            if (G::HP > 0 && tid < G::HP) store_pair9<Q>(halo, buf, 2 * tid, sc);
#pragma unroll
            for (int u = 0; u < 4; ++u) store_pair9<Q>(v[u], buf, G::H + 2 * (tid + G::NT * u), sc);
        }
    };
    auto reduce = [&](const float4 (&v)[4], unsigned& m, unsigned& z) {
        float mf = 0.f;
        z = ~0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mf = __builtin_elementwise_maximum(mf, max_abs4(v[u]));
            z = min(z, min_nz1(v[u]));
        }
        m = __float_as_uint(mf);
        m = wave_max(m);
        z = wave_min(z);
    };
    auto store_tile = [&](int64_t ch, const nf2 (&o)[8]) {
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(out, ch, n_out);
        const int base = wave * TILE + phase;
#if NSH_FIR_ABLATE & 2048 // timing only: one store per lane per chunk (keeps the results live)
        nf2 acc = o[0];
        for (int reg = 1; reg < 8; ++reg) acc += o[reg];
        if (acc.x == 1.2345e-30f) buf_store_f2(r, base * 8, acc);
        return;
#endif
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) buf_store_f2(r, (base + 32 * ((reg & 3) + 8 * (reg >> 2) + 4 * h)) * 8, o[reg]);
    };

    // ---- prologue: chunk c_begin (its halo from global memory / history), +1, +2 in flight
    float4 va[4], vb[4], vc[4];
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (G::HP > 0 && tid < G::HP) {
        const int64_t g = c_begin * G::CHUNK - G::H + 2 * tid;
        const float2 x0 = virt(in, hist_in, g, n_in, L), x1 = virt(in, hist_in, g + 1, n_in, L);
        hv = make_float4(x0.x, x0.y, x1.x, x1.y);
    }
    load_chunk9(va, in, c_begin, n_in);
    {
        unsigned m, z;
        reduce(va, m, z);
        m = max(m, wave_max(max_mag(hv)));
        z = min(z, wave_min(min_nz1(hv)));
        if (lane == 0) {
            slot_max[wave] = m;
            slot_mnz[wave] = z;
        }
    }
    nsh::lds_barrier();
    unsigned m_prev = max(max(slot_max[0], slot_max[1]), max(slot_max[2], slot_max[3]));
    unsigned z_prev = min(min(slot_mnz[0], slot_mnz[1]), min(slot_mnz[2], slot_mnz[3]));
    int s_cur = scale_of(m_prev);
    bool ex_cur = chunk_needs_exact(m_prev, z_prev, s_cur);
    put_chunk(lds, hv, va, ex_cur, s_cur);
    if (G::HP > 0 && tail_owner) stash[tid - (G::NT - G::HP)] = va[3];
    load_chunk9(va, in, clamp(c_begin + 1), n_in);
    load_chunk9(vb, in, clamp(c_begin + 2), n_in);
    {
        unsigned m, z;
        reduce(va, m, z);
        nsh::lds_barrier(); // everyone has read slots [0..3] above
        if (lane == 0) {
            slot_max[4 + wave] = m; // chunk c_begin + 1 -> parity 1
            slot_mnz[4 + wave] = z;
        }
    }
    nsh::lds_barrier();

    // step i (chunk ch = c_begin + i): nxt = chunk ch+1 (staged into the other buffer now),
    // nn = chunk ch+2 (reduced for the next step), ld receives ch+3.
    auto step = [&](float4 (&nxt)[4], float4 (&nn)[4], float4 (&ld)[4], int64_t ch) {
        const int i = (int)(ch - c_begin);
        const int pi = i & 1, pn = pi ^ 1;
        const unsigned char* cur = lds + pi * G::BUF;
        unsigned char* nbuf = lds + pn * G::BUF;
        const unsigned m_nxt = max(max(slot_max[4 * pn], slot_max[4 * pn + 1]), max(slot_max[4 * pn + 2], slot_max[4 * pn + 3]));
        const unsigned z_nxt = min(min(slot_mnz[4 * pn], slot_mnz[4 * pn + 1]), min(slot_mnz[4 * pn + 2], slot_mnz[4 * pn + 3]));
        const unsigned m2 = max(m_prev, m_nxt);
        const int s_nxt = scale_of(m2);
        // chunk ch+1 is split with chunk ch's tail (its halo) at 2^s_nxt: the test covers
        // all of chunk ch (a superset of the halo, so conservative)
        const bool ex_nxt = chunk_needs_exact(m2, min(z_prev, z_nxt), s_nxt);
        load_chunk9(ld, in, clamp(ch + 3), n_in);
        put_chunk(nbuf, G::HP > 0 && tid < G::HP ? stash[pi * G::HP + tid] : make_float4(0.f, 0.f, 0.f, 0.f), nxt, ex_nxt, s_nxt);
        if (G::HP > 0 && tail_owner) stash[pn * G::HP + tid - (G::NT - G::HP)] = nxt[3];
        nf2 o[8];
        if (ex_cur)
            direct_tile9<Q>(cur, taps, L, wave, h, phase, o);
        else
            mfma_tile9<Q>(cur, B0, B1, a_base, -(s_cur + sh), o);
        store_tile(ch, o);
        unsigned m, z;
        reduce(nn, m, z);
        if (lane == 0) {
            slot_max[4 * pi + wave] = m; // chunk ch+2 has this step's parity
            slot_mnz[4 * pi + wave] = z;
        }
        m_prev = m_nxt;
        z_prev = z_nxt;
        ex_cur = ex_nxt;
        s_cur = s_nxt;
        nsh::lds_barrier();
    };
    int64_t ch = c_begin;
    for (; ch + 2 <= c_last; ch += 3) {
        step(va, vb, vc, ch);
        step(vb, vc, va, ch + 1);
        step(vc, va, vb, ch + 2);
    }
    if (ch <= c_last) step(va, vb, vc, ch++);
    if (ch <= c_last) step(vb, vc, va, ch);
}

// ---- k_fir_mfma12: one chunk per workgroup, in address order per XCD -------------------------
// k_fir_mfma9's numerics (fp16x2 split at a per-chunk power-of-two scale, three products, the
// fp32 direct form for chunks that need it) with the access shape that copies at the HBM
// ceiling (tools/probe/shape_probe.hip, profiles/r02b_shape_probe28_runs.log): short-lived
// workgroups, each filtering ONE 2048-sample chunk, dispatched in address order with the
// chunk index remapped so that XCD x (workgroup ids x, x+8, ...) walks its own contiguous
// eighth of the stream -- 6.55 TB/s for the copy of that shape vs 5.6-5.7 TB/s for v9's
// contiguous per-workgroup ranges. Each workgroup re-reads its 32(Q-1)-sample halo (the
// previous chunk's tail, just read by the previous workgroup of the same XCD: an L2 hit) with
// the default cache policy; the probe measured no cost for it.
// Taps: v9 kept 2 x 2Q B fragments in VGPRs (80 registers, 20 KiB per wave from L2 at every
// workgroup start -- in the probe, 20 KiB of such loads per chunk cost 10-40 %). Here the
// fragments come from LDS: the scaled taps reversed, R[m] = h[32Q - 1 - m], hi and lo fp16
// planes, stored as NSH_V12_COPIES = 4 copies shifted by 0..3 elements, so the 8 consecutive taps
// a lane needs for one k-step (R[m0 .. m0 + 8)) are two aligned ds_read_b64 from copy m0 mod 4
// (or, with 8 copies, one ds_read_b128 from copy m0 mod 8). Copy pitch = 64 mod 128 bytes: each
// 32-lane group of a ds_read_b64 and each 16-lane group of a ds_read_b128 ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, and +32; MI355X_MICROARCH.md §LDS) hits distinct banks for every k-step and
// every Q (exhaustive check over pitches; the earlier 32 mod 64 pitch was 2-way on every tap
// read, 35 % of the kernel's LDS cycles in profiles/r02f_pmc_fir.json). The image
// (2 x 4 x (32Q + 32) fp16, 3 KiB at Q = 5) is prepared on the host and loaded per workgroup
// (L1/L2 hits: every workgroup reads the same bytes).
// Scale and exact-path test cover the chunk and its halo. Results match v9 to within the
// split's rounding (v9's scale also covered the whole previous chunk), not bit for bit.
// Chunk order inside an XCD: workgroup k of an XCD's sequence filters chunk k (address order), or,
// with NSH_V12_ROT (default), chunk k with its low two bits rotated by an xor-fold of k >> 2 (a
// bijection on every full group of 4, the order still ascending group by group). Without it, chunks
// that need the exact path every 4th or 8th chunk were as slow as all-exact streams
// (profiles/r02t_cliff_curve.log: k = 3 1381 us, k = 4 2775, k = 6 1260, k = 8 1602): consecutive
// workgroups of an XCD are dealt out round-robin, so a power-of-two stride landed every slow chunk
// on the same quarter of the XCD. Rotated: k = 4 1216 us, k = 8 957, k = 2 1703; main path
// bit-identical, 718.0 vs 721.2 us (profiles/r02u_*).
#ifndef NSH_V12_ROT
#define NSH_V12_ROT 1
#endif
#ifndef NSH_V12_LDS_PAD
#define NSH_V12_LDS_PAD 0 // probe builds: extra LDS per workgroup (fewer resident workgroups per CU)
#endif
// Shifted tap copies: 4, read as two ds_read_b64 per B fragment (8-B aligned), or 8, read as one
// ds_read_b128 (16-B aligned). Four copies take 3.5 KiB instead of 7 at Q = 5, which brings the
// workgroup to 25.5 KiB of LDS: 6 resident workgroups per CU instead of 5 (LDS-bound; 72 VGPRs
// would allow 7) -- the kernel's rate follows the chunks in flight per CU (5 -> 4 resident
// workgroups: 734 -> 802 us per 2^28, profiles/r02j_v12_occupancy_ab.log).
#ifndef NSH_V12_COPIES
#define NSH_V12_COPIES 4
#endif
constexpr int v12_tw(int Q) { return 32 * Q + (NSH_V12_COPIES == 8 ? 24 : 32); } // fp16 per copy (multiple of 8)
// Plane row pitch (32 fp16 samples = 64 B per row): 80 B (v9's padded rows) or 64 B with the
// row's four 16-B chunks XOR-swizzled by (row >> 2) & 3. Either way each 16-lane group of an
// A-fragment ds_read_b128 (16 consecutive rows, one chunk) hits 16 distinct 16-B slots; the
// unpadded form takes 17 KiB instead of 22 for the four planes (20.5 KiB per workgroup with the
// 4-copy tap image: 7 resident workgroups per CU, the 72-VGPR limit) but measured slower than 6
// (732 vs 708-719 us, bit-identical; profiles/r02j_v12_occupancy_ab.log): 80 is the default.
#ifndef NSH_V12_PITCH
#define NSH_V12_PITCH 80
#endif
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
template <int Q>
struct geom12 {
    static constexpr int NT = 256;
    static constexpr int CHUNK = 2048;
    static constexpr int H = 32 * (Q - 1);
    static constexpr int HP = H / 2;
    static constexpr int NB = (CHUNK + H) / 32;
    static constexpr int PITCH = NSH_V12_PITCH;
    static constexpr int PLANE = (NB * PITCH + 255) / 256 * 256;
    static constexpr int BUF = 4 * PLANE;
    static constexpr int NCP = NSH_V12_COPIES;                       // shifted copies per plane
    static constexpr int TW = v12_tw(Q);                             // fp16 per shifted copy
    static constexpr int COPY = ((2 * TW + 63) / 128) * 128 + 64;    // bytes, = 64 mod 128, >= 2 TW
    static constexpr int TAPS = 2 * NCP * COPY;                      // [plane][shift] copies
    static constexpr int IMG_UNITS = 2 * NCP * TW / 8;               // 16-B units of the global image
    static constexpr int SLOTS = BUF + TAPS;                         // u32 max[4], mnz[4]
    static constexpr int LDS = SLOTS + 32 + NSH_V12_LDS_PAD;
    static_assert(COPY >= 2 * TW && COPY % 128 == 64, "copy pitch");
    static_assert((HP + 4 * NT) * 16 <= BUF, "a raw fp32 chunk + halo fits the plane buffer");
    static_assert(HP <= NT, "halo pairs: one per thread");
    static_assert(NCP == 4 || NCP == 8, "4 or 8 shifted tap copies");
    static_assert(PITCH == 64 || PITCH == 80, "plane pitch");
    // byte offset of sample s (even) in a plane
    static __device__ __forceinline__ int at(int s)
    {
        const int row = s >> 5;
        if (PITCH == 80) return row * 80 + (s & 31) * 2;
        return row * 64 + ((((s >> 3) & 3) ^ ((row >> 2) & 3)) << 4) + (s & 7) * 2;
    }
    static_assert(IMG_UNITS <= 2 * NT, "tap image: two 16-B units per thread at most");
};

template <int Q>
__device__ __forceinline__ void store_pair12(const float4& v, unsigned char* buf, int s, int sc)
{
    using G = geom12<Q>;
    const int off = G::at(s);
    unsigned rh, rl, ih, il;
    split_pair16(v.x, v.z, sc, rh, rl);
    split_pair16(v.y, v.w, sc, ih, il);
    *reinterpret_cast<unsigned*>(buf + 0 * G::PLANE + off) = rh;
    *reinterpret_cast<unsigned*>(buf + 1 * G::PLANE + off) = rl;
    *reinterpret_cast<unsigned*>(buf + 2 * G::PLANE + off) = ih;
    *reinterpret_cast<unsigned*>(buf + 3 * G::PLANE + off) = il;
}

template <int Q>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_fir_mfma12(const float2* __restrict__ in,
                                                    const float2* __restrict__ hist_in,
                                                    float2* __restrict__ hist_out,
                                                    float2* __restrict__ out,
                                                    const uint4* __restrict__ timg, // [2][8][TW/8]
                                                    const float* __restrict__ taps,
                                                    int L,
                                                    int sh,
                                                    int64_t n_out,
                                                    int64_t per_x)
{
    using G = geom12<Q>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* tl = lds + G::BUF;
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    unsigned* slot_mnz = slot_max + 4;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out;
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    int64_t wi = blockIdx.x >> 3; // this workgroup's place in its XCD's sequence
#if NSH_V12_ROT
    if ((wi | 3) < per_x) { // full aligned group of 4: rotate it by an xor-fold of the group index
        const uint64_t grp = (uint64_t)wi >> 2;
        unsigned r = (unsigned)grp ^ (unsigned)(grp >> 32);
        r ^= r >> 16;
        r ^= r >> 8;
        r ^= r >> 4;
        r ^= r >> 2;
        wi = (wi & ~(int64_t)3) | ((wi - (int64_t)r) & 3);
    }
#endif
    const int64_t c_first = (int64_t)(blockIdx.x & 7) * per_x + wi;
    if (c_first >= nchunks) return; // whole workgroup: before any barrier

    // chunk ch -> registers (nontemporal) and its halo (default policy: the previous chunk's
    // tail was just read by this or the previous workgroup of this XCD). Branch-free: the halo
    // comes through one buffer resource, over `in` (ch > 0) or over hist_in (ch = 0; out-of-range
    // lanes and a null history read zeros), so no wait sits between the loads.
    auto load = [&](int64_t ch, float4 (&v)[4], float4& hv) {
        load_chunk9(v, in, ch, n_in);
        __amdgpu_buffer_rsrc_t hr;
        int off0, off1; // per sample: with an odd history length a pair straddles its start
        if (ch > 0) {
            hr = chunk_rsrc<G::H>(in + ch * G::CHUNK - G::H, 0, G::H);
            off0 = 16 * tid;
            off1 = off0 + 8;
        } else {
            hr = chunk_rsrc<1 << 20>(hist_in, 0, hist_in ? L - 1 : 0);
            const int e = 2 * tid - G::H + (L - 1); // history element of the lane's first sample
            off0 = e >= 0 ? 8 * e : 1 << 30;         // past num_records -> zeros
            off1 = e + 1 >= 0 ? 8 * (e + 1) : 1 << 30;
        }
        hv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tid < G::HP) {
            const nsh::buf_f2 a = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off0, 0, 0));
            const nsh::buf_f2 b = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off1, 0, 0));
            hv = make_float4(a.x, a.y, b.x, b.y);
        }
    };
    float4 va[4], ha;
    load(c_first, va, ha);
    constexpr int UPC = G::TW / 8; // 16-B units per copy
    uint4 ti[2] = {};
    {   // the tap image (L1/L2 hits), both units per lane issued before any wait
        const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc((void*)timg, (short)0, G::IMG_UNITS * 16, 0x00020000);
#pragma unroll
        for (int k = 0; k < 2; ++k)
            ti[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(tr, 16 * (tid + G::NT * k), 0, 0));
    }
    // tap image -> LDS at the padded copy pitch
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int u = tid + G::NT * k;
        if (u < G::IMG_UNITS) *reinterpret_cast<uint4*>(tl + (u / UPC) * G::COPY + 16 * (u % UPC)) = ti[k];
    }

    const int rho = lane & 31;
    const int h = lane >> 5;
    const int phase = rho;
    auto process = [&](int64_t ch, const float4 (&v)[4], const float4& hv) {
        {   // chunk + halo range -> workgroup scale and exact-path decision
            float mf = max_abs4(hv);
            unsigned z = min_nz1(hv);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                mf = __builtin_elementwise_maximum(mf, max_abs4(v[u]));
                z = min(z, min_nz1(v[u]));
            }
            const unsigned m = wave_max(__float_as_uint(mf));
            z = wave_min(z);
            if (lane == 0) {
                slot_max[wave] = m;
                slot_mnz[wave] = z;
            }
        }
        nsh::lds_barrier(); // also: every wave is done with the previous chunk's planes
        const unsigned m = max(max(slot_max[0], slot_max[1]), max(slot_max[2], slot_max[3]));
        const unsigned z = min(min(slot_mnz[0], slot_mnz[1]), min(slot_mnz[2], slot_mnz[3]));
        const int s = scale_of(m);
        const bool exact = chunk_needs_exact(m, z, s);
        if (exact) {
            float4* r = reinterpret_cast<float4*>(lds);
            if (tid < G::HP) r[tid] = hv;
#pragma unroll
            for (int u = 0; u < 4; ++u) r[G::HP + tid + G::NT * u] = v[u];
        } else {
            if (tid < G::HP) store_pair12<Q>(hv, lds, 2 * tid, s);
#pragma unroll
            for (int u = 0; u < 4; ++u) store_pair12<Q>(v[u], lds, G::H + 2 * (tid + G::NT * u), s);
        }
        nsh::lds_barrier();
        nf2 o[8];
        if (exact) {
            direct_tile9<Q>(lds, taps, L, wave, h, phase, o);
        } else {
            const int b = rho & 15, c = rho >> 4;
            const int row0 = (Q - 1) + 16 * wave + b; // A rows: row0 - (st >> 1); chunks h + 2 (st & 1)
            const int a_base = c * 2 * G::PLANE + row0 * G::PITCH + 16 * h;
            f32x16 acc_hi = {};
            f32x16 acc_lo = {};
#pragma unroll
            for (int st = 0; st < 2 * Q; ++st) {
                int off;
                if (G::PITCH == 80) {
                    off = a_base - (st >> 1) * 80 + 32 * (st & 1);
                } else {
                    const int row = row0 - (st >> 1);
                    off = c * 2 * G::PLANE + row * 64 + (((h + 2 * (st & 1)) ^ ((row >> 2) & 3)) << 4);
                }
                const f16x8 A0 = *reinterpret_cast<const f16x8*>(lds + off);
                const f16x8 A1 = *reinterpret_cast<const f16x8*>(lds + off + G::PLANE);
                // taps h[t0 - j], t0 = i - 16 (st & 1) - 8 h + 32 (st >> 1): R[m0 + j], m0 = 32Q - 1 - t0
                const int m0 = 32 * Q - 1 - rho + 16 * (st & 1) + 8 * h - 32 * (st >> 1);
                const int tb = (m0 & (G::NCP - 1)) * G::COPY + 2 * (m0 & ~(G::NCP - 1));
                f16x8 B0, B1;
                if (G::NCP == 8) {
                    B0 = *reinterpret_cast<const f16x8*>(tl + tb);
                    B1 = *reinterpret_cast<const f16x8*>(tl + G::NCP * G::COPY + tb);
                } else {
                    // four separate ds_read_b64 (the empty asm keeps the compiler from pairing
                    // them into ds_read2_b64, whose 16-lane groups conflict 2-way on this image)
                    const f16x4 b0 = *reinterpret_cast<const f16x4*>(tl + tb);
                    asm volatile("" ::: "memory");
                    const f16x4 b1 = *reinterpret_cast<const f16x4*>(tl + tb + 8);
                    asm volatile("" ::: "memory");
                    const f16x4 b2 = *reinterpret_cast<const f16x4*>(tl + G::NCP * G::COPY + tb);
                    asm volatile("" ::: "memory");
                    const f16x4 b3 = *reinterpret_cast<const f16x4*>(tl + G::NCP * G::COPY + tb + 8);
                    B0 = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
                    B1 = __builtin_shufflevector(b2, b3, 0, 1, 2, 3, 4, 5, 6, 7);
                }
                acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B0, acc_hi, 0, 0, 0);
                acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B1, acc_lo, 0, 0, 0);
                acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B0, acc_lo, 0, 0, 0);
            }
            const f32x16 sum = acc_hi + acc_lo;
            const int unscale = -(s + sh);
            if (unscale >= -126 && unscale <= 127) {
                const nf2 f = nf2{ __builtin_bit_cast(float, (unscale + 127) << 23), __builtin_bit_cast(float, (unscale + 127) << 23) };
#pragma unroll
                for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ sum[reg], sum[reg + 8] } * f;
            } else {
#pragma unroll
                for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ __builtin_ldexpf(sum[reg], unscale), __builtin_ldexpf(sum[reg + 8], unscale) };
            }
        }
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(out, ch, n_out);
        const int base = wave * TILE + phase;
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) buf_store_f2(r, (base + 32 * ((reg & 3) + 8 * (reg >> 2) + 4 * h)) * 8, o[reg]);
    };
    process(c_first, va, ha);
    if (c_first == 0) // the last L-1 inputs for the next call (after this workgroup's stores)
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
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
    static constexpr int PH = (IM_OFF + 2 * PLANE + 255) / 256 * 256;
    static constexpr int BUF = D * PH;
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

template <int D, int QH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma11(const float2* __restrict__ in,
                                                      const float2* __restrict__ hist_in,
                                                      float2* __restrict__ hist_out,
                                                      float2* __restrict__ out,
                                                      const _Float16* __restrict__ frag, // per phase: [2][KS][64] x8, [2][64] x4
                                                      const float* __restrict__ taps,
                                                      int L,
                                                      int sh,
                                                      int64_t n_out)
{
    using G = geom11<D, QH>;
    constexpr int KS = G::KS;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* stash = reinterpret_cast<float4*>(lds + 2 * G::BUF); // [2][HP] raw halo sources
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    unsigned* slot_mnz = slot_max + 8;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out * D;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    f16x8 B0[D][KS + 1], B1[D][KS + 1];
    f16x4 T0[D], T1[D];
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const _Float16* fr = frag + (size_t)r * G::PER_PHASE;
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            B0[r][st] = reinterpret_cast<const f16x8*>(fr)[(0 * KS + st) * 64 + lane];
            B1[r][st] = reinterpret_cast<const f16x8*>(fr)[(1 * KS + st) * 64 + lane];
        }
        const f16x4* tf = reinterpret_cast<const f16x4*>(fr + 2 * KS * 64 * 8);
        T0[r] = tf[lane];
        T1[r] = tf[64 + lane];
    }

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;

    const int rho = lane & 15;
    const int c = rho & 1, b = rho >> 1;
    const int g = lane >> 4;
    const int phase = lane & 15;
    const int row_base = c * G::IM_OFF + (G::HR + wave * (G::WAVE_OUT / 16) + b) * 32;
    const bool tail_owner = tid >= G::NT - G::H / 2; // holds the chunk's last D*H samples (last unit)
    // prefetch index: past the workgroup's range, an empty buffer range (loads return 0 and move
    // no bytes; a re-load of the last chunk would go to HBM again, the loads are nontemporal)
    auto clamp = [&](int64_t x) { return x <= c_last ? x : nchunks; };
    auto load = [&](float4 (&v)[4], int64_t ch) {
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK_IN>(in, ch, n_in);
#pragma unroll
        for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
            for (int f = 0; f < D; ++f) v[u * D + f] = buf_load_f4(r, ((tid + G::NT * u) * D + f) * 16);
    };
    auto stash_tail = [&](float4* st, const float4 (&v)[4]) {
        if (tail_owner) {
#pragma unroll
            for (int f = 0; f < D; ++f) st[(tid - (G::NT - G::H / 2)) * D + f] = v[(G::UNITS - 1) * D + f];
        }
    };
    // chunk -> buffer: raw fp32 (halo float4 [0, HP), chunk float4 HP + j) or split phase planes
    auto put_chunk = [&](unsigned char* buf, const float4* hsrc, const float4 (&v)[4], bool raw, int sc) {
        if (raw) {
            float4* rb = reinterpret_cast<float4*>(buf);
            if (tid < G::HP) rb[tid] = hsrc[tid];
#pragma unroll
            for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
                for (int f = 0; f < D; ++f) rb[G::HP + (tid + G::NT * u) * D + f] = v[u * D + f];
            return;
        }
        if (tid < D * (G::H / 2)) { // halo: phase r, pair pi from the raw halo samples
            const int r = tid / (G::H / 2), pi = tid % (G::H / 2);
            const int sr = r == 0 ? 0 : D - r;
            const int pa = D * (2 * pi) + sr, pb = D * (2 * pi + 1) + sr;
            const float2 a = f4_sample(hsrc[pa >> 1], pa & 1), bb = f4_sample(hsrc[pb >> 1], pb & 1);
            store_pair11<D, QH>(buf, r, 2 * pi, a.x, bb.x, a.y, bb.y, sc);
        }
#pragma unroll
        for (int u = 0; u < G::UNITS; ++u) {
            const int i0 = 2 * (tid + G::NT * u);
#pragma unroll
            for (int r = 0; r < D; ++r) {
                const int sr = r == 0 ? 0 : D - r;
                const int la = sr, lb = D + sr;
                const float2 a = f4_sample(v[u * D + la / 2], la & 1);
                const float2 bb = f4_sample(v[u * D + lb / 2], lb & 1);
                store_pair11<D, QH>(buf, r, G::H + i0, a.x, bb.x, a.y, bb.y, sc);
            }
        }
    };
    auto reduce = [&](const float4 (&v)[4], unsigned& m, unsigned& z) {
        float mf = 0.f;
        z = ~0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mf = __builtin_elementwise_maximum(mf, max_abs4(v[u]));
            z = min(z, min_nz1(v[u]));
        }
        m = __float_as_uint(mf);
        m = wave_max(m);
        z = wave_min(z);
    };
    auto mfma_tile = [&](const unsigned char* cur, int unscale, nf2 (&o)[2 * G::TILES]) {
        f32x4 hi[G::TILES], lo[G::TILES], hi_t[G::TILES], lo_t[G::TILES];
#pragma unroll
        for (int t = 0; t < G::TILES; ++t) {
            hi[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            lo[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            hi_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            lo_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        }
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const unsigned char* ph = cur + r * G::PH;
#pragma unroll
            for (int st = 0; st < KS; ++st) {
                const int q = 2 * st + (g >> 1);
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - q * 32 + (g & 1) * 16;
                    const f16x8 A0 = *reinterpret_cast<const f16x8*>(ph + off);
                    const f16x8 A1 = *reinterpret_cast<const f16x8*>(ph + off + G::PLANE);
                    hi[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0[r][st], hi[t], 0, 0, 0);
                    lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1[r][st], lo[t], 0, 0, 0);
                    lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0[r][st], lo[t], 0, 0, 0);
                }
            }
            if constexpr (G::TAIL) { // separate accumulators: see v5_compute
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - (QH - 1) * 32 + g * 8;
                    const f16x4 A0 = *reinterpret_cast<const f16x4*>(ph + off);
                    const f16x4 A1 = *reinterpret_cast<const f16x4*>(ph + off + G::PLANE);
                    hi_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, T0[r], hi_t[t], 0, 0, 0);
                    lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, T1[r], lo_t[t], 0, 0, 0);
                    lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A1, T0[r], lo_t[t], 0, 0, 0);
                }
            }
        }
        nf2 sum[2 * G::TILES];
#pragma unroll
        for (int t = 0; t < G::TILES; ++t)
#pragma unroll
            for (int half = 0; half < 2; ++half)
                sum[2 * t + half] = (nf2{ hi[t][2 * half], hi[t][2 * half + 1] } + nf2{ hi_t[t][2 * half], hi_t[t][2 * half + 1] }) +
                                    (nf2{ lo[t][2 * half], lo[t][2 * half + 1] } + nf2{ lo_t[t][2 * half], lo_t[t][2 * half + 1] });
        unscale_tile(sum, unscale, o);
    };
    // exact path: y[m] = sum_k h[k] x[D m - k] from the raw chunk (float2 index D H + D m - k)
    // exact path. D = 4: outputs 0 and 1 are 64 input samples apart and share their inputs
    // (direct_group; decim_qh gives L - 1 <= D H and every k <= D (H - 16) below L): dense-exact
    // floor 74.7 -> 97.6 GS/s input. D = 2 keeps one output at a time: its two unrolled groups
    // cost the main path a third of its speed (594 -> 890 us per 2^28, profiles/r02o_*).
    auto direct_tile = [&](const unsigned char* cur, nf2 (&o)[2 * G::TILES]) {
        if constexpr (D == 4 || NSH_DECIM2_SHARED) {
#pragma unroll 1
            for (int t = 0; t < G::TILES; ++t) {
                nf2 acc[2];
                direct_group<2, 16 * D, D * G::H, D * (G::H - 16)>(
                    reinterpret_cast<const nf2*>(cur), D * G::H + D * (wave * G::WAVE_OUT + (8 * t + 2 * g) * 16 + phase), taps, L, acc);
                if (t == 0) {
                    o[0] = acc[0];
                    o[1] = acc[1];
                } else {
                    o[2 * G::TILES - 2] = acc[0];
                    o[2 * G::TILES - 1] = acc[1];
                }
            }
        } else {
            const float2* raw = reinterpret_cast<const float2*>(cur);
            for (int oi = 0; oi < 2 * G::TILES; ++oi) {
                const int blk = (oi >> 1) * 8 + 2 * g + (oi & 1);
                const int j = D * G::H + D * (wave * G::WAVE_OUT + blk * 16 + phase);
                float re = 0.f, im = 0.f;
                for (int k = 0; k < L; ++k) {
                    const float2 x = raw[j - k];
                    re = fmaf(taps[k], x.x, re);
                    im = fmaf(taps[k], x.y, im);
                }
                o[oi] = nf2{ re, im };
            }
        }
    };
    auto store_tile = [&](int64_t ch, const nf2 (&o)[2 * G::TILES]) {
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK>(out, ch, n_out);
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi)
            buf_store_f2(r, (wave * G::WAVE_OUT + ((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase) * 8, o[oi]);
    };

    // ---- prologue: chunk c_begin's halo (global memory / history) into stash[1] (free until
    // step 0 writes it), the chunk itself; chunks +1, +2 in flight
    float4 va[4], vb[4], vc[4];
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < G::HP) {
        const int64_t gg = c_begin * G::CHUNK_IN - 2 * G::HP + 2 * tid;
        const float2 x0 = virt(in, hist_in, gg, n_in, L), x1 = virt(in, hist_in, gg + 1, n_in, L);
        hv = make_float4(x0.x, x0.y, x1.x, x1.y);
        stash[G::HP + tid] = hv;
    }
    load(va, c_begin);
    {
        unsigned m, z;
        reduce(va, m, z);
        m = max(m, wave_max(max_mag(hv)));
        z = min(z, wave_min(min_nz1(hv)));
        if (lane == 0) {
            slot_max[wave] = m;
            slot_mnz[wave] = z;
        }
    }
    nsh::lds_barrier();
    unsigned m_prev = max(max(slot_max[0], slot_max[1]), max(slot_max[2], slot_max[3]));
    unsigned z_prev = min(min(slot_mnz[0], slot_mnz[1]), min(slot_mnz[2], slot_mnz[3]));
    int s_cur = scale_of(m_prev);
    bool ex_cur = chunk_needs_exact(m_prev, z_prev, s_cur);
    put_chunk(lds, stash + G::HP, va, ex_cur, s_cur);
    stash_tail(stash, va);
    load(va, clamp(c_begin + 1));
    load(vb, clamp(c_begin + 2));
    {
        unsigned m, z;
        reduce(va, m, z);
        nsh::lds_barrier(); // slots [0..3] and stash[1] read above
        if (lane == 0) {
            slot_max[4 + wave] = m;
            slot_mnz[4 + wave] = z;
        }
    }
    nsh::lds_barrier();

    auto step = [&](float4 (&nxt)[4], float4 (&nn)[4], float4 (&ld)[4], int64_t ch) {
        const int i = (int)(ch - c_begin);
        const int pi = i & 1, pn = pi ^ 1;
        const unsigned char* cur = lds + pi * G::BUF;
        unsigned char* nbuf = lds + pn * G::BUF;
        const unsigned m_nxt = max(max(slot_max[4 * pn], slot_max[4 * pn + 1]), max(slot_max[4 * pn + 2], slot_max[4 * pn + 3]));
        const unsigned z_nxt = min(min(slot_mnz[4 * pn], slot_mnz[4 * pn + 1]), min(slot_mnz[4 * pn + 2], slot_mnz[4 * pn + 3]));
        const unsigned m2 = max(m_prev, m_nxt);
        const int s_nxt = scale_of(m2);
        const bool ex_nxt = chunk_needs_exact(m2, min(z_prev, z_nxt), s_nxt);
        load(ld, clamp(ch + 3));
        put_chunk(nbuf, stash + pi * G::HP, nxt, ex_nxt, s_nxt);
        stash_tail(stash + pn * G::HP, nxt);
        nf2 o[2 * G::TILES];
        if (ex_cur)
            direct_tile(cur, o);
        else
            mfma_tile(cur, -(s_cur + sh), o);
        store_tile(ch, o);
        unsigned m, z;
        reduce(nn, m, z);
        if (lane == 0) {
            slot_max[4 * pi + wave] = m;
            slot_mnz[4 * pi + wave] = z;
        }
        m_prev = m_nxt;
        z_prev = z_nxt;
        ex_cur = ex_nxt;
        s_cur = s_nxt;
        nsh::lds_barrier();
    };
    int64_t ch = c_begin;
    for (; ch + 2 <= c_last; ch += 3) {
        step(va, vb, vc, ch);
        step(vb, vc, va, ch + 1);
        step(vc, va, vb, ch + 2);
    }
    if (ch <= c_last) step(va, vb, vc, ch++);
    if (ch <= c_last) step(vb, vc, va, ch);
}

template <int D, int QH>
int launch_v7(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
              hipStream_t s)
{
    using G = geom7<D, QH>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma7<D, QH>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int wg_per_cu = (160 * 1024) / G::LDS >= 3 ? 3 : 2; // LDS-bound residency (VGPRs allow 3)
    const int64_t max_grid = (int64_t)n_cu * wg_per_cu;
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    hipLaunchKernelGGL((k_fir_mfma7<D, QH>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const unsigned short*)p->fragd_dev, p->L, n_out);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma decim)");
    return 0;
}

template <int D, int QH>
int launch_v11(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geom11<D, QH>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma11<D, QH>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int64_t max_grid = (int64_t)n_cu * 2; // launch_v9's longer grids measured 4-7 % slower here
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    hipLaunchKernelGGL((k_fir_mfma11<D, QH>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const _Float16*)p->fragd8_dev, (const float*)p->taps_dev, p->L, p->sh8, n_out);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma decim fp16x2)");
    return 0;
}

template <int D>
int launch_dec(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    if (p->fragd8_dev && p->variant != 7) {
        switch (p->QHD) {
        case 2: return launch_v11<D, 2>(p, in, hin, hout, out, n_out, s);
        case 3: return launch_v11<D, 3>(p, in, hin, hout, out, n_out, s);
        case 4: return launch_v11<D, 4>(p, in, hin, hout, out, n_out, s);
        case 5: return launch_v11<D, 5>(p, in, hin, hout, out, n_out, s);
        case 6: return launch_v11<D, 6>(p, in, hin, hout, out, n_out, s);
        default: return nsh::fail_msg("nsh_fir_ccf(mfma decim): unsupported tap count");
        }
    }
    switch (p->QHD) {
    case 2: return launch_v7<D, 2>(p, in, hin, hout, out, n_out, s);
    case 3: return launch_v7<D, 3>(p, in, hin, hout, out, n_out, s);
    case 4: return launch_v7<D, 4>(p, in, hin, hout, out, n_out, s);
    case 5: return launch_v7<D, 5>(p, in, hin, hout, out, n_out, s);
    case 6: return launch_v7<D, 6>(p, in, hin, hout, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma decim): unsupported tap count");
    }
}

// ---- k_fir_casc2: two decimate-by-2 FIRs fused, stage 1's outputs never leave the CU -------
// y1 = fir(h1, 2) x, y2 = fir(h2, 2) y1 in one launch. HBM per input sample: 8 B in + 0.5 B
// out, against 8 + 4 + 4 + 2 for the two kernels apart. Step s of a workgroup (one LDS
// barrier, every memory operation unconditional) does, for its chunk sequence:
//   stage 1, as k_fir_mfma11<2, QH1>'s step: prefetch x chunk s+3, split chunk s+1, MFMA
//     chunk s -> y1 (1024 samples, 4 per lane), kept in registers until the next step;
//   stage 2 split of y1 chunk s-1 (the previous step's registers), at a scale set by that
//     chunk's maximum (reduced last step, read after the barrier) and its predecessor's: lanes
//     pair same-phase samples y1[m], y1[m+2] with a DPP exchange inside each quad and write the
//     fp16x2 planes (or raw fp32 when the chunk needs the exact path); the 2 H2-sample halo is
//     the raw tail of y1 chunk s-2, kept in an LDS stash;
//   stage 2 MFMA (or fp32 direct form) on y1 chunk s-2's planes -> 512 y2, stored.
// So stage 2 lags stage 1 by two steps: the loop runs two extra steps (stage 1 on the clamped
// last chunk, results unused) and the first two steps' stage-2 stores go to an empty buffer
// range (dropped). The y1 tail before a workgroup's first chunk (its first halo) and the y1
// history the call hands on are computed by the fp32 direct form from x (or taken from the y1
// history at the stream start) before the loop. Stage-2 taps live in LDS (the stage-1 B fragments already fill
// the VGPR budget).
template <int QH>
struct geomc2 {
    static constexpr int NT = 256;
    static constexpr int CHUNK_IN = 1024;
    static constexpr int CHUNK = 512;
    static constexpr int WAVE_OUT = 128;
    static constexpr int KS = QH / 2;
    static constexpr int TAIL = QH % 2;
    static constexpr int H = 16 * (QH - 1);                    // halo samples per phase
    static constexpr int HR = QH - 1;
    static constexpr int NB = (CHUNK + H) / 16;
    static constexpr int PLANE = NB * 32;
    static constexpr int IM_OFF = (2 * PLANE + 255) / 256 * 256 + 128;
    static constexpr int PH = (IM_OFF + 2 * PLANE + 255) / 256 * 256;
    static constexpr int BUF = 2 * PH;
    static constexpr int PER_PHASE = 2 * KS * 64 * 8 + 2 * 64 * 4; // fp16 tap elements
    static_assert((2 * H + CHUNK_IN) * 8 <= BUF, "a raw fp32 y1 chunk + halo fits the plane buffer");
    static_assert(H / 2 <= NT, "halo: one thread per 4 samples");
};
template <int QH1, int QH2>
struct geomcasc {
    using G1 = geom11<2, QH1>;
    using G2 = geomc2<QH2>;
    static constexpr int P2 = G1::SLOTS + 64;                  // stage-2 planes [2][BUF]
    static constexpr int ST2 = P2 + 2 * G2::BUF;               // raw y1 tails float2 [2][2 H2]
    static constexpr int F2 = ST2 + 2 * 2 * G2::H * 8;         // stage-2 fragments, 2 phases
    static constexpr int S2 = F2 + 2 * G2::PER_PHASE * 2;      // u32 max[2][4], mnz[2][4]
    static constexpr int LDS = S2 + 64;
    static_assert(2 * LDS <= 160 * 1024, "two workgroups per CU");
};

template <int QH1, int QH2>
__global__ __launch_bounds__(256, 2) void k_fir_casc2(const float2* __restrict__ in,
                                                     const float2* __restrict__ hist1_in,
                                                     float2* __restrict__ hist1_out,
                                                     const float2* __restrict__ hist2_in,
                                                     float2* __restrict__ hist2_out,
                                                     float2* __restrict__ out,
                                                     const _Float16* __restrict__ frag1,
                                                     const float* __restrict__ taps1, int L1, int sh1,
                                                     const _Float16* __restrict__ frag2,
                                                     const float* __restrict__ taps2, int L2, int sh2,
                                                     int64_t n_out)
{
    constexpr int D = 2;
    using C = geomcasc<QH1, QH2>;
    using G = geom11<D, QH1>;
    using G2 = geomc2<QH2>;
    constexpr int KS = G::KS;
    constexpr int KS2 = G2::KS;
    constexpr int HY = 2 * G2::H; // stage-2 halo, y1 samples
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* stash = reinterpret_cast<float4*>(lds + 2 * G::BUF);
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    unsigned* slot_mnz = slot_max + 8;
    float2* st2 = reinterpret_cast<float2*>(lds + C::ST2);
    _Float16* F2 = reinterpret_cast<_Float16*>(lds + C::F2);
    unsigned* s2_max = reinterpret_cast<unsigned*>(lds + C::S2);
    unsigned* s2_mnz = s2_max + 8;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n1 = 2 * n_out;
    const int64_t n_in = 4 * n_out;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L1 - 1; j += G::NT) hist1_out[j] = virt(in, hist1_in, n_in - (L1 - 1) + j, n_in, L1);
    }
    // y1[v] by the fp32 direct form (v < 0: the y1 history); plain loads when the window lies
    // inside this call's input (every workgroup's first halo but the stream start's)
    auto y1_direct = [&](int64_t v) -> float2 {
        if (v < 0) return v >= -(int64_t)(L2 - 1) && hist2_in ? hist2_in[v + (L2 - 1)] : make_float2(0.f, 0.f);
        float re = 0.f, im = 0.f;
        if (2 * v - (L1 - 1) >= 0 && 2 * v < n_in) {
            const float2* xv = in + 2 * v;
#pragma unroll 8
            for (int k = 0; k < L1; ++k) {
                const float2 x = xv[-k];
                re = fmaf(taps1[k], x.x, re);
                im = fmaf(taps1[k], x.y, im);
            }
        } else {
            for (int k = 0; k < L1; ++k) {
                const float2 x = virt(in, hist1_in, 2 * v - k, n_in, L1);
                re = fmaf(taps1[k], x.x, re);
                im = fmaf(taps1[k], x.y, im);
            }
        }
        return make_float2(re, im);
    };

    f16x8 B0[D][KS + 1], B1[D][KS + 1];
    f16x4 T0[D], T1[D];
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const _Float16* fr = frag1 + (size_t)r * G::PER_PHASE;
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            B0[r][st] = reinterpret_cast<const f16x8*>(fr)[(0 * KS + st) * 64 + lane];
            B1[r][st] = reinterpret_cast<const f16x8*>(fr)[(1 * KS + st) * 64 + lane];
        }
        const f16x4* tf = reinterpret_cast<const f16x4*>(fr + 2 * KS * 64 * 8);
        T0[r] = tf[lane];
        T1[r] = tf[64 + lane];
    }
    for (int i = tid; i < 2 * G2::PER_PHASE / 8; i += G::NT)
        reinterpret_cast<f16x8*>(F2)[i] = reinterpret_cast<const f16x8*>(frag2)[i];

    const int64_t nchunks = (n1 + G::CHUNK - 1) / G::CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;
    const int64_t c_last = c_end - 1;
    // the y1 history the next call needs (its last L2 - 1 samples), by the workgroup that ends
    // the stream, up front so that it overlaps the other workgroups' work
    if (c_end == nchunks) {
        for (int j = tid; j < L2 - 1; j += G::NT) hist2_out[j] = y1_direct(n1 - (L2 - 1) + j);
    }

    const int rho = lane & 15;
    const int c = rho & 1, b = rho >> 1;
    const int g = lane >> 4;
    const int phase = lane & 15;
    const int q4 = lane & 3;
    const int row_base = c * G::IM_OFF + (G::HR + wave * (G::WAVE_OUT / 16) + b) * 32;
    const int row_base2 = c * G2::IM_OFF + (G2::HR + wave * (G2::WAVE_OUT / 16) + b) * 32;
    const bool tail_owner = tid >= G::NT - G::H / 2;
    // y1 chunk position of the lane's stage-1 output oi
    auto y1_pos = [&](int oi) { return wave * G::WAVE_OUT + ((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase; };
    // prefetch index: past the workgroup's range, an empty buffer range (loads return 0 and move
    // no bytes; a re-load of the last chunk would go to HBM again, the loads are nontemporal)
    auto clamp = [&](int64_t x) { return x <= c_last ? x : nchunks; };
    auto load = [&](float4 (&v)[4], int64_t ch) {
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK_IN>(in, ch, n_in);
#pragma unroll
        for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
            for (int f = 0; f < D; ++f) v[u * D + f] = buf_load_f4(r, ((tid + G::NT * u) * D + f) * 16);
    };
    auto stash_tail = [&](float4* st, const float4 (&v)[4]) {
        if (tail_owner) {
#pragma unroll
            for (int f = 0; f < D; ++f) st[(tid - (G::NT - G::H / 2)) * D + f] = v[(G::UNITS - 1) * D + f];
        }
    };
    auto put_chunk = [&](unsigned char* buf, const float4* hsrc, const float4 (&v)[4], bool raw, int sc) {
        if (raw) {
            float4* rb = reinterpret_cast<float4*>(buf);
            if (tid < G::HP) rb[tid] = hsrc[tid];
#pragma unroll
            for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
                for (int f = 0; f < D; ++f) rb[G::HP + (tid + G::NT * u) * D + f] = v[u * D + f];
            return;
        }
        if (tid < D * (G::H / 2)) {
            const int r = tid / (G::H / 2), pi = tid % (G::H / 2);
            const int sr = r == 0 ? 0 : D - r;
            const int pa = D * (2 * pi) + sr, pb = D * (2 * pi + 1) + sr;
            const float2 a = f4_sample(hsrc[pa >> 1], pa & 1), bb = f4_sample(hsrc[pb >> 1], pb & 1);
            store_pair11<D, QH1>(buf, r, 2 * pi, a.x, bb.x, a.y, bb.y, sc);
        }
#pragma unroll
        for (int u = 0; u < G::UNITS; ++u) {
            const int i0 = 2 * (tid + G::NT * u);
#pragma unroll
            for (int r = 0; r < D; ++r) {
                const int sr = r == 0 ? 0 : D - r;
                const int la = sr, lb = D + sr;
                const float2 a = f4_sample(v[u * D + la / 2], la & 1);
                const float2 bb = f4_sample(v[u * D + lb / 2], lb & 1);
                store_pair11<D, QH1>(buf, r, G::H + i0, a.x, bb.x, a.y, bb.y, sc);
            }
        }
    };
    auto reduce = [&](const float4 (&v)[4], unsigned& m, unsigned& z) {
        float mf = 0.f;
        z = ~0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mf = __builtin_elementwise_maximum(mf, max_abs4(v[u]));
            z = min(z, min_nz1(v[u]));
        }
        m = __float_as_uint(mf);
        m = wave_max(m);
        z = wave_min(z);
    };
    auto mfma_tile = [&](const unsigned char* cur, int unscale, nf2 (&o)[2 * G::TILES]) {
        f32x4 hi[G::TILES], lo[G::TILES], hi_t[G::TILES], lo_t[G::TILES];
#pragma unroll
        for (int t = 0; t < G::TILES; ++t) {
            hi[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            lo[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            hi_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
            lo_t[t] = f32x4{ 0.f, 0.f, 0.f, 0.f };
        }
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const unsigned char* ph = cur + r * G::PH;
#pragma unroll
            for (int st = 0; st < KS; ++st) {
                const int q = 2 * st + (g >> 1);
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - q * 32 + (g & 1) * 16;
                    const f16x8 A0 = *reinterpret_cast<const f16x8*>(ph + off);
                    const f16x8 A1 = *reinterpret_cast<const f16x8*>(ph + off + G::PLANE);
                    hi[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B0[r][st], hi[t], 0, 0, 0);
                    lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, B1[r][st], lo[t], 0, 0, 0);
                    lo[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, B0[r][st], lo[t], 0, 0, 0);
                }
            }
            if constexpr (G::TAIL) {
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - (QH1 - 1) * 32 + g * 8;
                    const f16x4 A0 = *reinterpret_cast<const f16x4*>(ph + off);
                    const f16x4 A1 = *reinterpret_cast<const f16x4*>(ph + off + G::PLANE);
                    hi_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, T0[r], hi_t[t], 0, 0, 0);
                    lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, T1[r], lo_t[t], 0, 0, 0);
                    lo_t[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(A1, T0[r], lo_t[t], 0, 0, 0);
                }
            }
        }
        nf2 sum[2 * G::TILES];
#pragma unroll
        for (int t = 0; t < G::TILES; ++t)
#pragma unroll
            for (int half = 0; half < 2; ++half)
                sum[2 * t + half] = (nf2{ hi[t][2 * half], hi[t][2 * half + 1] } + nf2{ hi_t[t][2 * half], hi_t[t][2 * half + 1] }) +
                                    (nf2{ lo[t][2 * half], lo[t][2 * half + 1] } + nf2{ lo_t[t][2 * half], lo_t[t][2 * half + 1] });
        unscale_tile(sum, unscale, o);
    };
    auto direct_tile = [&](const unsigned char* cur, nf2 (&o)[2 * G::TILES]) {
        const float2* raw = reinterpret_cast<const float2*>(cur);
        for (int oi = 0; oi < 2 * G::TILES; ++oi) {
            const int j = D * G::H + D * y1_pos(oi);
            float re = 0.f, im = 0.f;
            for (int k = 0; k < L1; ++k) {
                const float2 x = raw[j - k];
                re = fmaf(taps1[k], x.x, re);
                im = fmaf(taps1[k], x.y, im);
            }
            o[oi] = nf2{ re, im };
        }
    };
    // ---- stage 2. Split of y1 chunk (registers y, its halo the raw tail hs of the chunk
    // before) into planes p2: y1 position m (phase m & 1, index m >> 1). Quad lanes q4 = 0, 1
    // write the real parts of (y1[m], y1[m + 2]), lanes 2, 3 the imaginary parts of
    // (y1[m - 2], y1[m]): one DPP exchange (quad_perm [2,3,0,1]) per sample
    auto put_chunk2 = [&](unsigned char* p2, const float2* hs, float2* hs_next, const nf2 (&y)[2 * G::TILES], bool raw,
                          int sc) {
        if (raw) {
            float2* rb = reinterpret_cast<float2*>(p2);
            if (tid < HY / 2) reinterpret_cast<float4*>(rb)[tid] = reinterpret_cast<const float4*>(hs)[tid];
#pragma unroll
            for (int oi = 0; oi < 2 * G::TILES; ++oi) rb[HY + y1_pos(oi)] = make_float2(y[oi].x, y[oi].y);
        } else {
            if (tid < G2::H / 2) { // halo samples 4t..4t+3 -> phase 0 (4t, 4t+2), phase 1 (4t+1, 4t+3)
                const float4 u = reinterpret_cast<const float4*>(hs)[2 * tid], w = reinterpret_cast<const float4*>(hs)[2 * tid + 1];
                store_pair_g<G2>(p2, 0, 2 * tid, u.x, w.x, u.y, w.y, sc);
                store_pair_g<G2>(p2, 1, 2 * tid, u.z, w.z, u.w, w.w, sc);
            }
#pragma unroll
            for (int oi = 0; oi < 2 * G::TILES; ++oi) {
                const bool lo_q = q4 < 2;
                const float send = lo_q ? y[oi].y : y[oi].x;
                const float got = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x4E, 0xf, 0xf, false));
                const float a = lo_q ? y[oi].x : got, bb = lo_q ? got : y[oi].y;
                const int m = y1_pos(oi) - (lo_q ? 0 : 2);
                const int s = G2::H + (m >> 1);
                unsigned char* ph = p2 + (m & 1) * G2::PH + (lo_q ? 0 : G2::IM_OFF);
                const int off = (s >> 4) * 32 + (s & 15) * 2;
                unsigned hi, lo;
                split_pair16(a, bb, sc, hi, lo);
                *reinterpret_cast<unsigned*>(ph + off) = hi;
                *reinterpret_cast<unsigned*>(ph + G2::PLANE + off) = lo;
            }
        }
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi) {
            const int m = y1_pos(oi) - (G::CHUNK - HY);
            if (m >= 0) hs_next[m] = make_float2(y[oi].x, y[oi].y);
        }
    };
    auto mfma_tile2 = [&](const unsigned char* p2, int unscale, nf2 (&o)[2]) {
        f32x4 hi = { 0.f, 0.f, 0.f, 0.f }, lo = { 0.f, 0.f, 0.f, 0.f };
        f32x4 hi_t = { 0.f, 0.f, 0.f, 0.f }, lo_t = { 0.f, 0.f, 0.f, 0.f };
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const unsigned char* ph = p2 + r * G2::PH;
            const _Float16* fr = F2 + r * G2::PER_PHASE;
#pragma unroll
            for (int st = 0; st < KS2; ++st) {
                const int q = 2 * st + (g >> 1);
                const int off = row_base2 - q * 32 + (g & 1) * 16;
                const f16x8 A0 = *reinterpret_cast<const f16x8*>(ph + off);
                const f16x8 A1 = *reinterpret_cast<const f16x8*>(ph + off + G2::PLANE);
                const f16x8 b0 = reinterpret_cast<const f16x8*>(fr)[(0 * KS2 + st) * 64 + lane];
                const f16x8 b1 = reinterpret_cast<const f16x8*>(fr)[(1 * KS2 + st) * 64 + lane];
                hi = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, b0, hi, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0, b1, lo, 0, 0, 0);
                lo = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1, b0, lo, 0, 0, 0);
            }
            if constexpr (G2::TAIL) {
                const int off = row_base2 - (QH2 - 1) * 32 + g * 8;
                const f16x4 A0 = *reinterpret_cast<const f16x4*>(ph + off);
                const f16x4 A1 = *reinterpret_cast<const f16x4*>(ph + off + G2::PLANE);
                const f16x4* tf = reinterpret_cast<const f16x4*>(fr + 2 * KS2 * 64 * 8);
                const f16x4 t0 = tf[lane], t1 = tf[64 + lane];
                hi_t = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, t0, hi_t, 0, 0, 0);
                lo_t = __builtin_amdgcn_mfma_f32_16x16x16f16(A0, t1, lo_t, 0, 0, 0);
                lo_t = __builtin_amdgcn_mfma_f32_16x16x16f16(A1, t0, lo_t, 0, 0, 0);
            }
        }
        nf2 sum[2];
#pragma unroll
        for (int half = 0; half < 2; ++half)
            sum[half] = (nf2{ hi[2 * half], hi[2 * half + 1] } + nf2{ hi_t[2 * half], hi_t[2 * half + 1] }) +
                        (nf2{ lo[2 * half], lo[2 * half + 1] } + nf2{ lo_t[2 * half], lo_t[2 * half + 1] });
        unscale_tile(sum, unscale, o);
    };
    auto direct_tile2 = [&](const unsigned char* p2, nf2 (&o)[2]) {
        const float2* raw = reinterpret_cast<const float2*>(p2);
        for (int half = 0; half < 2; ++half) {
            const int j = HY + 2 * (wave * G2::WAVE_OUT + (2 * g + half) * 16 + phase);
            float re = 0.f, im = 0.f;
            for (int k = 0; k < L2; ++k) {
                const float2 x = raw[j - k];
                re = fmaf(taps2[k], x.x, re);
                im = fmaf(taps2[k], x.y, im);
            }
            o[half] = nf2{ re, im };
        }
    };
    // chunks before c_begin (the first two steps' lagging stage 2) store into an empty range
    auto store_tile2 = [&](int64_t ch, const nf2 (&o)[2]) {
        const int64_t past = (n_out + G2::CHUNK - 1) / G2::CHUNK;
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G2::CHUNK>(out, ch >= c_begin ? ch : past, n_out);
#pragma unroll
        for (int half = 0; half < 2; ++half)
            buf_store_f2(r, (wave * G2::WAVE_OUT + (2 * g + half) * 16 + phase) * 8, o[half]);
    };

    // ---- prologue. Stage 1 as k_fir_mfma11's. Stage 2: y (the "chunk c_begin - 1" the first
    // step splits) holds that chunk's real tail (direct form) in the lanes that own it, zeros
    // elsewhere; its magnitude range goes to s2 slot 1 (parity of c_begin - 1)
    float4 va[4], vb[4], vc[4];
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < G::HP) {
        const int64_t gg = c_begin * G::CHUNK_IN - 2 * G::HP + 2 * tid;
        const float2 x0 = virt(in, hist1_in, gg, n_in, L1), x1 = virt(in, hist1_in, gg + 1, n_in, L1);
        hv = make_float4(x0.x, x0.y, x1.x, x1.y);
        stash[G::HP + tid] = hv;
    }
    nf2 y[2 * G::TILES];
    unsigned ym = 0, yz = ~0u;
#pragma unroll
    for (int oi = 0; oi < 2 * G::TILES; ++oi) {
        y[oi] = nf2{ 0.f, 0.f };
        if (y1_pos(oi) >= G::CHUNK - HY) {
            const float2 v = y1_direct(c_begin * G::CHUNK - G::CHUNK + y1_pos(oi));
            y[oi] = nf2{ v.x, v.y };
        }
        ym = max(ym, __float_as_uint(max_abs(y[oi].x, y[oi].y)));
        yz = min(yz, min(nz_code(y[oi].x), nz_code(y[oi].y)));
    }
    ym = wave_max(ym);
    yz = wave_min(yz);
    load(va, c_begin);
    {
        unsigned m, z;
        reduce(va, m, z);
        m = max(m, wave_max(max_mag(hv)));
        z = min(z, wave_min(min_nz1(hv)));
        if (lane == 0) {
            slot_max[wave] = m;
            slot_mnz[wave] = z;
            s2_max[4 + wave] = ym;
            s2_mnz[4 + wave] = yz;
        }
    }
    nsh::lds_barrier();
    unsigned m_prev = max(max(slot_max[0], slot_max[1]), max(slot_max[2], slot_max[3]));
    unsigned z_prev = min(min(slot_mnz[0], slot_mnz[1]), min(slot_mnz[2], slot_mnz[3]));
    int s_cur = scale_of(m_prev);
    bool ex_cur = chunk_needs_exact(m_prev, z_prev, s_cur);
    put_chunk(lds, stash + G::HP, va, ex_cur, s_cur);
    stash_tail(stash, va);
    load(va, clamp(c_begin + 1));
    load(vb, clamp(c_begin + 2));
    {
        unsigned m, z;
        reduce(va, m, z);
        nsh::lds_barrier();
        if (lane == 0) {
            slot_max[4 + wave] = m;
            slot_mnz[4 + wave] = z;
        }
    }
    nsh::lds_barrier();
    unsigned m2_prev = 0, z2_prev = ~0u; // y1 chunk before the one being split
    int s2_lag = 0;                       // chunk s-2's stage-2 scale / exact flag
    bool ex2_lag = false;

    // step for chunk ch (i = ch - c_begin): stage 1 on ch, stage-2 split of ch-1, stage-2
    // MFMA + store of ch-2
    auto step = [&](float4 (&nxt)[4], float4 (&nn)[4], float4 (&ld)[4], int64_t ch) {
        const int i = (int)(ch - c_begin);
        const int pi = i & 1, pn = pi ^ 1;
        const unsigned char* cur = lds + pi * G::BUF;
        unsigned char* nbuf = lds + pn * G::BUF;
        const unsigned m_nxt = max(max(slot_max[4 * pn], slot_max[4 * pn + 1]), max(slot_max[4 * pn + 2], slot_max[4 * pn + 3]));
        const unsigned z_nxt = min(min(slot_mnz[4 * pn], slot_mnz[4 * pn + 1]), min(slot_mnz[4 * pn + 2], slot_mnz[4 * pn + 3]));
        const unsigned m2 = max(m_prev, m_nxt);
        const int s_nxt = scale_of(m2);
        const bool ex_nxt = chunk_needs_exact(m2, min(z_prev, z_nxt), s_nxt);
        // y1 chunk ch-1 (parity pn): its range was reduced last step
        const unsigned m2c = max(max(s2_max[4 * pn], s2_max[4 * pn + 1]), max(s2_max[4 * pn + 2], s2_max[4 * pn + 3]));
        const unsigned z2c = min(min(s2_mnz[4 * pn], s2_mnz[4 * pn + 1]), min(s2_mnz[4 * pn + 2], s2_mnz[4 * pn + 3]));
        const unsigned mm = max(m2c, m2_prev);
        const int s2 = scale_of(mm);
        const bool ex2 = chunk_needs_exact(mm, min(z2c, z2_prev), s2);
        load(ld, clamp(ch + 3));
        put_chunk(nbuf, stash + pi * G::HP, nxt, ex_nxt, s_nxt);
        stash_tail(stash + pn * G::HP, nxt);
        // y1 chunk ch-1 -> planes [pn]; halo = raw tail of ch-2 (stash [pi]); its tail -> [pn]
        put_chunk2(lds + C::P2 + pn * G2::BUF, st2 + pi * HY, st2 + pn * HY, y, ex2, s2);
        if (ex_cur)
            direct_tile(cur, y);
        else
            mfma_tile(cur, -(s_cur + sh1), y);
        nf2 o2[2];
        if (ex2_lag)
            direct_tile2(lds + C::P2 + pi * G2::BUF, o2);
        else
            mfma_tile2(lds + C::P2 + pi * G2::BUF, -(s2_lag + sh2), o2);
        store_tile2(ch - 2, o2);
        unsigned ymx = 0, yzn = ~0u;
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi) {
            ymx = max(ymx, __float_as_uint(max_abs(y[oi].x, y[oi].y)));
            yzn = min(yzn, min(nz_code(y[oi].x), nz_code(y[oi].y)));
        }
        ymx = wave_max(ymx);
        yzn = wave_min(yzn);
        unsigned m, z;
        reduce(nn, m, z);
        if (lane == 0) {
            slot_max[4 * pi + wave] = m;
            slot_mnz[4 * pi + wave] = z;
            s2_max[4 * pi + wave] = ymx;
            s2_mnz[4 * pi + wave] = yzn;
        }
        m_prev = m_nxt;
        z_prev = z_nxt;
        ex_cur = ex_nxt;
        s_cur = s_nxt;
        m2_prev = m2c;
        z2_prev = z2c;
        s2_lag = s2;
        ex2_lag = ex2;
        nsh::lds_barrier();
    };
    const int64_t s_last = c_last + 2;
    int64_t ch = c_begin;
    for (; ch + 2 <= s_last; ch += 3) {
        step(va, vb, vc, ch);
        step(vb, vc, va, ch + 1);
        step(vc, va, vb, ch + 2);
    }
    if (ch <= s_last) step(va, vb, vc, ch++);
    if (ch <= s_last) step(vb, vc, va, ch);
}

template <int QH1, int QH2>
int launch_casc2(const nsh_fir_plan* p1, const nsh_fir_plan* p2, const float2* in, const float2* h1i, float2* h1o,
                 const float2* h2i, float2* h2o, float2* out, int64_t n_out, hipStream_t s)
{
    using C = geomcasc<QH1, QH2>;
    NSH_CK(set_lds_attr((const void*)k_fir_casc2<QH1, QH2>, C::LDS, p1->dev));
    const int64_t nchunks = (2 * n_out + 1023) / 1024;
    const int n_cu = plan_cus(p1);
    const int64_t max_grid = (int64_t)n_cu * 2;
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    hipLaunchKernelGGL((k_fir_casc2<QH1, QH2>), dim3(grid), dim3(256), C::LDS, s, in, h1i, h1o, h2i, h2o, out,
                       (const _Float16*)p1->fragd8_dev, (const float*)p1->taps_dev, p1->L, p1->sh8,
                       (const _Float16*)p2->fragd8_dev, (const float*)p2->taps_dev, p2->L, p2->sh8, n_out);
    NSH_CK_LAUNCH("nsh_fir_cascade2_ccf");
    return 0;
}

template <int QH1>
int casc2_qh2(const nsh_fir_plan* p1, const nsh_fir_plan* p2, const float2* in, const float2* h1i, float2* h1o,
              const float2* h2i, float2* h2o, float2* out, int64_t n_out, hipStream_t s)
{
    switch (p2->QHD) {
    case 3: return launch_casc2<QH1, 3>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 4: return launch_casc2<QH1, 4>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 5: return launch_casc2<QH1, 5>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 6: return launch_casc2<QH1, 6>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_cascade2_ccf: unsupported stage-2 tap count");
    }
}

// Host-side bf16 round-to-nearest-even (taps are finite).
unsigned short bf16_rne(float f)
{
    unsigned u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}
float bf16_to_f(unsigned short b)
{
    const unsigned u = (unsigned)b << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}


template <int Q, int DEPTH>
int launch_v2(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
              hipStream_t s, int wg_per_cu)
{
    using G = geom2<Q>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma2<Q, DEPTH>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int64_t max_grid = (int64_t)n_cu * wg_per_cu;
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    const int aligned = ((uintptr_t)in % 16 == 0) ? 1 : 0;
    hipLaunchKernelGGL((k_fir_mfma2<Q, DEPTH>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const bf16x8*)p->frag_dev, p->L, n_out, aligned);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma2)");
    return 0;
}


template <int Q>
int launch_v9(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
              hipStream_t s)
{
    using G = geom8<Q>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma9<Q>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    // Workgroups over the whole launch (2 resident per CU at a time): 16 chunks each from 2^26
    // samples on (at most 32 per CU), else about 32 chunks each (2..16 per CU). Long streams then
    // walk in shorter contiguous ranges, which keeps the window of addresses in flight compact:
    // at 2^28 samples 16 per CU ran 807 us vs 855 with 2; after the step's VALU cuts, 32 per CU
    // (16 chunks) 773 vs 779 us, and 16 chunks per workgroup also wins at 2^26 and 2^27, while
    // 2^25 keeps 2 per CU (tools/fir_variants.py VARIANTS=0:g, same process).
    int64_t max_grid = (int64_t)n_cu * 2;
    if (p->wg_per_cu > 0)
        max_grid = (int64_t)n_cu * p->wg_per_cu; // NSH_FIR_WG_PER_CU (A/B)
    else if (nchunks / 16 >= (int64_t)n_cu * 8) // >= 2^26 samples: 16 chunks per workgroup
        max_grid = std::min<int64_t>(nchunks / 16, (int64_t)n_cu * 32);
    else if (nchunks / 32 > max_grid)
        max_grid = std::min<int64_t>(nchunks / 32, (int64_t)n_cu * 16);
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    hipLaunchKernelGGL((k_fir_mfma9<Q>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const f16x8*)p->frag8_dev, (const float*)p->taps_dev, p->L, p->sh8, n_out);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma fp16x2 v9)");
    return 0;
}


template <int Q>
int launch_v12(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geom12<Q>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma12<Q>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per_x = (nchunks + 7) / 8; // workgroups (= chunks) per XCD
    const int64_t grid = per_x * 8;
    if (grid > 0x7fffffff) return nsh::fail_msg("nsh_fir_ccf(mfma v12): stream too long for one launch");
    hipLaunchKernelGGL((k_fir_mfma12<Q>), dim3((unsigned)grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const uint4*)p->frag12_dev, (const float*)p->taps_dev, p->L, p->sh8, n_out, per_x);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma fp16x2 v12)");
    return 0;
}

// Tuning variants (selected by NSH_FIR_MFMA_VARIANT for A/B runs; default = measured best).
template <int Q>
int launch_q(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out, hipStream_t s)
{
    if (p->frag12_dev && !p->force_x3 && (p->variant == 0 || p->variant == 12))
        return launch_v12<Q>(p, in, hin, hout, out, n_out, s); // default
    if (p->frag8_dev && !p->force_x3 && p->variant != 6 && p->variant != 7)
        return launch_v9<Q>(p, in, hin, hout, out, n_out, s);
    switch (p->variant) {
    case 6: return launch_v2<Q, 1>(p, in, hin, hout, out, n_out, s, 2);
    case 7: return launch_v2<Q, 2>(p, in, hin, hout, out, n_out, s, 2);
    default: return launch_v2<Q, 2>(p, in, hin, hout, out, n_out, s, 2);
    }
}

} // namespace

namespace {
int decim_qh(const nsh_fir_plan* p) { return ((p->L + p->D - 1) / p->D + 1 + 15 + 15) / 16; }
bool finite_taps(const nsh_fir_plan* p)
{
    for (float t : p->taps_host)
        if (!(t == t) || t - t != 0.f) return false;
    return true;
}
} // namespace

bool nsh_fir_mfma_supported(const nsh_fir_plan* p)
{
    if (!finite_taps(p)) return false;
    if (p->D == 2 || p->D == 4) return decim_qh(p) <= 6;
    if (p->D != 1) return false;
    const int Q = (p->L + 30) / 32 + 1;
    return Q <= QMAX;
}

int nsh_fir_mfma_prepare_decim(nsh_fir_plan* p)
{
    // polyphase taps h'_0[j] = h[D j], h'_r[j] = h[D (j - 1) + r] (r >= 1, j >= 1), laid out
    // per phase as the 16-sample form's fragments (see k_fir_mfma7)
    const int D = p->D, QH = decim_qh(p), KS = QH / 2;
    const bool tail = QH % 2;
    p->QHD = QH;
    const size_t per_phase = (size_t)3 * KS * 64 * 8 + (tail ? (size_t)3 * 64 * 4 : 0);
    std::vector<unsigned short> f((size_t)D * per_phase, 0);
    auto tap = [&](int r, int j) -> float {
        const int k = r == 0 ? D * j : (j >= 1 ? D * (j - 1) + r : -1);
        return (k >= 0 && k < p->L) ? p->taps_host[k] : 0.f;
    };
    auto put3 = [&](float hv, size_t i0, size_t i1, size_t i2) {
        const unsigned short h1 = bf16_rne(hv);
        const float r1 = hv - bf16_to_f(h1);
        const unsigned short h2 = bf16_rne(r1);
        f[i0] = h1;
        f[i1] = h2;
        f[i2] = bf16_rne(r1 - bf16_to_f(h2));
    };
    for (int r = 0; r < D; ++r) {
        const size_t base = (size_t)r * per_phase;
        for (int st = 0; st < KS; ++st)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 8; ++j) {
                    const int kk = 8 * (lane >> 4) + j;
                    const float hv = tap(r, (lane & 15) - (kk & 15) + 16 * (2 * st + (kk >> 4)));
                    put3(hv, base + (((size_t)0 * KS + st) * 64 + lane) * 8 + j, base + (((size_t)1 * KS + st) * 64 + lane) * 8 + j,
                         base + (((size_t)2 * KS + st) * 64 + lane) * 8 + j);
                }
        if (tail) {
            const size_t t0 = base + (size_t)3 * KS * 64 * 8;
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 4; ++j) {
                    const float hv = tap(r, (lane & 15) - (4 * (lane >> 4) + j) + 16 * (QH - 1));
                    put3(hv, t0 + ((size_t)0 * 64 + lane) * 4 + j, t0 + ((size_t)1 * 64 + lane) * 4 + j,
                         t0 + ((size_t)2 * 64 + lane) * 4 + j);
                }
        }
    }
    NSH_CK(hipMalloc(&p->fragd_dev, f.size() * sizeof(unsigned short)));
    NSH_CK(hipMemcpy(p->fragd_dev, f.data(), f.size() * sizeof(unsigned short), hipMemcpyHostToDevice));

    // k_fir_mfma11: the same polyphase taps scaled by 2^sh8 (max |h| * 2^sh8 in [2^14, 2^15),
    // as for decim 1) and split into two fp16 terms; per phase [2][KS][64] x8 then [2][64] x4
    {
        unsigned maxbits = 0;
        for (float t : p->taps_host) {
            unsigned u;
            std::memcpy(&u, &t, 4);
            maxbits = std::max(maxbits, u & 0x7fffffffu);
        }
        const int sh = 141 - (int)(maxbits >> 23);
        p->sh8 = sh;
        const size_t pp = (size_t)2 * KS * 64 * 8 + (size_t)2 * 64 * 4;
        std::vector<_Float16> f8((size_t)D * pp, (_Float16)0.f);
        auto put2 = [&](float hv, size_t i0, size_t i1) {
            const float hs = std::ldexp(hv, sh);
            const _Float16 h0 = (_Float16)hs;
            f8[i0] = h0;
            f8[i1] = (_Float16)(hs - (float)h0);
        };
        for (int r = 0; r < D; ++r) {
            const size_t base = (size_t)r * pp;
            for (int st = 0; st < KS; ++st)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const int kk = 8 * (lane >> 4) + j;
                        put2(tap(r, (lane & 15) - (kk & 15) + 16 * (2 * st + (kk >> 4))),
                             base + (((size_t)0 * KS + st) * 64 + lane) * 8 + j, base + (((size_t)1 * KS + st) * 64 + lane) * 8 + j);
                    }
            if (tail) {
                const size_t t0 = base + (size_t)2 * KS * 64 * 8;
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 4; ++j)
                        put2(tap(r, (lane & 15) - (4 * (lane >> 4) + j) + 16 * (QH - 1)), t0 + (size_t)lane * 4 + j,
                             t0 + (size_t)(64 + lane) * 4 + j);
            }
        }
        NSH_CK(hipMalloc(&p->fragd8_dev, f8.size() * sizeof(_Float16)));
        NSH_CK(hipMemcpy(p->fragd8_dev, f8.data(), f8.size() * sizeof(_Float16), hipMemcpyHostToDevice));
    }
    return 0;
}

int nsh_fir_mfma_prepare(nsh_fir_plan* p)
{
    if (const char* v = std::getenv("NSH_FIR_MFMA_VARIANT")) p->variant = std::atoi(v);
    if (const char* v = std::getenv("NSH_FIR_WG_PER_CU")) { // A/B only
        const int w = std::atoi(v);
        if (w >= 1 && w <= 64) p->wg_per_cu = w;
    }
    if (p->D > 1) return nsh_fir_mfma_prepare_decim(p);
    const int Q = (p->L + 30) / 32 + 1;
    const int S = 2 * Q;
    p->Q = Q;
    p->S = S;
    std::vector<unsigned short> frag((size_t)3 * S * 64 * 8, 0);
    for (int st = 0; st < S; ++st)
        for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
                const int i = lane & 31;
                const int r = 16 * (st & 1) + 8 * (lane >> 5) + j;
                const int q = st >> 1;
                const int t = i - r + 32 * q;
                const float hv = (t >= 0 && t < p->L) ? p->taps_host[t] : 0.f;
                const unsigned short h1 = bf16_rne(hv);
                const float r1 = hv - bf16_to_f(h1);
                const unsigned short h2 = bf16_rne(r1);
                const float r2 = r1 - bf16_to_f(h2);
                const unsigned short h3 = bf16_rne(r2);
                frag[(((size_t)0 * S + st) * 64 + lane) * 8 + j] = h1;
                frag[(((size_t)1 * S + st) * 64 + lane) * 8 + j] = h2;
                frag[(((size_t)2 * S + st) * 64 + lane) * 8 + j] = h3;
            }
    NSH_CK(hipMalloc(&p->frag_dev, frag.size() * sizeof(unsigned short)));
    NSH_CK(hipMemcpy(p->frag_dev, frag.data(), frag.size() * sizeof(unsigned short), hipMemcpyHostToDevice));

    // fp16x2 (k_fir_mfma9): taps scaled by 2^sh8 (max |h| * 2^sh8 in [2^14, 2^15)), split into two fp16 terms
    // (RNE), same lane order as v2. A tap far below the largest (e.g. firwin's ~1e-18 taps
    // at the sinc zeros) lands in fp16's subnormal range or flushes: it is then exact to
    // 2^-39 of the largest tap, which moves an output by at most 2^-39 max|h| sum|x|, far
    // below fp32's own rounding of the sum. So every finite tap set qualifies.
    {
        unsigned maxbits = 0;
        for (float t : p->taps_host) {
            unsigned u;
            std::memcpy(&u, &t, 4);
            maxbits = std::max(maxbits, u & 0x7fffffffu);
        }
        const int sh = 141 - (int)(maxbits >> 23);
        {
            std::vector<_Float16> f8((size_t)2 * S * 64 * 8, (_Float16)0.f);
            for (int st = 0; st < S; ++st)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const int i = lane & 31;
                        const int r = 16 * (st & 1) + 8 * (lane >> 5) + j;
                        const int t = i - r + 32 * (st >> 1);
                        const float hs = (t >= 0 && t < p->L) ? std::ldexp(p->taps_host[t], sh) : 0.f;
                        const _Float16 h0 = (_Float16)hs;
                        const _Float16 h1 = (_Float16)(hs - (float)h0);
                        f8[(((size_t)0 * S + st) * 64 + lane) * 8 + j] = h0;
                        f8[(((size_t)1 * S + st) * 64 + lane) * 8 + j] = h1;
                    }
            p->sh8 = sh;
            // v12 tap image: R[m] = h[32Q - 1 - m] (scaled, hi/lo fp16), copy k holds R[k .. k + TW)
            const int TW = v12_tw(Q), NCP = NSH_V12_COPIES;
            std::vector<_Float16> f12((size_t)2 * NCP * TW, (_Float16)0.f);
            for (int k = 0; k < NCP; ++k)
                for (int e = 0; e < TW; ++e) {
                    const int t = 32 * Q - 1 - (e + k);
                    const float hs = (t >= 0 && t < p->L) ? std::ldexp(p->taps_host[t], sh) : 0.f;
                    const _Float16 h0 = (_Float16)hs;
                    f12[(size_t)(0 * NCP + k) * TW + e] = h0;
                    f12[(size_t)(1 * NCP + k) * TW + e] = (_Float16)(hs - (float)h0);
                }
            NSH_CK(hipMalloc(&p->frag12_dev, f12.size() * sizeof(_Float16)));
            NSH_CK(hipMemcpy(p->frag12_dev, f12.data(), f12.size() * sizeof(_Float16), hipMemcpyHostToDevice));
            NSH_CK(hipMalloc(&p->frag8_dev, f8.size() * sizeof(_Float16)));
            NSH_CK(hipMemcpy(p->frag8_dev, f8.data(), f8.size() * sizeof(_Float16), hipMemcpyHostToDevice));
        }
    }

    // v5: QH/2 k-steps of 32 for v_mfma_f32_16x16x32_bf16 (lane l holds B[k = 8(l >> 4) + j]
    // [col = l & 15], k = 32 st + kk -> q = 2 st + (kk >> 4), r = kk & 15), then for odd QH a
    // tail for v_mfma_f32_16x16x16_bf16 (q = QH - 1, lane l holds B[r = 4(l >> 4) + j][l & 15]).
    // Tap index i - r + 16 q; each tap split into three bf16 terms (RNE).
    p->QH = (p->L + 15 + 15) / 16;
    if (p->QH <= 10) {
        const int KS = p->QH / 2;
        const bool tail = p->QH % 2;
        std::vector<unsigned short> f16((size_t)3 * KS * 64 * 8 + (tail ? (size_t)3 * 64 * 4 : 0), 0);
        auto put3 = [&](float hv, size_t i0, size_t i1, size_t i2) {
            const unsigned short h1 = bf16_rne(hv);
            const float r1 = hv - bf16_to_f(h1);
            const unsigned short h2 = bf16_rne(r1);
            const float r2 = r1 - bf16_to_f(h2);
            f16[i0] = h1;
            f16[i1] = h2;
            f16[i2] = bf16_rne(r2);
        };
        auto tap = [&](int t) { return (t >= 0 && t < p->L) ? p->taps_host[t] : 0.f; };
        for (int st = 0; st < KS; ++st)
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 8; ++j) {
                    const int kk = 8 * (lane >> 4) + j;
                    const float hv = tap((lane & 15) - (kk & 15) + 16 * (2 * st + (kk >> 4)));
                    put3(hv, (((size_t)0 * KS + st) * 64 + lane) * 8 + j, (((size_t)1 * KS + st) * 64 + lane) * 8 + j,
                         (((size_t)2 * KS + st) * 64 + lane) * 8 + j);
                }
        if (tail) {
            const size_t t0 = (size_t)3 * KS * 64 * 8;
            for (int lane = 0; lane < 64; ++lane)
                for (int j = 0; j < 4; ++j) {
                    const int r = 4 * (lane >> 4) + j;
                    const float hv = tap((lane & 15) - r + 16 * (p->QH - 1));
                    put3(hv, t0 + ((size_t)0 * 64 + lane) * 4 + j, t0 + ((size_t)1 * 64 + lane) * 4 + j,
                         t0 + ((size_t)2 * 64 + lane) * 4 + j);
                }
        }
        NSH_CK(hipMalloc(&p->frag16_dev, f16.size() * sizeof(unsigned short)));
        NSH_CK(hipMemcpy(p->frag16_dev, f16.data(), f16.size() * sizeof(unsigned short), hipMemcpyHostToDevice));
    }
    return 0;
}

std::string nsh_fir_mfma_kernel_name(const nsh_fir_plan* p)
{
    auto t = [](const char* k, int a, int b = -1) {
        return std::string(k) + "<" + std::to_string(a) + (b >= 0 ? "," + std::to_string(b) : std::string()) + ">";
    };
    if (p->algo == NSH_FIR_MFMA16) return t("k_fir_mfma5", p->QH, p->variant == 20 ? 2 : 1);
    if (p->D > 1) return t(p->fragd8_dev && p->variant != 7 ? "k_fir_mfma11" : "k_fir_mfma7", p->D, p->QHD);
    if (p->frag12_dev && !p->force_x3 && (p->variant == 0 || p->variant == 12)) return t("k_fir_mfma12", p->Q);
    if (p->frag8_dev && !p->force_x3 && p->variant != 6 && p->variant != 7) return t("k_fir_mfma9", p->Q);
    if (p->variant >= 20) return t("k_fir_mfma5", p->QH, p->variant == 20 ? 2 : 1);
    return t("k_fir_mfma2", p->Q, p->variant == 6 ? 1 : 2);
}

bool nsh_fir_mfma16_supported(const nsh_fir_plan* p)
{
    if (p->D != 1) return false;
    for (float t : p->taps_host)
        if (!(t == t) || t - t != 0.f) return false;
    return (p->L + 30) / 16 <= 10;
}

int nsh_fir_mfma16_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                       int64_t n_out, hipStream_t s)
{
    if (p->frag16_dev) {
        switch (p->QH) {
        case 1: return launch_qh<1>(p, in, hist_in, hist_out, out, n_out, s);
        case 2: return launch_qh<2>(p, in, hist_in, hist_out, out, n_out, s);
        case 3: return launch_qh<3>(p, in, hist_in, hist_out, out, n_out, s);
        case 4: return launch_qh<4>(p, in, hist_in, hist_out, out, n_out, s);
        case 5: return launch_qh<5>(p, in, hist_in, hist_out, out, n_out, s);
        case 6: return launch_qh<6>(p, in, hist_in, hist_out, out, n_out, s);
        case 7: return launch_qh<7>(p, in, hist_in, hist_out, out, n_out, s);
        case 8: return launch_qh<8>(p, in, hist_in, hist_out, out, n_out, s);
        case 9: return launch_qh<9>(p, in, hist_in, hist_out, out, n_out, s);
        case 10: return launch_qh<10>(p, in, hist_in, hist_out, out, n_out, s);
        default: break;
        }
    }
    return nsh::fail_msg("nsh_fir_ccf(mfma16): unsupported tap count");
}

int nsh_fir_mfma_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out, int64_t n_out, hipStream_t s)
{
    if (p->D == 2) return launch_dec<2>(p, in, hist_in, hist_out, out, n_out, s);
    if (p->D == 4) return launch_dec<4>(p, in, hist_in, hist_out, out, n_out, s);
    if (p->variant >= 20) return nsh_fir_mfma16_run(p, in, hist_in, hist_out, out, n_out, s); // A/B tuning
    switch (p->Q) {
    case 1: return launch_q<1>(p, in, hist_in, hist_out, out, n_out, s);
    case 2: return launch_q<2>(p, in, hist_in, hist_out, out, n_out, s);
    case 3: return launch_q<3>(p, in, hist_in, hist_out, out, n_out, s);
    case 4: return launch_q<4>(p, in, hist_in, hist_out, out, n_out, s);
    case 5: return launch_q<5>(p, in, hist_in, hist_out, out, n_out, s);
    case 6: return launch_q<6>(p, in, hist_in, hist_out, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma): unsupported tap count");
    }
}

bool nsh_fir_cascade2_ok(const nsh_fir_plan* p1, const nsh_fir_plan* p2)
{
    auto ok = [](const nsh_fir_plan* p) {
        return p && p->D == 2 && (p->algo == NSH_FIR_MFMA) && p->fragd8_dev && p->variant != 7 && p->QHD >= 3 &&
               p->QHD <= 6;
    };
    return ok(p1) && ok(p2) && p1->dev == p2->dev;
}

int nsh_fir_cascade2_run(const nsh_fir_plan* p1, const nsh_fir_plan* p2, const float2* in, const float2* h1i, float2* h1o,
                         const float2* h2i, float2* h2o, float2* out, int64_t n_out, hipStream_t s)
{
    switch (p1->QHD) {
    case 3: return casc2_qh2<3>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 4: return casc2_qh2<4>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 5: return casc2_qh2<5>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    case 6: return casc2_qh2<6>(p1, p2, in, h1i, h1o, h2i, h2o, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_cascade2_ccf: unsupported stage-1 tap count");
    }
}
