// libnsh_hip.so, legacy build only (`make LEGACY=1`): the FIR matrix-core forms that the product
// kernels (nsh_fir_mfma.hip: k_fir_mfma12, k_fir_mfma11) superseded, kept for A/B runs and their
// parity tests (pytest marker `legacy`, skipped when nsh_fir_legacy_available() is 0):
//   k_fir_mfma2  bf16x3 split, six products (NSH_FIR_MFMA_BF16X3; NSH_FIR_MFMA_VARIANT 6 / 7)
//   k_fir_mfma5  16-sample blocks on v_mfma_f32_16x16x32_bf16 (NSH_FIR_MFMA16; variant >= 20)
//   k_fir_mfma7  bf16x3 polyphase decimator (decim 2 / 4, variant 7)
//   k_fir_mfma9  v12's predecessor: contiguous per-workgroup chunk ranges, taps in VGPRs (variant 9)
//   k_fir_casc2  two decimate-by-2 FIRs in one pass (nsh_fir_cascade2_ccf)
// and the timing-only ablation hooks (NSH_FIR_ABLATE) of tools/probe/fir_ablate.sh. Their
// measurements are in DESIGN.md section 4. The strong definitions here replace the weak stubs of
// nsh_fir_mfma.hip.
#include "../nsh_fir_mfma_shared.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

// Ablation hooks for tools/probe/fir_ablate.sh only (bit mask; 0 in every product build):
// 1 = no MFMA, 2 = no global loads, 4 = no bf16 split, 8 = no global stores; timing-only
// (wrong results): 16 = half the MFMAs, 32 = int8 MFMA instruction count, 64 = the same
// FLOPs as 16x16x32 MFMAs, 128 = A fragments read once and reused.
#ifndef NSH_FIR_ABLATE
#define NSH_FIR_ABLATE 0
#endif

namespace {

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


// Tuning variants (selected by NSH_FIR_MFMA_VARIANT for A/B runs; default = measured best).
template <int Q>
int launch_q_legacy(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out, hipStream_t s)
{
    if (p->frag8_dev && !p->force_x3 && p->variant != 6 && p->variant != 7)
        return launch_v9<Q>(p, in, hin, hout, out, n_out, s);
    switch (p->variant) {
    case 6: return launch_v2<Q, 1>(p, in, hin, hout, out, n_out, s, 2);
    case 7: return launch_v2<Q, 2>(p, in, hin, hout, out, n_out, s, 2);
    default: return launch_v2<Q, 2>(p, in, hin, hout, out, n_out, s, 2);
    }
}

int legacy_prepare_decim(nsh_fir_plan* p)
{
    // polyphase taps h'_0[j] = h[D j], h'_r[j] = h[D (j - 1) + r] (r >= 1, j >= 1), laid out
    // per phase as the 16-sample form's fragments (see k_fir_mfma7)
    const int D = p->D, QH = decim_qh(p), KS = QH / 2;
    const bool tail = QH % 2;
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
    return 0;
}


int legacy_prepare_dec1(nsh_fir_plan* p)
{
    const int S = p->S;
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


} // namespace

bool nsh_fir_legacy_built() { return true; }

int nsh_fir_legacy_prepare(nsh_fir_plan* p)
{
    return p->D > 1 ? legacy_prepare_decim(p) : legacy_prepare_dec1(p);
}

std::string nsh_fir_legacy_kernel_name(const nsh_fir_plan* p)
{
    auto t = [](const char* k, int a, int b = -1) {
        return std::string(k) + "<" + std::to_string(a) + (b >= 0 ? "," + std::to_string(b) : std::string()) + ">";
    };
    if (p->algo == NSH_FIR_MFMA16 || p->variant >= 20) return t("k_fir_mfma5", p->QH, p->variant == 20 ? 2 : 1);
    if (p->D > 1) return t("k_fir_mfma7", p->D, p->QHD);
    if (p->frag8_dev && !p->force_x3 && p->variant != 6 && p->variant != 7) return t("k_fir_mfma9", p->Q);
    return t("k_fir_mfma2", p->Q, p->variant == 6 ? 1 : 2);
}

int nsh_fir_legacy_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out,
                       int64_t n_out, hipStream_t s)
{
    if (p->algo == NSH_FIR_MFMA16 || p->variant >= 20) return nsh_fir_mfma16_run(p, in, hist_in, hist_out, out, n_out, s);
    if (p->D == 2 || p->D == 4) {
        switch (p->QHD * 8 + p->D) {
        case 2 * 8 + 2: return launch_v7<2, 2>(p, in, hist_in, hist_out, out, n_out, s);
        case 3 * 8 + 2: return launch_v7<2, 3>(p, in, hist_in, hist_out, out, n_out, s);
        case 4 * 8 + 2: return launch_v7<2, 4>(p, in, hist_in, hist_out, out, n_out, s);
        case 5 * 8 + 2: return launch_v7<2, 5>(p, in, hist_in, hist_out, out, n_out, s);
        case 6 * 8 + 2: return launch_v7<2, 6>(p, in, hist_in, hist_out, out, n_out, s);
        case 2 * 8 + 4: return launch_v7<4, 2>(p, in, hist_in, hist_out, out, n_out, s);
        case 3 * 8 + 4: return launch_v7<4, 3>(p, in, hist_in, hist_out, out, n_out, s);
        case 4 * 8 + 4: return launch_v7<4, 4>(p, in, hist_in, hist_out, out, n_out, s);
        case 5 * 8 + 4: return launch_v7<4, 5>(p, in, hist_in, hist_out, out, n_out, s);
        case 6 * 8 + 4: return launch_v7<4, 6>(p, in, hist_in, hist_out, out, n_out, s);
        default: return nsh::fail_msg("nsh_fir_ccf(mfma7): unsupported tap count");
        }
    }
    switch (p->Q) {
    case 1: return launch_q_legacy<1>(p, in, hist_in, hist_out, out, n_out, s);
    case 2: return launch_q_legacy<2>(p, in, hist_in, hist_out, out, n_out, s);
    case 3: return launch_q_legacy<3>(p, in, hist_in, hist_out, out, n_out, s);
    case 4: return launch_q_legacy<4>(p, in, hist_in, hist_out, out, n_out, s);
    case 5: return launch_q_legacy<5>(p, in, hist_in, hist_out, out, n_out, s);
    case 6: return launch_q_legacy<6>(p, in, hist_in, hist_out, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma legacy): unsupported tap count");
    }
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
