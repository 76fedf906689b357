// libnsh_hip.so: fir_filter_ccf as a Toeplitz GEMM on the bf16 matrix cores (decim 1).
//
// Blocked form. Split the output stream into 32-sample blocks; output n = 32*beta + i:
//     y[32 beta + i] = sum_{q<Q} sum_{r<32} h[i - r + 32 q] * x[32 (beta - q) + r]
// i.e. C[rho][i] = sum_k A[rho][k] B[k][i] with k = 32 q + r (K = 32 Q),
//     A[rho][k] = x_c[32 (beta - q) + r]    rho = (block beta, component c)  -- the stream
//     B[k][i]   = h[i - r + 32 q]           (zero outside [0, L))           -- the taps
// One v_mfma_f32_32x32x16_bf16 covers 32 rows (16 blocks x {re, im}) x 32 phases x 16 k;
// a wave owns a 512-sample tile and runs 2Q k-steps. Q = 5 for L = 127 (K = 160: 26 %
// zero padding, irrelevant because the kernel is HBM-bound with ~2x matrix-core slack).
//
// Precision: fp32 emulated by a 3-term bf16 split of both operands (x = x1 + x2 + x3 and
// h = h1 + h2 + h3, each split exact for finite normal fp32) and the six products with
// term-order sum <= 4 (x1h1 | x1h2 x2h1 x1h3 x2h2 x3h1), accumulated in fp32 by the MFMA;
// the leading product and the correction terms use separate accumulators. Dropped terms
// are < 2^-24 relative; measured error is at the fp32 direct-form level (tests/).
// bf16 keeps the fp32 exponent range, so no input scaling is needed. Non-finite inputs
// are not supported by this form (use NSH_FIR_DIRECT).
//
// Data movement: a 256-thread workgroup walks a contiguous range of 2048-output chunks.
// Each chunk's 2048 + 32(Q-1) input samples are loaded with 16-byte global loads into
// registers one chunk ahead (overlapping the MFMAs of the current chunk), split, and
// written as six bf16 planes (re/im x 3 terms) to LDS, with every 32-sample row padded to
// 80 B so the per-lane ds_read_b128 A-fragment reads are bank-conflict free (lanes of one
// 16-lane group read 16 distinct 16-B slots: 5*beta mod 16 is a bijection). The taps'
// B fragments (3 terms x 2Q k-steps, prepared on the host in lane order) stay in VGPRs for
// the whole launch. Outputs leave the accumulators as (re, im) float2 pairs: lanes 0-31
// of a store cover 32 consecutive samples (256 contiguous bytes).
#include "nsh_common.hpp"

#include <cstring>
#include <vector>

#include "nsh_fir_plan.hpp"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef float nf2 __attribute__((ext_vector_type(2)));

constexpr int NT = 256;     // threads per workgroup (4 waves)
constexpr int TILE = 512;   // outputs per wave per chunk
constexpr int CHUNK = 2048; // outputs per workgroup per chunk
constexpr int QMAX = 6;     // L <= 161

template <int Q>
struct geom {
    static constexpr int S = 2 * Q;                           // k-steps of 16
    static constexpr int H = 32 * (Q - 1);                    // halo samples
    static constexpr int NS = CHUNK + H;                      // staged samples per chunk
    static constexpr int NB = NS / 32;                        // staged 32-sample rows
    static constexpr int PLANE = (NB * 80 + 255) / 256 * 256; // bytes per bf16 plane
    static constexpr int LDS = 6 * PLANE;
    static constexpr int NV = NS / 2;                         // 16-byte vectors per chunk
    static constexpr int VPT = (NV + NT - 1) / NT;            // vectors per thread
};

__device__ __forceinline__ void split3(float x, __bf16& t1, __bf16& t2, __bf16& t3)
{
    t1 = (__bf16)x;
    const float r1 = x - (float)t1; // exact
    t2 = (__bf16)r1;
    const float r2 = r1 - (float)t2; // exact
    t3 = (__bf16)r2;                 // exact for finite normal x
}

__device__ __forceinline__ unsigned pack2(__bf16 a, __bf16 b)
{
    return (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
}

__device__ __forceinline__ float2 virt(const float2* __restrict__ in, const float2* __restrict__ hist, int64_t g, int64_t n_in, int L)
{
    if (g >= 0) return g < n_in ? in[g] : make_float2(0.f, 0.f);
    if (g >= -(int64_t)(L - 1)) return hist[g + (L - 1)];
    return make_float2(0.f, 0.f);
}

template <int Q>
__device__ __forceinline__ void stage_load(float4 (&v)[geom<Q>::VPT],
                                           const float2* __restrict__ in,
                                           const float2* __restrict__ hist,
                                           int64_t chunk,
                                           int64_t n_in,
                                           int L,
                                           bool in_aligned)
{
    using G = geom<Q>;
    const int64_t g0 = chunk * CHUNK - G::H;
    const bool interior = in_aligned && g0 >= 0 && g0 + G::NS <= n_in;
    if (interior) {
        const float4* src = reinterpret_cast<const float4*>(in + g0);
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const int vi = threadIdx.x + NT * u;
            if (G::NV % NT == 0 || vi < G::NV) {
                const nf4 t = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(src + vi));
                v[u] = make_float4(t.x, t.y, t.z, t.w);
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < G::VPT; ++u) {
            const int vi = threadIdx.x + NT * u;
            if (G::NV % NT == 0 || vi < G::NV) {
                const float2 a = virt(in, hist, g0 + 2 * vi, n_in, L);
                const float2 b = virt(in, hist, g0 + 2 * vi + 1, n_in, L);
                v[u] = make_float4(a.x, a.y, b.x, b.y);
            }
        }
    }
}

template <int Q>
__device__ __forceinline__ void stage_store(const float4 (&v)[geom<Q>::VPT], unsigned char* lds)
{
    using G = geom<Q>;
#pragma unroll
    for (int u = 0; u < G::VPT; ++u) {
        const int vi = threadIdx.x + NT * u;
        if (G::NV % NT == 0 || vi < G::NV) {
            const int s = 2 * vi; // even local sample
            const int off = (s >> 5) * 80 + (s & 31) * 2;
            __bf16 r1a, r2a, r3a, i1a, i2a, i3a, r1b, r2b, r3b, i1b, i2b, i3b;
            split3(v[u].x, r1a, r2a, r3a);
            split3(v[u].y, i1a, i2a, i3a);
            split3(v[u].z, r1b, r2b, r3b);
            split3(v[u].w, i1b, i2b, i3b);
            *reinterpret_cast<unsigned*>(lds + 0 * G::PLANE + off) = pack2(r1a, r1b);
            *reinterpret_cast<unsigned*>(lds + 1 * G::PLANE + off) = pack2(r2a, r2b);
            *reinterpret_cast<unsigned*>(lds + 2 * G::PLANE + off) = pack2(r3a, r3b);
            *reinterpret_cast<unsigned*>(lds + 3 * G::PLANE + off) = pack2(i1a, i1b);
            *reinterpret_cast<unsigned*>(lds + 4 * G::PLANE + off) = pack2(i2a, i2b);
            *reinterpret_cast<unsigned*>(lds + 5 * G::PLANE + off) = pack2(i3a, i3b);
        }
    }
}

template <int Q>
__global__ __launch_bounds__(NT, 2) void k_fir_mfma(const float2* __restrict__ in,
                                                    const float2* __restrict__ hist_in,
                                                    float2* __restrict__ hist_out,
                                                    float2* __restrict__ out,
                                                    const bf16x8* __restrict__ frag, // [3][S][64]
                                                    int L,
                                                    int64_t n_out,
                                                    int in_aligned)
{
    using G = geom<Q>;
    constexpr int S = G::S;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out;

    if (blockIdx.x == 0) {
        for (int j = tid; j < L - 1; j += NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }

    // Tap fragments for the whole launch.
    bf16x8 B0[S], B1[S], B2[S];
#pragma unroll
    for (int st = 0; st < S; ++st) {
        B0[st] = frag[(0 * S + st) * 64 + lane];
        B1[st] = frag[(1 * S + st) * 64 + lane];
        B2[st] = frag[(2 * S + st) * 64 + lane];
    }

    const int64_t nchunks = (n_out + CHUNK - 1) / CHUNK;
    const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = (int64_t)blockIdx.x * per;
    const int64_t c_end = c_begin + per < nchunks ? c_begin + per : nchunks;
    if (c_begin >= c_end) return;

    // A-fragment addressing: row rho = b + 16c; lane half h selects k offset 8h.
    const int rho = lane & 31;
    const int b = rho & 15;
    const int c = rho >> 4;
    const int h = lane >> 5;
    const int a_base = c * 3 * G::PLANE + ((Q - 1) + 16 * wave + b) * 80 + 16 * h; // bytes, k-step 0
    // Output addressing: C[row][col], col = lane&31 = phase, row = (reg&3) + 8(reg>>2) + 4h.
    const int phase = lane & 31;

    float4 v[G::VPT];
    stage_load<Q>(v, in, hist_in, c_begin, n_in, L, in_aligned != 0);

    for (int64_t ch = c_begin; ch < c_end; ++ch) {
        if (ch != c_begin) __syncthreads(); // previous chunk's fragment reads are done
        stage_store<Q>(v, lds);
        __syncthreads();
        if (ch + 1 < c_end) stage_load<Q>(v, in, hist_in, ch + 1, n_in, L, in_aligned != 0);

        f32x16 acc_hi = {};
        f32x16 acc_lo = {};
#pragma unroll
        for (int st = 0; st < S; ++st) {
            const int q = st >> 1;
            const int off = a_base - q * 80 + 32 * (st & 1);
            const bf16x8 A0 = *reinterpret_cast<const bf16x8*>(lds + off);
            const bf16x8 A1 = *reinterpret_cast<const bf16x8*>(lds + off + G::PLANE);
            const bf16x8 A2 = *reinterpret_cast<const bf16x8*>(lds + off + 2 * G::PLANE);
            acc_hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0[st], acc_hi, 0, 0, 0);
            acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1[st], acc_lo, 0, 0, 0);
            acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0[st], acc_lo, 0, 0, 0);
            acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B2[st], acc_lo, 0, 0, 0);
            acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1[st], acc_lo, 0, 0, 0);
            acc_lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A2, B0[st], acc_lo, 0, 0, 0);
        }

        const int64_t n_tile = ch * CHUNK + (int64_t)wave * TILE;
#pragma unroll
        for (int reg = 0; reg < 8; ++reg) {
            const int blk = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int64_t n = n_tile + 32 * blk + phase;
            const float re = acc_hi[reg] + acc_lo[reg];
            const float im = acc_hi[reg + 8] + acc_lo[reg + 8];
            if (n < n_out) {
                nf2 o = { re, im };
                __builtin_nontemporal_store(o, reinterpret_cast<nf2*>(out + n));
            }
        }
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

template <int Q>
int launch_q(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out, hipStream_t s)
{
    using G = geom<Q>;
    static bool attr_set = false;
    if (!attr_set) {
        NSH_CK(hipFuncSetAttribute((const void*)k_fir_mfma<Q>, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS));
        attr_set = true;
    }
    const int64_t nchunks = (n_out + CHUNK - 1) / CHUNK;
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, p->dev);
    const int64_t max_grid = (int64_t)n_cu * 2;
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    const int aligned = ((uintptr_t)in % 16 == 0) ? 1 : 0;
    hipLaunchKernelGGL(k_fir_mfma<Q>, dim3(grid), dim3(NT), G::LDS, s, in, hin, hout, out,
                       (const bf16x8*)p->frag_dev, p->L, n_out, aligned);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma)");
    return 0;
}

} // namespace

bool nsh_fir_mfma_supported(const nsh_fir_plan* p)
{
    if (p->D != 1) return false;
    const int Q = (p->L + 30) / 32 + 1;
    for (float t : p->taps_host)
        if (!(t == t) || t - t != 0.f) return false; // finite taps only
    return Q <= QMAX;
}

int nsh_fir_mfma_prepare(nsh_fir_plan* p)
{
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
    return 0;
}

int nsh_fir_mfma_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out, int64_t n_out, hipStream_t s)
{
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
