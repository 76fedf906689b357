// libnsh_hip.so: a chain of decimating FIRs in one pass over HBM -- the fused form of
// fir_filter_ccf(h_1, D_1) -> ... -> fir_filter_ccf(h_S, D_S) (BASELINE config C5:
// 4 x fir_filter_ccf(firwin(127, 0.45), 2)), by polyphase-FFT overlap-save on the composite
// filter. No reference counterpart (the reference has no FIR block); the block
// convention is the one nsh_fir_ccf and the oracle follow (oracle/nsh_oracle.c orc_fir_ccf):
//   y_s[m] = sum_k h_s[k] y_{s-1}[m D_s - k]
// which composes exactly (in real arithmetic) into one decimating filter
//   y[m] = sum_n heq[n] x[m D - n],  D = prod D_s,  heq = h_1 * (h_2 up D_1) * (h_3 up D_1 D_2) * ...
// (4 x (127, 2): D = 16, 1891 composite taps). heq is composed in double on the host.
//
// Algorithm (P = D phases, M = 512): a frame is P*M consecutive input samples
// u[t] = x[P (j0 - Q) + t], Q = ceil((Leq - 1) / P); its decimated circular convolution
//   c[q] = sum_p (u_p (*) g_p)[q],  u_p[n] = u[P n + p],  g_p[q'] = heq[P q' - p]   (512-periodic)
// equals the linear output y[j0 + q - Q] for q >= Q, i.e. V = M - Q outputs per frame
// (C5: Q = 119, V = 393), frames hopping by V rows of P samples. In frequency:
//   c = IFFT_512( sum_p FFT_512(u_p) . F_p ),   F_p = FFT_512(g_p) / 512   (host, double -> fp32)
// so a frame costs P forward 512-point FFTs, a P-term complex MAC per bin and one inverse
// FFT -- about 60 FLOP per input sample instead of the cascade's ~480 (direct or Toeplitz).
//
// Kernels: k_fir_pfft2<16> (below; the default at P = 16 since round 5: no ring, two image sets, the
// phase sum and the inverse pipelined into the next frames) and k_fir_pfft<P> (P = 8, and P = 16
// with NSH_PFFT_FORM=1), which works as follows.
// Kernel k_fir_pfft<P>: one workgroup of P waves per CU, walking a contiguous range of frames.
//   * LDS ring of M rows x P samples (row = one P-sample input row, XOR-swizzled so that wave p
//     reading phase p of 64 consecutive rows is bank-conflict-free); a frame shares Q rows with
//     the previous one, so each input sample is read from HBM once (plus Q rows at the start of
//     the workgroup's range). The next frame's V new rows are prefetched into registers (16-B
//     nontemporal buffer loads) one frame ahead and written into the rows the current frame
//     has finished with.
//   * wave p: its 512 phase samples -> registers (scaled by 2^k, below) -> radix-8 Stockham FFT
//     (3 passes, two exchanges through a wave-private padded LDS image, no barrier) -> times
//     F_p (held in registers for the whole launch) -> its image.
//   * barrier; waves 0..7 sum the P images per bin in a fixed order (deterministic) into Z;
//     every wave writes its share of the next frame's rows; barrier.
//   * wave (frame mod P) runs the inverse FFT of Z from LDS and stores the V valid outputs
//     (nontemporal 8-B stores); the other waves go on with the next frame meanwhile.
// Scale: the frame's input is multiplied by 2^k (k from the frame's largest magnitude, reduced
// per wave over the rows as they arrive) so that it lies in [1, 2) before the transforms, and
// the outputs by 2^-k: exact power-of-two scaling, so no finite input overflows or loses
// precision to fp32's range. A frame holding inf or NaN is computed by the staged chain itself
// in the fp32 direct form, stage by stage over the frame's window, in the same launch: its
// outputs carry the chain's exact NaN / inf pattern (the composite filter could give +-inf
// where the chain's intermediate inf - inf is NaN). One-stage plans: the direct form on h.
// Accuracy contract: transform rounding is relative to the frame's level, not to each output --
// an output of a quiet stretch that shares its 512-row frame with a loud burst carries the
// burst's rounding, |dy| <~ 1e-6 max|x in frame| sum|heq|.
// Accuracy: fp32 transforms, error ~1e-7 of the frame's RMS (C5: 2.2e-7 of max|y| vs the
// oracle's double-accumulated cascade; north-star tolerance 1e-5).
#include "nsh_common.hpp"
#include "nsh_cplx.hpp"

#include <cmath>
#include <cstdlib>
#include <mutex>
#include <set>
#include <string>
#include <utility>
#include <vector>

// Timing-only ablation hooks for tools/probe/pfft_ab.py (0 in every product build): 1 = no inverse
// transform, 2 = no forward transform, 4 = no global loads, 8 = no phase reduction, 16 = no
// window reads from the ring, 32 = no ring writes, 64 = no exchange writes, 128 = no product
// writes.
#ifndef NSH_PFFT_ABLATE
#define NSH_PFFT_ABLATE 0
#endif

namespace {

using nsh::cf;
using nsh::cmulw;
using nsh::dft4;
using nsh::dft8;
using nsh::rot;

#ifndef NSH_PFFT_ASM_CMUL
#define NSH_PFFT_ASM_CMUL 1
#endif
// a * w for the per-lane twiddles and the filter spectrum: nsh::cmul_asm (the C form cost a
// v_xor + v_mov per product, ~4 % of the kernel)
__device__ __forceinline__ cf cmul_tw(cf a, cf w)
{
#if NSH_PFFT_ASM_CMUL
    return nsh::cmul_asm(a, w);
#else
    return cmulw(a, w);
#endif
}

constexpr int M = 512;          // FFT length per phase
constexpr int MAX_STAGES = 8;   // stages of a chain (total decimation <= 16)
constexpr int IMG = 572;         // a wave's LDS image: the largest padded index below + 1, kept even so
                                // every carve stays 16-B aligned (an off-alignment b64/b128 access
                                // replays at 64-128 cycles)

// Three layouts of a wave's 512-entry image, each bank-conflict-free for both of its access
// patterns as the compiler emits them -- stores (ds_write_b64 / ds_write2_b64) and paired loads
// (ds_read2_b64) serve 16-lane groups from 32 banks, i.e. 16 distinct entries mod 16 per group
// (MI355X_MICROARCH.md §LDS) -- and each a base register plus immediate offsets (exhaustive
// search over paddings, tools/probe/lds_banks.py):
//   exchange 1 (pass-1 stores at 8 j + r, pass-2 loads at j + 64 r):        e = i + (i >> 4)
//   exchange 2 (pass-2 stores at 64 (j >> 3) + (j & 7) + 8 r, pass-3 loads):  e = i + 3 (i >> 5) + 2 (i >> 6)
//   products / reduction / Z (stores and loads at j + 64 r, or at tid):       e = i
// (i + (i >> 3) made 2-way conflicts on every natural-order access: 34 % of LDS cycles; i + (i >> 5),
// conflict-free under the 32-lane model of ds_read_b64, left the exchange-1 stores 2-way.)

// ring entry of (slot s, phase p): rows of P samples, phase XOR-swizzled by (s / (32 / P)) so
// that 32 consecutive slots read at one phase hit 32 distinct bank pairs
template <int P>
__device__ __forceinline__ int ring_at(int s, int p)
{
    return s * P + (p ^ ((s / (32 / P)) & (P - 1)));
}


// A wave's image addresses (one base register each, the rest immediate offsets):
//   x1 + r        = e1(8 j + r)       = 8 j + (j >> 1) + r
//   b1 + 68 r     = e1(j + 64 r)      = j + (j >> 4) + 68 r
//   x2 + o2(r)    = e2(64 (j >> 3) + (j & 7) + 8 r) = 72 (j >> 3) + (j & 7) + 8 r + 3 [r >= 4]
//   b2 + 72 r     = e2(j + 64 r)      = j + 3 (j >> 5) + 72 r
//   n  + 64 r     = j + 64 r          (products, natural order)
struct img_bases {
    cf* x1;
    cf* b1;
    cf* x2;
    cf* b2;
    cf* n;
};
__device__ __forceinline__ img_bases bases_of(cf* img, int j)
{
    return img_bases{ img + 8 * j + (j >> 1), img + j + (j >> 4), img + 72 * (j >> 3) + (j & 7), img + j + 3 * (j >> 5),
                      img + j };
}
__device__ __forceinline__ img_bases bases_of(cf* img) { return bases_of(img, threadIdx.x & 63); }

#ifndef NSH_PFFT_REGX2
#define NSH_PFFT_REGX2 0
#endif
// Exchange 2 without LDS. Stockham's pass-2 -> pass-3 exchange moves (lane 8 a + b, register r) to
// (lane 8 r + b, register a): it swaps lane bits 3..5 with register bits 0..2, one bit pair at a
// time -- lane bit 5 <-> register bit 2 by v_permlane32_swap on (v[r], v[r + 4]), lane bit 4 <->
// register bit 1 by v_permlane16_swap on (v[r], v[r + 2]), lane bit 3 <-> register bit 0 by DPP
// row_ror:8 moves on (v[r], v[r + 1]) whose bank_mask writes only the lanes that change (lanes
// 8..15 of each row take v[r + 1] from 8 lanes down, lanes 0..7 take v[r] from 8 lanes up).
// 32 VALU instructions (40 as compiled) per transform instead of 8 LDS stores and 8 loads.
// Bit-identical; measured no faster (572 vs 569 us per 2^28 inputs, profiles/r02j_pfft_lds_ab.log):
// the VALU it adds costs what the LDS traffic it removes did. Off by default.
__device__ __forceinline__ void swap32(cf& a, cf& b)
{
    const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = cf{ __uint_as_float(x[0]), __uint_as_float(y[0]) };
    b = cf{ __uint_as_float(x[1]), __uint_as_float(y[1]) };
}
__device__ __forceinline__ void swap16(cf& a, cf& b)
{
    const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = cf{ __uint_as_float(x[0]), __uint_as_float(y[0]) };
    b = cf{ __uint_as_float(x[1]), __uint_as_float(y[1]) };
}
__device__ __forceinline__ float ror8_into(float old, float src, int bank_mask_is_upper)
{
    return bank_mask_is_upper
               ? __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x128, 0xf, 0xc, false))
               : __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), 0x128, 0xf, 0x3, false));
}
__device__ __forceinline__ void swap8(cf& a, cf& b)
{
    const cf na = cf{ ror8_into(a.x, b.x, 1), ror8_into(a.y, b.y, 1) };
    const cf nb = cf{ ror8_into(b.x, a.x, 0), ror8_into(b.y, a.y, 0) };
    a = na;
    b = nb;
}
__device__ __forceinline__ void exchange2_regs(cf (&v)[8])
{
#pragma unroll
    for (int r = 0; r < 4; ++r) swap32(v[r], v[r + 4]);
#pragma unroll
    for (int r = 0; r < 8; r += 4) {
        swap16(v[r], v[r + 2]);
        swap16(v[r + 1], v[r + 3]);
    }
#pragma unroll
    for (int r = 0; r < 8; r += 2) swap8(v[r], v[r + 1]);
}

// Forward 512-point transforms of PW phase sequences per wave, v[i][r] = x_i[lane + 64 r]
// (Stockham, radix 8, three passes, the PW transforms interleaved pass by pass for ILP); on
// return v[i][r] = X_i[lane + 64 r]. Transform i exchanges through image i of the wave (ib + i IMG).
// t2[r] = W_64^{(lane & 7) r}, t3[r] = W_512^{lane r}. The images are this wave's own: no
// workgroup barrier. (The inverse transform is conj(FFT(conj(.))), the conjugations folded into
// the neighbouring operations.)
template <int PW>
__device__ __forceinline__ void fft512_multi(cf (&v)[PW][8], const img_bases& ib, const cf (&t2)[8], const cf (&t3)[8])
{
#pragma unroll
    for (int i = 0; i < PW; ++i) dft8<false>(v[i]); // pass 1 (Ns = 1) -> dst[8 j + r]
#pragma unroll
    for (int i = 0; i < PW; ++i)
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (!(NSH_PFFT_ABLATE & 64)) ib.x1[i * IMG + r] = v[i][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < PW; ++i)
#pragma unroll
        for (int r = 0; r < 8; ++r) v[i][r] = ib.b1[i * IMG + 68 * r];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
#pragma unroll
        for (int r = 1; r < 8; ++r) v[i][r] = cmul_tw(v[i][r], t2[r]);
        dft8<false>(v[i]); // pass 2 (Ns = 8) -> dst[(j >> 3) 64 + (j & 7) + 8 r]
    }
    if (NSH_PFFT_REGX2) {
#pragma unroll
        for (int i = 0; i < PW; ++i) exchange2_regs(v[i]);
    } else {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < PW; ++i)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (!(NSH_PFFT_ABLATE & 64)) ib.x2[i * IMG + 8 * r + (r >= 4 ? 3 : 0)] = v[i][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < PW; ++i)
#pragma unroll
            for (int r = 0; r < 8; ++r) v[i][r] = ib.b2[i * IMG + 72 * r];
    }
#pragma unroll
    for (int i = 0; i < PW; ++i) {
#pragma unroll
        for (int r = 1; r < 8; ++r) v[i][r] = cmul_tw(v[i][r], t3[r]);
        dft8<false>(v[i]); // pass 3 (Ns = 64) -> X[j + 64 r], kept in registers
    }
    __builtin_amdgcn_wave_barrier(); // the images are rewritten next
}

__device__ __forceinline__ float2 virt(const float2* __restrict__ in, const float2* __restrict__ hist, int64_t g,
                                       int64_t n_in, int L)
{
    if (g >= 0) return g < n_in ? in[g] : make_float2(0.f, 0.f);
    if (g >= -(int64_t)(L - 1)) return hist ? hist[g + (L - 1)] : make_float2(0.f, 0.f); // null: zeros
    return make_float2(0.f, 0.f);
}

__device__ __forceinline__ unsigned absbits(float v) { return __float_as_uint(v) & 0x7fffffffu; }
__device__ __forceinline__ unsigned maxbits4(const float4& v)
{
    return max(max(absbits(v.x), absbits(v.y)), max(absbits(v.z), absbits(v.w)));
}

// raw buffer resource over [base, base + items) (items clamped to [0, cap]): loads past the end
// return 0, stores past it are dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const float2* base, int64_t items, int64_t cap)
{
    items = items < 0 ? 0 : (items > cap ? cap : items);
    const uint64_t a = (uint64_t)base;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(items * 8));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes, 0x00020000);
}

struct pfft_args {
    const float2* x;
    const float2* hist_in;
    float2* hist_out;
    float2* out;
    int64_t n_out;
    const float2* F;   // [P][M]: FFT_512(g_p) / 512
    const float2* tw;  // [M]: e^{-2 pi i t / 512}
    const float* heq;  // [L] composite taps (fp32), for frames with inf/NaN
    int L;
    int Q;
    int V;
    int64_t nf;        // frames in the launch
    int64_t fpw;       // frames per workgroup
    unsigned long long* trace; // NSH_PFFT_TRACE builds only: per-frame phase timestamps of workgroup 0
    // the stages, for frames holding inf/NaN (0 stages: the composite direct form on heq)
    const float* stap; // concatenated stage taps
    int nst;
    int sl[MAX_STAGES];
    int sd[MAX_STAGES];
    int n1;            // entries of stage-1 output within a window (buffer A; buffer B follows it)
};

#ifndef NSH_PFFT_TRACE
#define NSH_PFFT_TRACE 0
#endif
// probe builds: s_memtime at phase k of frame f (< 64) by wave w of workgroup 0
#define PFFT_T(k)                                                                                      \
    do {                                                                                               \
        if (NSH_PFFT_TRACE == 1 && blockIdx.x == 0 && f - f0 < 64 && j == 0)                            \
            a.trace[((f - f0) * 16 + w) * 8 + (k)] = __builtin_amdgcn_s_memtime();                     \
    } while (0)

// Workgroup shape: P phases, PW per wave, NT = 64 P / PW threads. A frame's V new rows are P V / 2
// 16-B loads, i.e. ceil(V PW / 128) <= 4 PW per thread (V <= 512).
template <int P, int PW>
struct pshape {
    static constexpr int NT = 64 * P / PW;
    static constexpr int WAVES = P / PW;
    static constexpr int PRE = 4 * PW;
    static constexpr int RSTEP = 128 / PW; // ring rows between a thread's consecutive slots
};

#ifndef NSH_PFFT_RINGORDER
#define NSH_PFFT_RINGORDER 1 // the window transformed in ring order (rotated), the rotation undone at the output
#endif
#ifndef NSH_PFFT_SPLIT_WIN
#define NSH_PFFT_SPLIT_WIN 1
#endif
#ifndef NSH_PFFT_SPLIT_READS
#define NSH_PFFT_SPLIT_READS 1
#endif
#ifndef NSH_PFFT_SCALE_ALWAYS
#define NSH_PFFT_SCALE_ALWAYS 0
#endif
#ifndef NSH_PFFT_ROWPERM
#define NSH_PFFT_ROWPERM 1
#endif
// The 16-B slot (2 samples, phases 2m and 2m + 1 of one row) that thread t moves: a permutation of
// the slots within each wave's 1 KiB (loads stay one contiguous 1 KiB per wave-instruction) such
// that each 16-lane store group covers rows whose swizzles differ in parity -- P = 16: rows b and
// b + 2; P = 8: rows b, b + 1, b + 4, b + 5 -- so its 16 ring entries are distinct mod 16 (a
// ds_write_b64 group's banks). In wave order the group covered rows b, b + 1, which share their
// swizzle: every ring store was 2-way conflicted.
template <int P>
__device__ __forceinline__ int row_slot(int t)
{
    if (!NSH_PFFT_ROWPERM) return t;
    const int l = t & 63, g = l >> 4;
    if (P == 16) return (t & ~63) + (4 * (g >> 1) + (g & 1) + 2 * ((l >> 3) & 1)) * 8 + (l & 7);
    const int h = (l >> 2) & 3;
    return (t & ~63) + (8 * (g >> 1) + 2 * (g & 1) + (h & 1) + 4 * (h >> 1)) * 4 + (l & 3);
}

template <int P, int PW>
__device__ __forceinline__ void load_rows(float4 (&pre)[4 * PW], const pfft_args& a, int64_t n_in, int64_t fn)
{
    using S = pshape<P, PW>;
    // window fn's new rows = x[P fn V, P (fn + 1) V); slots past them read 0
    const int64_t b = (int64_t)P * fn * a.V;
    const __amdgpu_buffer_rsrc_t r = span_rsrc(a.x + b, n_in - b, (int64_t)P * a.V);
#pragma unroll
    for (int k = 0; k < S::PRE; ++k) pre[k] = nsh::buf_load_f4(r, (row_slot<P>(threadIdx.x) + S::NT * k) * 16);
}

// write the prefetched rows of window fn into the ring; returns this thread's max magnitude bits.
// Slot k of thread t holds samples 2 i, 2 i + 1, i = u + NT k, u = row_slot(t): rows (2 u) / P +
// RSTEP k, phases (2 u) % P and + 1 -- one swizzle for every k (RSTEP k / (32 / P) is a multiple
// of P), so each ring entry is one of two bases plus RSTEP P k, modulo the ring.
template <int P, int PW>
__device__ __forceinline__ unsigned store_rows(const float4 (&pre)[4 * PW], cf* __restrict__ ring,
                                               const pfft_args& a, int64_t fn)
{
    using S = pshape<P, PW>;
    const int items = P * a.V / 2;
    const int t = row_slot<P>(threadIdx.x);
    const int s0 = (int)((fn * a.V + a.Q + (2 * t) / P) & (M - 1)), ph = (2 * t) % P;
    const int ea = ring_at<P>(s0, ph), eb = ring_at<P>(s0, ph + 1);
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < S::PRE; ++k) {
        if (t + S::NT * k < items) {
            ring[(ea + S::RSTEP * P * k) & (M * P - 1)] = cf{ pre[k].x, pre[k].y };
            ring[(eb + S::RSTEP * P * k) & (M * P - 1)] = cf{ pre[k].z, pre[k].w };
            m = max(m, maxbits4(pre[k]));
        }
    }
    return m;
}

template <int P, int PW>
__global__ __launch_bounds__(64 * P / PW, 1) void k_fir_pfft(pfft_args a)
{
    using S = pshape<P, PW>;
    constexpr int NT = S::NT, WAVES = S::WAVES;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    cf* ring = reinterpret_cast<cf*>(lds);   // M * P
    cf* imgs = ring + M * P;                  // P * IMG
    cf* zb = imgs + P * IMG;                  // IMG
    unsigned* mx = reinterpret_cast<unsigned*>(zb + IMG); // [2][WAVES] per-wave max bits of new rows

    const int tid = threadIdx.x, j = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6); // wave-uniform: SGPR arithmetic
    const int64_t f0 = (int64_t)blockIdx.x * a.fpw;
    const int64_t f1 = min(a.nf, f0 + a.fpw);
    if (f0 >= f1) return; // whole workgroup
    const int64_t n_in = a.n_out * P;
    const int L = a.L, Q = a.Q, V = a.V;
    const img_bases ib = bases_of(imgs + w * PW * IMG); // the wave's PW images; products in the first
    if (NSH_PFFT_TRACE == 2 && tid == 0) a.trace[2 * blockIdx.x] = __builtin_amdgcn_s_memtime(); // probe: workgroup span

    if (a.hist_out && blockIdx.x == gridDim.x - 1) // the next call's history: the L-1 samples before x[n_in]
        for (int k = tid; k < L - 1; k += NT) a.hist_out[k] = virt(a.x, a.hist_in, n_in - (L - 1) + k, n_in, L);

    cf t2[8], t3[8], fw[PW][8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const float2 u = a.tw[8 * (((j & 7) * r) & 63)], v = a.tw[(j * r) & (M - 1)];
        t2[r] = cf{ u.x, u.y };
        t3[r] = cf{ v.x, v.y };
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            const float2 f = a.F[(w * PW + i) * M + j + 64 * r];
            fw[i][r] = cf{ f.x, f.y };
        }
    }

    // first window: rows [f0 V, f0 V + M), history-aware
    unsigned m = 0;
    for (int i = tid; i < M * P; i += NT) {
        const float2 xv = virt(a.x, a.hist_in, (int64_t)P * (f0 * V - Q) + i, n_in, L);
        const int s = (int)((f0 * V + i / P) & (M - 1));
        ring[ring_at<P>(s, i % P)] = cf{ xv.x, xv.y };
        m = max(m, max(absbits(xv.x), absbits(xv.y)));
    }
    m = nsh::wave_umax(m);
    if (j == 0) {
        mx[(f0 & 1) * WAVES + w] = m;
        mx[((f0 + 1) & 1) * WAVES + w] = 0u;
    }
    float4 pre[S::PRE];
    load_rows<P, PW>(pre, a, n_in, f0 + 1);
    nsh::lds_barrier();

    for (int64_t f = f0; f < f1; ++f) {
        PFFT_T(0);
        // The next window's rows (consumed in this frame's phase B) are requested here, at the top
        // of the transform phase: the CU's texture path moves 64 B/clk, so the 50 KB of a frame's
        // new rows take ~800 cycles to issue and ~800 to return -- issued in phase B they held
        // every wave there; here they overlap the transforms.
        if (f > f0 && !(NSH_PFFT_ABLATE & 4)) load_rows<P, PW>(pre, a, n_in, f + 1 < f1 ? f + 1 : a.nf + 1);
        // Re-define the per-lane constants each frame (empty asm): otherwise the compiler hoists
        // the swizzled/negated copies that cmulw's operand modifiers give for free, i.e. holds
        // every twiddle twice (the kernel has 128 VGPRs at 16 waves per CU).
#pragma unroll
        for (int i = 0; i < PW; ++i)
#pragma unroll
            for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(fw[i][r]));
#pragma unroll
        for (int r = 1; r < 8; ++r) asm volatile("" : "+v"(t2[r]), "+v"(t3[r]));
        // the window's largest magnitude: this frame's new rows and the previous frame's (which
        // hold the overlap; the first window's slot covers all of it)
        const unsigned wm = nsh::wave_umax(j < 2 * WAVES ? mx[j] : 0u); // one LDS read, DPP max
        const bool bad = wm >= 0x7f800000u; // inf or NaN in the window
        int ks = 127 - (int)(wm >> 23);      // max * 2^ks in [1, 2)
        ks = ks > 126 ? 126 : (ks < -126 ? -126 : ks);
        // A window whose largest magnitude lies in [2^-40, 2^41) -- every stream but extreme ones --
        // is not scaled: a power-of-two scale is exact, so this changes no output bit, and none of
        // such a frame's intermediates leaves fp32's normal range (saves 8 packed multiplies).
        const bool scale = NSH_PFFT_SCALE_ALWAYS || ks < -40 || ks > 40;
        if (!scale) ks = 0;
        const float sc = __uint_as_float((unsigned)(ks + 127) << 23);
        const float usc = __uint_as_float((unsigned)(127 - ks) << 23);
        const int64_t rowf = f * V;
        if (!bad) {
            cf v[PW][8];
#if NSH_PFFT_RINGORDER
            // The window in ring order: slot t = (rowf + q) mod M holds window row q, i.e. the
            // sequence read is the window rotated by s = rowf mod M. Its transform is the window's
            // times W^{s k} for every phase alike, so the inverse yields c rotated by s, which the
            // output stores undo (q = (t - s) mod M). Slots j + 64 r share one swizzle, so the eight
            // reads are one per-lane base plus immediate offsets -- no per-frame address arithmetic
            // (the rotation-free form spent ~30 VALU per wave and frame on it).
#pragma unroll
            for (int i = 0; i < PW; ++i) {
                const cf* rb = ring + ring_at<P>(j, w * PW + i);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    v[i][r] = (NSH_PFFT_ABLATE & 16) ? cf{ sc, (float)r } : rb[64 * P * r];
                    // single ds_read_b64 each: paired (ds_read2st64_b64) they are served in 16-lane
                    // groups, where lanes 2 t and 2 t + 1 share a swizzle -- 2-way conflicts on every
                    // window read (2.7 M conflict cycles per 2^25 inputs, r04zm); in the 32-lane
                    // groups of single reads the two rows of a pair sit 16 bank pairs apart
                    if (NSH_PFFT_SPLIT_WIN) asm volatile("" ::: "memory");
                }
            }
#else
            // rows rowf + j + 64 r share one swizzle (64 r moves s / (32 / P) by a multiple of P)
            const int sr = (int)((rowf + j) & (M - 1));
#pragma unroll
            for (int i = 0; i < PW; ++i) {
                const int e0 = ring_at<P>(sr, w * PW + i);
#pragma unroll
                for (int r = 0; r < 8; ++r)
                    v[i][r] = (NSH_PFFT_ABLATE & 16) ? cf{ sc, (float)r } : ring[(e0 + 64 * P * r) & (M * P - 1)];
            }
#endif
            if (scale) { // wave-uniform branch
#pragma unroll
                for (int i = 0; i < PW; ++i)
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[i][r] *= sc;
            }
            if (!(NSH_PFFT_ABLATE & 2)) fft512_multi<PW>(v, ib, t2, t3);
            // this wave's share of the phase sum, in a fixed order (deterministic)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                cf pr = cmul_tw(v[0][r], fw[0][r]);
#pragma unroll
                for (int i = 1; i < PW; ++i) pr += cmul_tw(v[i][r], fw[i][r]);
                if (!(NSH_PFFT_ABLATE & 128)) ib.n[64 * r] = pr;
            }
        } else if (a.nst < 2) {
            // one stage: the fp32 direct form on its taps (heq = h): y[j] = sum_n heq[n] u[P q - n], q = Q + t
            for (int t = tid; t < V; t += NT) {
                const int q = Q + t;
                cf acc = cf{ 0.f, 0.f };
                for (int n = 0; n < L; ++n) {
                    const int tau = P * q - n;
                    const cf u = ring[ring_at<P>((int)((rowf + tau / P) & (M - 1)), tau % P)];
                    acc = __builtin_elementwise_fma(cf{ a.heq[n], a.heq[n] }, u, acc);
                }
                if (rowf + t < a.n_out) a.out[rowf + t] = make_float2(acc.x, acc.y);
            }
        } else {
            // The staged chain itself, stage by stage in the fp32 direct form over the window (which
            // holds the chain's whole history: P Q >= sum_s (L_s - 1) prod_{j<s} D_j), so a frame
            // holding inf/NaN gets the chain's non-finite pattern exactly (the composite filter can
            // give +-inf where the chain's intermediate inf - inf gives NaN). Stage outputs ping-pong
            // between two buffers in the wave images (free now: the barrier waits for the previous
            // frame's inverse wave); values near the window start use a truncated history and are
            // never read by a final output.
            nsh::lds_barrier();
            cf* buf[2] = { imgs, imgs + a.n1 };
            const float* hs = a.stap;
            int n_prev = P * M;
            for (int st = 0; st < a.nst; ++st) {
                const int Ds = a.sd[st], Ls = a.sl[st];
                const int n_cur = (n_prev - 1) / Ds + 1;
                const cf* src = buf[(st + 1) & 1];
                cf* dst = buf[st & 1];
                for (int i = tid; i < n_cur; i += NT) {
                    cf acc = cf{ 0.f, 0.f };
                    for (int k = 0; k < Ls; ++k) {
                        const int jj = Ds * i - k;
                        if (jj < 0) break;
                        const cf u = st == 0 ? ring[ring_at<P>((int)((rowf + jj / P) & (M - 1)), jj % P)] : src[jj];
                        acc = __builtin_elementwise_fma(cf{ hs[k], hs[k] }, u, acc);
                    }
                    dst[i] = acc;
                }
                hs += Ls;
                n_prev = n_cur;
                nsh::lds_barrier();
            }
            const cf* last = buf[(a.nst - 1) & 1]; // y[m] at local m = Q + t
            for (int t = tid; t < V; t += NT)
                if (rowf + t < a.n_out) a.out[rowf + t] = make_float2(last[Q + t].x, last[Q + t].y);
        }
        PFFT_T(1);
        nsh::lds_barrier(); // B1: window f read, images hold the per-phase products
        PFFT_T(2);
        if (!bad) {
#pragma unroll
            for (int k = tid; k < M; k += NT) {
                const cf* src = imgs + k;
                // all WAVES loads first, as separate ds_read_b64 (paired ds_read2_b64 run at half
                // the LDS read rate), then the sum in a fixed order
                cf pv[WAVES];
#pragma unroll
                for (int u = 0; u < WAVES; ++u) {
                    pv[u] = src[u * PW * IMG];
                    if (NSH_PFFT_SPLIT_READS) asm volatile("" ::: "memory");
                }
                cf z = pv[0];
#pragma unroll
                for (int u = 1; u < ((NSH_PFFT_ABLATE & 8) ? 1 : WAVES); ++u) z += pv[u];
                zb[k] = cf{ z.x, -z.y }; // conj: the inverse runs as a forward transform
            }
        }
        PFFT_T(6);
        if (f + 1 < f1) {
            unsigned mn = nsh::wave_umax(store_rows<P, PW>(pre, ring, a, f + 1));
            if (j == 0) mx[((f + 1) & 1) * WAVES + w] = mn;
            PFFT_T(7);
        }
        PFFT_T(3);
        nsh::lds_barrier(); // B2: Z and window f+1 complete
        PFFT_T(4);
        // the inverse transform goes to one of waves 0..3 (one per SIMD, the oldest and so the
        // first in each SIMD's issue arbitration), rotating over the four SIMDs
        if (!(NSH_PFFT_ABLATE & 1) && !bad && w == (int)(f & 3)) {
            cf v[1][8];
#pragma unroll
            for (int r = 0; r < 8; ++r) v[0][r] = zb[j + 64 * r];
            fft512_multi<1>(v, ib, t2, t3);
            const __amdgpu_buffer_rsrc_t ro = span_rsrc(a.out + rowf, a.n_out - rowf, V);
            const cf us = cf{ usc, -usc }; // 2^-k and the output conjugation
#if NSH_PFFT_RINGORDER
            // slot t = j + 64 r holds output row q = (t - s) mod M (the window was read in ring order)
            int t0 = j - (int)(rowf & (M - 1));
            asm volatile("" : "+v"(t0)); // computed here, not hoisted
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int q = (t0 + 64 * r) & (M - 1);
                if (q >= Q) nsh::buf_store_f2(ro, (q - Q) * 8, v[0][r] * us);
            }
#else
            int ob = (j - Q) * 8;
            asm volatile("" : "+v"(ob)); // computed here, not hoisted (8 offsets would spill)
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (j + 64 * r >= Q) nsh::buf_store_f2(ro, ob + 512 * r, v[0][r] * us);
#endif
            PFFT_T(5);
        }
    }
    if (NSH_PFFT_TRACE == 2 && j == 0) // probe: the last wave to leave sets the workgroup's end
        __hip_atomic_fetch_max(&a.trace[2 * blockIdx.x + 1], (unsigned long long)__builtin_amdgcn_s_memtime(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- k_fir_pfft2: the P = 16 frame without a ring, phase images double-buffered (round 5) ----
//
// The default C5 form since r05za (NSH_PFFT_FORM=1 selects the ring form above at plan creation;
// the tests run both). The ring form spends a quarter of each frame in phase B (the phase sum and
// the ring stores, between its two barriers) with the VALU idle, and a second product set to overlap
// it with the next frame's transforms does not fit next to the 64 KiB ring. This form drops the
// ring: each lane loads its rows straight from HBM in 16-B loads and a half-wave swap regroups them
// the way Stockham's first pass wants (lane l of wave w ends with one phase at window rows
// 4 w + g + 64 r, r = 0..7; load_frame), runs pass 1 in registers and stores its outputs into that
// phase's image: exchange 1 becomes the cross-wave row -> phase transpose the ring did. The Q
// overlap rows a frame shares with the previous one are loaded again, as L2 hits (the split cache
// policy below: 8.66 HBM B per input sample, as the ring form's 8.65). With the ring gone, two sets
// of 16 phase images fit (frame f in set f & 1), and the frame pipelines:
//   A0:  frame f's pass-1 outputs (computed at the end of the previous A) -> set s
//   B1
//   A:   the inverse of frame f - 2 (one of waves 4..7, own image); every wave: frame f + 1's row
//        loads issued (16 VGPRs), pass 2, exchange 2, pass 3, times F_p, products into its image of
//        set s; waves 0..7: the phase sum of frame f - 1 (set s ^ 1) into Z[(f - 1) & 1]; every
//        wave: frame f + 1's rows -> wave max -> half-wave swap -> pass 1, kept in registers
//   B2
// Measured (profiles/r05g-r05zs): 32 % fewer LDS-active cycles than the ring form and
// no bank conflicts, the same VALU and load counts; 2.2-2.5 % faster than the ring form once its
// loads sat after B1 and the phase sum on the oldest waves (r05u, r05v, r05y). Without its row loads
// it runs ~520 us per 2^28 inputs; what the loads cost depends on how their issue interleaves with
// the young waves' transforms, not on their count (a row-reusing hop with 25 % fewer loads was 4 %
// slower, r05zd, r05zm).
// Scaling: the frame's maximum is known only after B1 (each wave sees its own rows), so pass 1 runs
// unscaled and the 2^k scale multiplies its outputs -- exact, and pass 1 cannot overflow or lose
// precision to subnormals for frames whose maximum lies in [2^-100, 2^124); a frame outside that
// range (finite, nonzero) reloads its rows, scales them, redoes pass 1 and takes one more barrier.
// A frame holding inf/NaN runs the staged chain (or the one-stage direct form) as in k_fir_pfft,
// reading its window from HBM.
constexpr int IMG2 = 571; // odd: a 16-lane group's exchange-1 stores (16 phases, one position) hit 16 bank pairs

// timing-only ablation hook for tools/probe (0 in every product build): 2 = no row loads
#ifndef NSH_PFFT2_ABLATE
#define NSH_PFFT2_ABLATE 0
#endif
// The inverse of a frame runs on wave INV_BASE + (frame & 3), one per SIMD. Waves 4..7 (the
// second-oldest quartet: the phase sum's waves 0..3 start their transforms without it, and waves
// 4..7 arrive ~1.8k cycles early at B2 in the phase trace) measured 0.6-0.8 % faster than 0..3 in four two-library
// A/Bs (r05zq; r05zo 2-3 %); 8..11 and 12..15 are 5-18 % slower (r05zp); after the wave's row loads
// instead of before them, level or slower (r05zo).
#ifndef NSH_PFFT2_REGX2
#define NSH_PFFT2_REGX2 0
#endif
#ifndef NSH_PFFT2_INV_BASE
#define NSH_PFFT2_INV_BASE 4
#endif
// Probe (round 6): waves w >= NSH_PFFT2_LATE_FROM issue the next frame's row loads after their
// products instead of after B1 (into the same registers: a second set spills). The phase
// trace puts the youngest waves' load issue ~2.7k cycles after B1, behind the older waves' loads
// in the CU's vector-memory queue, with their transforms waiting behind it; loading late, they
// transform first and meet an idle queue while the older waves run the phase sum. Measured 12-17 %
// slower (waves 4..15 / 8..15 / 12..15 late: 615-620 / 637-641 / 614 vs 542-549 us per 2^28
// inputs, bit-identical, both orders, profiles/r06w_pfft2_late_loads_ab.log): the data's latency,
// exposed before pass 1, costs more than the issue queue did. 16 = off (the product build).
#ifndef NSH_PFFT2_LATE_FROM
#define NSH_PFFT2_LATE_FROM 16
#endif
// Row-load cache policy: a frame's rows V .. M - 1 (V >= 384 for Q <= 128) are the next frame's
// first rows, read again one frame later (mostly L2 hits); rows below V are read for the last
// time. Load 3 holds rows 384 .. 511 and keeps the default policy; loads 0..2 stream
// (nontemporal), so they do not push the overlap rows out of L2 before they are read again:
// 8.72 vs 9.00 HBM B per input, time level or 0.3 % faster (r05zi); nontemporal on all four
// loses the overlap hits (10.44 B, 2 % slower).
#ifndef NSH_PFFT2_LD_AUX
#define NSH_PFFT2_LD_AUX 2 // loads 0..2
#endif
#ifndef NSH_PFFT2_LD_AUX3
#define NSH_PFFT2_LD_AUX3 0 // load 3
#endif

// Frame f's window, x[P (f V - Q) + i], i < P M, in 16-B loads: lane l = 32 h + q of wave w loads
// phases 2 m, 2 m + 1 (m = q & 7) of rows jp + 64 (2 k + h), k = 0..3, jp = 4 w + g,
// g = 2 ((q >> 3) & 1) + (q >> 4) -- each load instruction reads two 512-B runs of 4 whole rows --
// into v[2 k] (phase 2 m) and v[2 k + 1] (phase 2 m + 1); swap_pairs then leaves lane l with phase
// pp = 2 m + h at rows jp + 64 r, r = 0..7 (Stockham's pass-1 input at position jp). Load k holds
// the row blocks 2 k, 2 k + 1: load 3 the overlap rows the next frame reads again.
__device__ __forceinline__ int jp_of_lane(int w, int l)
{
    const int q = l & 31;
    return 4 * w + 2 * ((q >> 3) & 1) + (q >> 4);
}
// this lane's element of load k = 0 in a window (load k: + 128 P k)
template <int P>
__device__ __forceinline__ int e0_of_lane(int w, int l)
{
    return P * (jp_of_lane(w, l) + 64 * (l >> 5)) + 2 * (l & 7);
}
template <int P>
__device__ __forceinline__ void load_frame(cf (&v)[8], const pfft_args& a, int64_t n_in, int64_t f, int w, int j)
{
    const int64_t b = (int64_t)P * (f * a.V - a.Q);
    const int e0 = e0_of_lane<P>(w, j);
    if (b >= 0) {
        const __amdgpu_buffer_rsrc_t r = span_rsrc(a.x + b, n_in - b, (int64_t)P * M);
        nsh::buf_f4 t[4];
#pragma unroll
        for (int k = 0; k < 3; ++k)
            t[k] = __builtin_bit_cast(nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, (e0 + 128 * P * k) * 8, 0, NSH_PFFT2_LD_AUX));
        t[3] = __builtin_bit_cast(nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, (e0 + 384 * P) * 8, 0, NSH_PFFT2_LD_AUX3));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = cf{ t[k].x, t[k].y };
            v[2 * k + 1] = cf{ t[k].z, t[k].w };
        }
    } else { // the stream's first frame: history, then zeros before it
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float2 u0 = virt(a.x, a.hist_in, b + e0 + 128 * P * k, n_in, a.L);
            const float2 u1 = virt(a.x, a.hist_in, b + e0 + 128 * P * k + 1, n_in, a.L);
            v[2 * k] = cf{ u0.x, u0.y };
            v[2 * k + 1] = cf{ u1.x, u1.y };
        }
    }
}
// Frame f >= 1 (no history: f V - Q >= V - Q > 0) as raw 16-B loads into x, branch-free: the
// loads of the next frame are issued in a phase A and consumed at its end, and any register copy
// between them would wait for them (a branchy load, joined by copies, did: every wave stalled for
// the HBM round trip right after its loads). live = false: no bytes (reads 0).
template <int P>
__device__ __forceinline__ void load_rows16(nsh::buf_f4 (&x)[4], const pfft_args& a, int64_t n_in, int64_t f, bool live,
                                            int e0)
{
    const int64_t b = (int64_t)P * (f * a.V - a.Q);
    const __amdgpu_buffer_rsrc_t r = span_rsrc(a.x + b, live ? n_in - b : 0, (int64_t)P * M);
#if NSH_PFFT2_ABLATE & 2 // timing only: no row loads
    (void)r;
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = nsh::buf_f4{ (float)k, 1.f, 2.f, (float)e0 };
#else
#pragma unroll
    for (int k = 0; k < 3; ++k) // one address VGPR: the load's distance in the scalar offset
        x[k] = __builtin_bit_cast(nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, e0 * 8, 1024 * P * k, NSH_PFFT2_LD_AUX));
    x[3] = __builtin_bit_cast(nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, e0 * 8, 1024 * P * 3, NSH_PFFT2_LD_AUX3));
#endif
}
__device__ __forceinline__ void unpack_rows(cf (&v)[8], const nsh::buf_f4 (&x)[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = cf{ x[k].x, x[k].y };
        v[2 * k + 1] = cf{ x[k].z, x[k].w };
    }
}
// lanes l < 32 keep phase 2 m (row block 2 k theirs, 2 k + 1 from lane l + 32), lanes l >= 32
// keep phase 2 m + 1 (block 2 k from lane l - 32, 2 k + 1 theirs): v[2 k] <-> v[2 k + 1] across
// the halves
__device__ __forceinline__ void swap_pairs(cf (&v)[8])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * k].x), __float_as_uint(v[2 * k + 1].x), false,
                                                        false);
        const auto y = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * k].y), __float_as_uint(v[2 * k + 1].y), false,
                                                        false);
        v[2 * k] = cf{ __uint_as_float(x[0]), __uint_as_float(y[0]) };
        v[2 * k + 1] = cf{ __uint_as_float(x[1]), __uint_as_float(y[1]) };
    }
}

__device__ __forceinline__ unsigned maxbits8(const cf (&v)[8])
{
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) m = max(m, max(absbits(v[k].x), absbits(v[k].y)));
    return m;
}

template <int P>
__global__ __launch_bounds__(64 * P, 1) void k_fir_pfft2(pfft_args a)
{
    static_assert(P == 16, "the ring-less form is built for 16 phases (16 waves)");
    constexpr int NT = 64 * P, SET = P * IMG2;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    cf* sets = reinterpret_cast<cf*>(lds);              // [2][P][IMG2] phase images, frame f in set f & 1
    cf* zb = sets + 2 * SET;                             // [2][M] conj(Z), frame f in f & 1
    cf* iimg = zb + 2 * M;                               // [IMG2] the inverse wave's exchange image
    unsigned* mx = reinterpret_cast<unsigned*>(iimg + IMG2 + 1); // [2][P] per-wave max bits of the frame's rows

    const int tid = threadIdx.x, j = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t f0 = (int64_t)blockIdx.x * a.fpw;
    const int64_t f1 = min(a.nf, f0 + a.fpw);
    if (f0 >= f1) return; // whole workgroup
    const int64_t n_in = a.n_out * P;
    const int L = a.L, Q = a.Q, V = a.V;
    // pass 1: phase pp at Stockham position jp (= 4 w + g); its outputs go to image pp at 8 jp + r
    const int pp = 2 * (j & 7) + (j >> 5), jp = jp_of_lane(w, j);
    const int e0 = e0_of_lane<P>(w, j); // this lane's element of load 0 in a window
    const int e1off = pp * IMG2 + 8 * jp + (jp >> 1);

    if (a.hist_out && blockIdx.x == gridDim.x - 1) // the next call's history: the L-1 samples before x[n_in]
        for (int k = tid; k < L - 1; k += NT) a.hist_out[k] = virt(a.x, a.hist_in, n_in - (L - 1) + k, n_in, L);

    cf t2[8], t3[8], fw[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const float2 u = a.tw[8 * (((j & 7) * r) & 63)], v = a.tw[(j * r) & (M - 1)];
        t2[r] = cf{ u.x, u.y };
        t3[r] = cf{ v.x, v.y };
        const float2 fv = a.F[w * M + j + 64 * r];
        fw[r] = cf{ fv.x, fv.y };
    }

    // the inverse of frame fi (conj(Z) in zb[fi & 1]) by this wave, its exchanges in iimg
    // (the lane's addresses of the inverse and the phase sum are recomputed from an opaque copy of
    // the lane id each time: hoisted out of the frame loop they would hold VGPRs the transform needs)
    auto inverse = [&](int64_t fi, int ksi) {
        int jj = j;
        asm volatile("" : "+v"(jj));
        cf v[1][8];
        const cf* z = zb + (int)(fi & 1) * M + jj;
#pragma unroll
        for (int r = 0; r < 8; ++r) v[0][r] = z[64 * r];
        fft512_multi<1>(v, bases_of(iimg, jj), t2, t3);
        const int64_t rowi = fi * V;
        const __amdgpu_buffer_rsrc_t ro = span_rsrc(a.out + rowi, a.n_out - rowi, V);
        const float us = __uint_as_float((unsigned)(127 - ksi) << 23);
        const cf u2 = cf{ us, -us }; // 2^-k and the output conjugation
        const int ob = (jj - Q) * 8;
#pragma unroll
        for (int r = 0; r < 8; ++r)
            if (jj + 64 * r >= Q) nsh::buf_store_f2(ro, ob + 512 * r, v[0][r] * u2);
    };
    // the phase sum of frame fi (products in set fi & 1) into zb[fi & 1], by waves 0..7, in a fixed
    // order (deterministic). (The oldest waves: the youngest, last in issue arbitration, wait longest
    // at their row loads and must not carry the sum as well -- 4 % faster, r05v.)
    auto phase_sum = [&](int64_t fi) {
        int k = tid;
        asm volatile("" : "+v"(k));
        const cf* src = sets + (int)(fi & 1) * SET + k;
        cf zz = cf{ 0.f, 0.f };
#pragma unroll
        for (int h = 0; h < P; h += 8) { // eight loads in flight at a time (register budget), summed in order
            cf pv[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                pv[q] = src[(h + q) * IMG2];
                asm volatile("" ::: "memory"); // single ds_read_b64 each (paired reads run at half rate)
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) zz = (h + q == 0) ? pv[0] : zz + pv[q];
        }
        zb[(int)(fi & 1) * M + k] = cf{ zz.x, -zz.y }; // conj: the inverse runs as a forward transform
    };

    auto inv_wave = [](int64_t fi) { return (int)(fi & 3) + NSH_PFFT2_INV_BASE; };
    // v: the next frame's rows, loaded during the current frame's phase A, then its pass 1
    cf v[8];
    auto pass1_of = [&](int64_t fn) { // rows of frame fn in v -> its wave max in mx[fn & 1], pass 1 in v
        const unsigned m = nsh::wave_umax(maxbits8(v));
        if (j == 0) mx[(int)(fn & 1) * P + w] = m;
        swap_pairs(v);
        dft8<false>(v);
    };
    load_frame<P>(v, a, n_in, f0, w, j);
    pass1_of(f0);
    // the pipeline: in frame f's phase A, the phase sum of frame f - 1 and the inverse of frame f - 2
    bool sum1 = false, inv2 = false; // owed: the phase sum of f - 1, the inverse of f - 2
    int ks1 = 0, ks2 = 0;            // their scales

    for (int64_t f = f0; f < f1; ++f) {
        const int s = (int)(f & 1);
        cf* cur = sets + s * SET;
#pragma unroll
        for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(fw[r]));
#pragma unroll
        for (int r = 1; r < 8; ++r) asm volatile("" : "+v"(t2[r]), "+v"(t3[r]));
        PFFT_T(0);
        nsh::buf_f4 nx[4]; // the next frame's rows, requested after B1
        // A0: frame f's pass-1 outputs (computed at the end of the previous phase A) into set s
#pragma unroll
        for (int r = 0; r < 8; ++r) cur[e1off + r] = v[r];
        PFFT_T(1);
        nsh::lds_barrier(); // B1: exchange 1 of frame f complete
        PFFT_T(2);

        const unsigned wm = nsh::wave_umax(j < P ? mx[s * P + j] : 0u);
        const bool bad = wm >= 0x7f800000u; // inf or NaN in the window
        int ks = 127 - (int)(wm >> 23);
        ks = ks > 126 ? 126 : (ks < -126 ? -126 : ks);
        const bool scale = ks < -40 || ks > 40;
        if (!scale) ks = 0;
        const float sc = __uint_as_float((unsigned)(ks + 127) << 23);
        // pass 1 unscaled is safe for maxima in [2^-100, 2^124); outside it, redo pass 1 on scaled rows
        const bool redo = !bad && (wm >= (251u << 23) || (wm != 0u && wm < (27u << 23)));
        if (redo) { // workgroup-uniform
            cf u[8];
            load_frame<P>(u, a, n_in, f, w, j);
            swap_pairs(u);
#pragma unroll
            for (int r = 0; r < 8; ++r) u[r] *= sc;
            dft8<false>(u);
#pragma unroll
            for (int r = 0; r < 8; ++r) cur[e1off + r] = u[r]; // no wave has read set s since B1
            nsh::lds_barrier();
        }

        // A: the inverse of frame f - 2 (one of waves 4..7, rotating over the SIMDs), the next frame's
        // rows requested (after B1: 6 % faster than at the frame top, r05u; s_setprio variants and
        // loads split over phase A slower, r05w, r05x, r05z, r05zb), phase w of frame f, the phase sum
        // of frame f - 1 (waves 0..7; set s ^ 1 is rewritten only by frame f + 1's pass 1, after B2),
        // the next frame's pass 1
        if (inv2 && w == inv_wave(f - 2)) inverse(f - 2, ks2);
#if NSH_PFFT2_LATE_FROM < 16
        const bool late = w >= NSH_PFFT2_LATE_FROM; // wave-uniform
        if (!late)
#endif
            load_rows16<P>(nx, a, n_in, f + 1, f + 1 < f1, e0);
        PFFT_T(3);
        const int64_t rowf = f * V;
        if (!bad) {
            const img_bases ib = bases_of(cur + w * IMG2);
            cf u[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) u[r] = ib.b1[68 * r];
            if (scale && !redo) {
#pragma unroll
                for (int r = 0; r < 8; ++r) u[r] *= sc;
            }
#pragma unroll
            for (int r = 1; r < 8; ++r) u[r] = cmul_tw(u[r], t2[r]);
            dft8<false>(u); // pass 2 -> dst[(j >> 3) 64 + (j & 7) + 8 r]
#if NSH_PFFT2_REGX2
            exchange2_regs(u); // probe: exchange 2 by lane swaps instead of the wave's image
#else
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 8; ++r) ib.x2[8 * r + (r >= 4 ? 3 : 0)] = u[r];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 8; ++r) u[r] = ib.b2[72 * r];
#endif
#pragma unroll
            for (int r = 1; r < 8; ++r) u[r] = cmul_tw(u[r], t3[r]);
            dft8<false>(u); // pass 3 -> X[j + 64 r]
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 8; ++r) ib.n[64 * r] = cmul_tw(u[r], fw[r]);
        } else if (a.nst < 2) {
            // one stage: the fp32 direct form on its taps (heq = h) over the window in HBM
            const int64_t wb = (int64_t)P * (rowf - Q);
            for (int t = tid; t < V; t += NT) {
                const int q = Q + t;
                cf acc = cf{ 0.f, 0.f };
                for (int n = 0; n < L; ++n) {
                    const float2 x = virt(a.x, a.hist_in, wb + P * q - n, n_in, L);
                    acc = __builtin_elementwise_fma(cf{ a.heq[n], a.heq[n] }, cf{ x.x, x.y }, acc);
                }
                if (rowf + t < a.n_out) a.out[rowf + t] = make_float2(acc.x, acc.y);
            }
        } else {
            // the staged chain, stage by stage in the fp32 direct form (as k_fir_pfft), its window
            // read from HBM, stage outputs ping-ponging between two buffers in set s
            const int64_t wb = (int64_t)P * (rowf - Q);
            cf* buf[2] = { cur, cur + a.n1 };
            const float* hs = a.stap;
            int n_prev = P * M;
            for (int st = 0; st < a.nst; ++st) {
                const int Ds = a.sd[st], Ls = a.sl[st];
                const int n_cur = (n_prev - 1) / Ds + 1;
                const cf* src = buf[(st + 1) & 1];
                cf* dst = buf[st & 1];
                for (int i = tid; i < n_cur; i += NT) {
                    cf acc = cf{ 0.f, 0.f };
                    for (int k = 0; k < Ls; ++k) {
                        const int jj = Ds * i - k;
                        if (jj < 0) break;
                        cf u;
                        if (st == 0) {
                            const float2 x = virt(a.x, a.hist_in, wb + jj, n_in, L);
                            u = cf{ x.x, x.y };
                        } else {
                            u = src[jj];
                        }
                        acc = __builtin_elementwise_fma(cf{ hs[k], hs[k] }, u, acc);
                    }
                    dst[i] = acc;
                }
                hs += Ls;
                n_prev = n_cur;
                nsh::lds_barrier();
            }
            const cf* last = buf[(a.nst - 1) & 1]; // y[m] at local m = Q + t
            for (int t = tid; t < V; t += NT)
                if (rowf + t < a.n_out) a.out[rowf + t] = make_float2(last[Q + t].x, last[Q + t].y);
        }
        PFFT_T(4);
#if NSH_PFFT2_LATE_FROM < 16
        if (late) load_rows16<P>(nx, a, n_in, f + 1, f + 1 < f1, e0); // the same registers, loaded late
#endif
        if (sum1 && w < P / 2) phase_sum(f - 1);
        if (f + 1 < f1) {
            unpack_rows(v, nx);
            pass1_of(f + 1);
        }
        PFFT_T(5);
        nsh::lds_barrier(); // B2: the products of frame f and Z of frame f - 1 complete
        PFFT_T(6);
        inv2 = sum1;
        ks2 = ks1;
        sum1 = !bad;
        ks1 = ks;
    }
    // drain the pipeline: the phase sum of the last frame and the inverses of the last two
    if (inv2 && w == inv_wave(f1 - 2)) inverse(f1 - 2, ks2);
    if (sum1) {
        if (w < P / 2) phase_sum(f1 - 1);
        nsh::lds_barrier();
        if (w == inv_wave(f1 - 1)) inverse(f1 - 1, ks1);
    }
}

hipError_t set_lds_attr(const void* fn, int bytes, int dev)
{
    static std::mutex mtx;
    static std::set<std::pair<const void*, int>> done;
    std::lock_guard<std::mutex> g(mtx);
    if (done.count({ fn, dev })) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert({ fn, dev });
    return e;
}

// Phases per wave. Two per wave (8 waves at P = 16, half the product and reduction LDS traffic,
// two independent transforms per wave) measured 650 vs 600 us per 2^28 inputs against one per
// wave (16 waves: more waves per SIMD to cover LDS latency; profiles/r02i_ab_pfft_pw.log).
#ifndef NSH_PFFT_PW16
#define NSH_PFFT_PW16 1
#endif
constexpr int PW16 = NSH_PFFT_PW16;
constexpr int PW8 = 1;

template <int P>
constexpr int lds_bytes()
{
    static_assert(((M * P + P * IMG + IMG) * 8) % 16 == 0, "LDS carves must stay 16-B aligned");
    return (M * P + P * IMG + IMG) * 8 + 2 * P * 4;
}
template <int P>
constexpr int lds_bytes2()
{
    return (2 * P * IMG2 + 2 * M + IMG2 + 1) * 8 + 2 * P * 4;
}
static_assert(lds_bytes2<16>() <= 160 * 1024, "k_fir_pfft2's LDS");

// The C5 (P = 16) form: 2 = k_fir_pfft2 (round 5, default: 2.2-2.5 % faster, r05y), 1 = k_fir_pfft (environment
// NSH_PFFT_FORM at plan creation, for one-process A/B and the tests of both)
#ifndef NSH_PFFT_FORM16
#define NSH_PFFT_FORM16 2
#endif

} // namespace

struct nsh_fir_casc_plan {
    int dev = 0;
    int D = 1;    // total decimation = phases P
    int L = 0;    // composite taps
    int Q = 0;    // overlap rows
    int V = 0;    // outputs per frame
    int n_cu = 256;
    int wg_per_cu = 1;
    int form = 1; // 2: k_fir_pfft2 (P = 16)
    float2* F = nullptr;
    float2* tw = nullptr;
    float* heq = nullptr;
    float* stap = nullptr; // stage taps, concatenated (non-finite frames)
    int nst = 0;           // stages the non-finite path runs (0: composite direct form)
    int sl[MAX_STAGES] = {};
    int sd[MAX_STAGES] = {};
    int n1 = 0;
    std::string kernel;
};

#if NSH_PFFT_TRACE
unsigned long long* g_pfft_trace = nullptr;
extern "C" int nsh_pfft_trace_copy(unsigned long long* host) // probe builds only
{
    NSH_CK(hipDeviceSynchronize());
    NSH_CK(hipMemcpy(host, g_pfft_trace, 64 * 16 * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return 0;
}
#endif

extern "C" {

int nsh_fir_cascade_plan_create(int dev, const float* const* taps_host, const int* ntaps, const int* decims,
                                int nstages, void** plan)
{
    if (!plan) return nsh::fail_msg("nsh_fir_cascade_plan_create: null plan pointer");
    *plan = nullptr;
    if (nstages < 1 || !taps_host || !ntaps || !decims) return nsh::fail_msg("nsh_fir_cascade_plan_create: no stages");
    // composite taps, in double: heq = h_1 * (h_2 up D_1) * ...
    std::vector<double> heq(1, 1.0);
    int D = 1;
    for (int s = 0; s < nstages; ++s) {
        if (ntaps[s] < 1 || !taps_host[s] || decims[s] < 1)
            return nsh::fail_msg("nsh_fir_cascade_plan_create: every stage needs >= 1 tap and decim >= 1");
        if ((int64_t)D * decims[s] > 16) return nsh::fail_msg("nsh_fir_cascade_plan_create: total decimation above 16");
        for (int k = 0; k < ntaps[s]; ++k)
            if (!std::isfinite(taps_host[s][k])) return nsh::fail_msg("nsh_fir_cascade_plan_create: taps must be finite");
        std::vector<double> c(heq.size() + (size_t)(ntaps[s] - 1) * D, 0.0);
        for (size_t i = 0; i < heq.size(); ++i)
            for (int k = 0; k < ntaps[s]; ++k) c[i + (size_t)k * D] += heq[i] * (double)taps_host[s][k];
        heq.swap(c);
        D *= decims[s];
    }
    if (D != 8 && D != 16) return nsh::fail_msg("nsh_fir_cascade_plan_create: total decimation must be 8 or 16");
    const int L = (int)heq.size();
    const int Q = (L - 1 + D - 1) / D;
    if (Q > M / 2) return nsh::fail_msg("nsh_fir_cascade_plan_create: composite filter longer than 256 output rows");
    auto* p = new nsh_fir_casc_plan();
    p->D = D;
    p->L = L;
    p->Q = Q;
    p->V = M - Q;
    p->dev = dev;
    hipError_t e = hipSetDevice(dev); // as nsh_fir_plan_create: the plan's device becomes current
    int ncu = 0;
    if (e == hipSuccess && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->dev) == hipSuccess && ncu > 0)
        p->n_cu = ncu;
    p->wg_per_cu = D == 16 ? 1 : 2;
    // F_p[k] = FFT_512(g_p)[k] / 512, g_p[q'] = heq[D q' - p]
    std::vector<float2> F((size_t)D * M), tw(M);
    std::vector<double> cs(M), sn(M);
    for (int t = 0; t < M; ++t) {
        const double ang = -2.0 * M_PI * (double)t / (double)M;
        cs[t] = std::cos(ang);
        sn[t] = std::sin(ang);
        tw[t] = make_float2((float)cs[t], (float)sn[t]);
    }
    for (int ph = 0; ph < D; ++ph)
        for (int k = 0; k < M; ++k) {
            double re = 0.0, im = 0.0;
            for (int q = 0; q <= Q; ++q) {
                const int n = D * q - ph;
                if (n < 0 || n >= L) continue;
                const int t = (int)(((int64_t)k * q) & (M - 1));
                re += heq[n] * cs[t];
                im += heq[n] * sn[t];
            }
            F[(size_t)ph * M + k] = make_float2((float)(re / M), (float)(im / M));
        }
    std::vector<float> hf(heq.begin(), heq.end());
    // the stages for non-finite frames: stage outputs within one window ping-pong between two
    // buffers in the wave images (stage 1's, then stage 2's size); a chain that does not fit (a
    // leading decim-1 stage), or has one stage, uses the composite direct form instead
    std::vector<float> st;
    if (nstages >= 2 && nstages <= MAX_STAGES) {
        const int n1 = (D * M - 1) / decims[0] + 1, n2 = (n1 - 1) / decims[1] + 1;
        if ((int64_t)(n1 + n2) <= (int64_t)D * IMG2) { // the smaller of both forms' image sets
            p->nst = nstages;
            p->n1 = n1;
            for (int s = 0; s < nstages; ++s) {
                p->sl[s] = ntaps[s];
                p->sd[s] = decims[s];
                st.insert(st.end(), taps_host[s], taps_host[s] + ntaps[s]);
            }
        }
    }
    if (e == hipSuccess && !st.empty()) e = hipMalloc(&p->stap, st.size() * sizeof(float));
    if (e == hipSuccess && !st.empty()) e = hipMemcpy(p->stap, st.data(), st.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->F, F.size() * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&p->tw, tw.size() * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&p->heq, hf.size() * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(p->F, F.data(), F.size() * sizeof(float2), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->tw, tw.data(), tw.size() * sizeof(float2), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->heq, hf.data(), hf.size() * sizeof(float), hipMemcpyHostToDevice);
    if (D == 16) {
        const char* fe = std::getenv("NSH_PFFT_FORM");
        p->form = fe && *fe ? std::atoi(fe) : NSH_PFFT_FORM16;
        if (p->form != 1 && p->form != 2) {
            delete p;
            return nsh::fail_msg("nsh_fir_cascade_plan_create: NSH_PFFT_FORM must be 1 or 2");
        }
    }
    if (e == hipSuccess) {
        if (p->form == 2)
            e = set_lds_attr((const void*)k_fir_pfft2<16>, lds_bytes2<16>(), p->dev);
        else if (D == 16)
            e = set_lds_attr((const void*)k_fir_pfft<16, PW16>, lds_bytes<16>(), p->dev);
        else
            e = set_lds_attr((const void*)k_fir_pfft<8, PW8>, lds_bytes<8>(), p->dev);
    }
    if (e != hipSuccess) {
        if (p->F) (void)hipFree(p->F);
        if (p->tw) (void)hipFree(p->tw);
        if (p->heq) (void)hipFree(p->heq);
        if (p->stap) (void)hipFree(p->stap);
        delete p;
        return nsh::fail(e, "nsh_fir_cascade_plan_create");
    }
    p->kernel = p->form == 2 ? std::string("k_fir_pfft2<16>")
                             : "k_fir_pfft<" + std::to_string(D) + "," + std::to_string(D == 16 ? PW16 : PW8) + ">";
    *plan = p;
    return 0;
}

int nsh_fir_cascade_plan_destroy(void* plan)
{
    auto* p = static_cast<nsh_fir_casc_plan*>(plan);
    if (!p) return 0;
    if (p->F) (void)hipFree(p->F);
    if (p->tw) (void)hipFree(p->tw);
    if (p->heq) (void)hipFree(p->heq);
    if (p->stap) (void)hipFree(p->stap);
    delete p;
    return 0;
}

int nsh_fir_cascade_decim(void* plan) { return plan ? static_cast<nsh_fir_casc_plan*>(plan)->D : 0; }
int nsh_fir_cascade_hist_len(void* plan) { return plan ? static_cast<nsh_fir_casc_plan*>(plan)->L - 1 : 0; }
const char* nsh_fir_cascade_kernel(void* plan) { return plan ? static_cast<nsh_fir_casc_plan*>(plan)->kernel.c_str() : ""; }

int nsh_fir_cascade_ccf(void* plan, const float* in, const float* hist_in, float* hist_out, float* out, int64_t n_out,
                        void* stream)
{
    nsh::launch_events_guard timing_guard; // the armed event pair never outlives this call
    auto* p = static_cast<nsh_fir_casc_plan*>(plan);
    if (!p) return nsh::fail_msg("nsh_fir_cascade_ccf: null plan");
    if (n_out <= 0) return 0;
    if (n_out > ((int64_t)1 << 40)) return nsh::fail_msg("nsh_fir_cascade_ccf: n_out too large");
    if (!in || !out) return nsh::fail_msg("nsh_fir_cascade_ccf: null input or output");
    if (hist_in == hist_out && hist_out && p->L > 1) return nsh::fail_msg("nsh_fir_cascade_ccf: hist_out must not alias hist_in");
    pfft_args a;
    a.x = (const float2*)in;
    a.hist_in = (const float2*)hist_in;
    a.hist_out = (float2*)hist_out;
    a.out = (float2*)out;
    a.n_out = n_out;
    a.F = p->F;
    a.tw = p->tw;
    a.heq = p->heq;
    a.L = p->L;
    a.Q = p->Q;
    a.V = p->V;
    a.nf = (n_out + p->V - 1) / p->V;
    const int64_t max_wg = (int64_t)p->n_cu * p->wg_per_cu;
    int64_t wg = a.nf < max_wg ? a.nf : max_wg;
    a.fpw = (a.nf + wg - 1) / wg;
    a.trace = nullptr;
    a.stap = p->stap;
    a.nst = p->nst;
    a.n1 = p->n1;
    for (int k = 0; k < MAX_STAGES; ++k) {
        a.sl[k] = p->sl[k];
        a.sd[k] = p->sd[k];
    }
#if NSH_PFFT_TRACE
    {
        static unsigned long long* tr = nullptr;
        if (!tr) NSH_CK(hipMalloc(&tr, 64 * 16 * 8 * sizeof(unsigned long long)));
        NSH_CK(hipMemsetAsync(tr, 0, 64 * 16 * 8 * sizeof(unsigned long long), nsh::S(stream)));
        a.trace = tr;
        g_pfft_trace = tr;
    }
#endif
    wg = (a.nf + a.fpw - 1) / a.fpw;
    if (p->form == 2)
        nsh::launch((k_fir_pfft2<16>), dim3((unsigned)wg), dim3(64 * 16), lds_bytes2<16>(), nsh::S(stream), a);
    else if (p->D == 16)
        nsh::launch((k_fir_pfft<16, PW16>), dim3((unsigned)wg), dim3(pshape<16, PW16>::NT), lds_bytes<16>(),
                    nsh::S(stream), a);
    else
        nsh::launch((k_fir_pfft<8, PW8>), dim3((unsigned)wg), dim3(pshape<8, PW8>::NT), lds_bytes<8>(),
                    nsh::S(stream), a);
    NSH_CK_LAUNCH("nsh_fir_cascade_ccf");
    return 0;
}

} // extern "C"
