// libnsh_hip.so: fir_filter_ccf on the matrix cores -- the product kernels.
//
//   k_fir_mfma12<Q>      decim 1 (the C3 bench kernel)
//   k_fir_exact12<Q>     decim 1: the chunks k_fir_mfma12 queued for an exact form (same call, same stream)
//   k_fir_mfma11<D, QH>  decim 2 and 4 (polyphase; the staged C5 chain's stages)
//
// Blocked Toeplitz form. Split the output stream into 32-sample blocks; output n = 32*beta + i:
//     y[32 beta + i] = sum_{q<Q} sum_{r<32} h[i - r + 32 q] * x[32 (beta - q) + r]
// i.e. C[rho][i] = sum_k A[rho][k] B[k][i] with k = 32 q + r (K = 32 Q),
//     A[rho][k] = x_c[32 (beta - q) + r]    rho = (block beta, component c)  -- the stream
//     B[k][i]   = h[i - r + 32 q]           (zero outside [0, L))           -- the taps
// One v_mfma_f32_32x32x16_f16 covers 32 rows (16 blocks x {re, im}) x 32 phases x 16 k; a wave
// owns a 512-sample tile and runs 2Q k-steps (Q = 5 for L = 127, K = 160).
// Precision: fp32 from fp16x2 -- both operands split into two fp16 terms at a power-of-two
// scale (taps once on the host, samples per 2048-sample chunk), three products
// x0h0 + x0h1 + x1h0 accumulated in fp32 (see the fp16x2 notes in nsh_fir_mfma_shared.hpp and
// below); chunks whose range the split cannot hold take the exact-fp32 matrix tile, chunks holding
// inf/NaN the fp32 direct form (exact IEEE semantics) -- at decim 1 in k_fir_exact12, at decim 2
// and 4 inside the same launch.
//
// The forms this file superseded -- k_fir_mfma2 (bf16x3, six products), k_fir_mfma5 (16-sample
// blocks), k_fir_mfma7 (bf16x3 decimator), k_fir_mfma9 (v12's predecessor) and k_fir_casc2 (two
// decimators fused) -- were retired in round 4 (git history before that round has them);
// DESIGN.md section 4 keeps their measurements.
#include "nsh_fir_mfma_shared.hpp"
#include "nsh_fir_f32_tile.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

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
// Cache policy of the decimators' chunk loads. A thread loads its D float4 (2 D consecutive
// samples) in D instructions, so one instruction's lanes are 16 D bytes apart and D instructions
// touch the same lines: at D = 4 nontemporal loads fetched each line from L2 four times, the
// default policy lets the later instructions hit L1 -- 642 -> 544 us per 2^28 inputs, 52 -> 62 %;
// at D = 2 nontemporal stays faster (591 vs 638 us; profiles/r03w_v11_load_policy_ab.log).
#ifndef NSH_V11_AUX2
#define NSH_V11_AUX2 2 // nt
#endif
#ifndef NSH_V11_AUX4
#define NSH_V11_AUX4 0 // default
#endif
#ifndef NSH_V12_F32T
#define NSH_V12_F32T 1 // probe builds: 0 = finite wide-range chunks on the fp32 direct form
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

// Chunks the split cannot carry leave the bench kernel (round 4, verdict r03 item 4). A chunk
// whose samples (with its halo) are finite but span more than the fp16x2 split holds, or that
// holds inf/NaN, is not filtered by k_fir_mfma12: the workgroup appends it to the launch's exact
// queue and stops, and k_fir_exact12, launched right after on the same stream, filters the queued
// chunks -- finite ones on the exact-fp32 matrix tile of k_fir_f32mfma (nsh_fir_f32_tile.hpp: fp32
// products and sums on v_mfma_f32_16x16x4_f32, QF = 2Q - 1 tap blocks of 16 over the same
// 32 (Q - 1)-sample halo; outputs bit-identical to k_fir_f32mfma's wherever it uses the same
// blocking), non-finite ones by the fp32 direct form (exact IEEE semantics). Nothing the queued
// chunks read is written by k_fir_mfma12 (outputs never alias the input, hist_out never aliases
// hist_in), so the second kernel sees the inputs the first one saw. With the two exact forms
// compiled into it, k_fir_mfma12 ran 3 % slower on streams that never take them (735 vs 711 us
// per 2^28, profiles/r04i_v12_no_exact_ab.log): their code shaped the main path's registers and
// schedule. The queue (per plan and stream, device memory, u32 words) is split into XQ_N sub-queues
// so that a stream whose every chunk is exact does not serialise 2^17 atomics on one address
// (one counter: k_fir_mfma12 took 1.53 ms instead of ~0.4 on such a stream, profiles/r04m_*):
// workgroup b appends to sub-queue b mod XQ_N -- counter at word XQ_LINE (b mod XQ_N), entries
// from word XQ_E + (b mod XQ_N) subcap, entry = (chunk << 1) | non-finite. A queue holds two such
// sets; launch k on a stream uses set k & 1, and its k_fir_exact12 zeroes the other set's
// counters (set k - 1's, consumed by the previous k_fir_exact12 on this stream; the next
// k_fir_mfma12 appends to it) -- no count of finished workgroups: 1280 agent-scope atomics on one
// word serialised into ~40 us whenever a launch queued anything (profiles/r04t_*).
template <int Q>
using geom12f = nsh_f32t::geom<2 * Q - 2, 2 * Q - 1>;
constexpr int XQ_N = 64;                   // sub-queues (one counter each)
constexpr int XQ_LINE = 64;                // words between counters (256 B)
constexpr int XQ_E = XQ_N * XQ_LINE;       // first entry word
__host__ __device__ constexpr int64_t xq_subcap(int64_t grid) { return (grid + XQ_N - 1) / XQ_N; }
#ifndef NSH_X12_PER_CU
#define NSH_X12_PER_CU 5 // k_fir_exact12 workgroups per CU (a persistent walk over the queue) = its waves per SIMD
#endif

// chunk ch -> registers (nontemporal) and its halo (default policy: the previous chunk's tail was
// just read by the previous workgroup of this XCD). Branch-free: the halo comes through one buffer
// resource, over `in` (ch > 0) or over hist_in (ch = 0; out-of-range lanes and a null history
// read zeros), so no wait sits between the loads.
template <int Q>
__device__ __forceinline__ void load12(const float2* __restrict__ in, const float2* __restrict__ hist_in, int L,
                                       int64_t n_in, int64_t ch, float4 (&v)[4], float4& hv)
{
    using G = geom12<Q>;
    const int tid = threadIdx.x;
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
}

// One chunk on an exact form, from its samples in registers: finite -> the exact-fp32 tile, else the
// fp32 direct form. Stages the chunk in LDS (after a barrier: the caller may have used LDS), then
// filters and stores it.
template <int Q>
__device__ __forceinline__ void exact_chunk12(unsigned char* lds, float2* __restrict__ out, const float4* __restrict__ timg32,
                                              const float* __restrict__ taps, int L, int64_t n_out, int64_t ch,
                                              const float4 (&v)[4], const float4& hv, bool f32t)
{
    using G = geom12<Q>;
    using GF = geom12f<Q>;
    static_assert(GF::H == G::H && GF::BYTES <= G::SLOTS, "the fp32 tile's image fits the planes + tap image");
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int h = lane >> 5;
    const int phase = lane & 31;
    nsh::lds_barrier(); // every wave is done with what LDS held before
    if (f32t) {
        float4 t32[2];
        nsh_f32t::load_taps<GF>(timg32, t32, tid, G::NT);
        if (tid < G::HP) nsh_f32t::put<GF>(lds, hv, 2 * tid);
#pragma unroll
        for (int u = 0; u < 4; ++u) nsh_f32t::put<GF>(lds, v[u], G::H + 2 * (tid + G::NT * u));
        nsh_f32t::put_taps<GF>(lds, t32, tid, G::NT);
    } else { // inf / NaN in range: the fp32 direct form (exact IEEE semantics)
        float4* r = reinterpret_cast<float4*>(lds);
        if (tid < G::HP) r[tid] = hv;
#pragma unroll
        for (int u = 0; u < 4; ++u) r[G::HP + tid + G::NT * u] = v[u];
    }
    nsh::lds_barrier();
    nf2 o[8];
    if (f32t) {
        nsh_f32t::f32x4 acc[4];
        nsh_f32t::tile<GF, 2 * Q - 1>(lds, wave, lane, acc);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int u = 0; u < 2; ++u) o[2 * t + u] = nf2{ acc[t][2 * u], acc[t][2 * u + 1] };
    } else {
        direct_tile9<Q>(lds, taps, L, wave, h, phase, o);
    }
    // direct: output wave TILE + phase + 32 ((reg & 3) + 8 (reg >> 2) + 4 h);
    // exact-fp32 tile: output 16 (32 wave + 8 t + 2 g + u) + i of o[2 t + u] (nsh_f32t::tile)
    const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(out, ch, n_out);
    const int lb = f32t ? (16 * (32 * wave + 2 * (lane >> 4)) + (lane & 15)) * 8 : (wave * TILE + phase + 128 * h) * 8;
#pragma unroll
    for (int reg = 0; reg < 8; ++reg) {
        const int c = f32t ? 128 * (4 * reg - 3 * (reg & 1)) : 256 * ((reg & 3) + 8 * (reg >> 2));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(nsh::u32x2, o[reg]), r, lb, c, nsh::AUX_ST);
    }
}

template <int Q>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_fir_mfma12(const float2* __restrict__ in,
                                                    const float2* __restrict__ hist_in,
                                                    float2* __restrict__ hist_out,
                                                    float2* __restrict__ out,
                                                    const uint4* __restrict__ timg, // [2][8][TW/8]
                                                    unsigned* __restrict__ xq,      // exact queue (above)
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
    const int64_t ch = (int64_t)(blockIdx.x & 7) * per_x + wi;
    if (ch >= nchunks) return; // whole workgroup: before any barrier

    float4 v[4], hv;
    load12<Q>(in, hist_in, L, n_in, ch, v, hv);
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
    nsh::lds_barrier();
    // workgroup-uniform, and made provably so (SGPRs): the branch on it is a scalar branch
    const unsigned m = __builtin_amdgcn_readfirstlane(max(max(slot_max[0], slot_max[1]), max(slot_max[2], slot_max[3])));
    const unsigned z = __builtin_amdgcn_readfirstlane(min(min(slot_mnz[0], slot_mnz[1]), min(slot_mnz[2], slot_mnz[3])));
    const int s = scale_of(m);
    if (__builtin_expect(chunk_needs_exact(m, z, s), 0)) {
        // k_fir_exact12 filters it (a vector atomic and a vector store from one lane)
        if (tid == 0) {
            const unsigned k = blockIdx.x % XQ_N;
            const unsigned i = __hip_atomic_fetch_add(xq + XQ_LINE * k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // i < subcap always, on a queue whose counters were zeroed (xq_reset after a failed
            // call): the bound keeps a stale counter from writing into the next sub-queue, and
            // k_fir_exact12 refilters the whole launch if the count ever exceeds it
            if (i < (unsigned)xq_subcap(gridDim.x))
                __hip_atomic_store(xq + XQ_E + k * xq_subcap(gridDim.x) + i, (unsigned)(ch << 1) | (m >= 0x7f800000u ? 1u : 0u),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        if (tid < G::HP) store_pair12<Q>(hv, lds, 2 * tid, s);
#pragma unroll
        for (int u = 0; u < 4; ++u) store_pair12<Q>(v[u], lds, G::H + 2 * (tid + G::NT * u), s);
        nsh::lds_barrier();
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
        nf2 o[8];
        if (unscale >= -126 && unscale <= 127) {
            const nf2 f = nf2{ __builtin_bit_cast(float, (unscale + 127) << 23), __builtin_bit_cast(float, (unscale + 127) << 23) };
#pragma unroll
            for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ sum[reg], sum[reg + 8] } * f;
        } else {
#pragma unroll
            for (int reg = 0; reg < 8; ++reg) o[reg] = nf2{ __builtin_ldexpf(sum[reg], unscale), __builtin_ldexpf(sum[reg + 8], unscale) };
        }
        // output wave TILE + phase + 32 ((reg & 3) + 8 (reg >> 2) + 4 h)
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<2048>(out, ch, n_out);
        const int lb = (wave * TILE + phase + 128 * h) * 8;
#pragma unroll
        for (int reg = 0; reg < 8; ++reg)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(nsh::u32x2, o[reg]), r, lb, 256 * ((reg & 3) + 8 * (reg >> 2)),
                                                  nsh::AUX_ST);
    }
    if (ch == 0) // the last L-1 inputs for the next call (after this workgroup's stores)
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
}

// The chunks k_fir_mfma12 queued: a persistent walk over the queue (NSH_X12_PER_CU workgroups per
// CU), one chunk per workgroup step, staged in the same LDS geometry (the fp32 tile's image fits
// the planes + tap image; a raw fp32 chunk + halo fits the planes).
template <int Q>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NSH_X12_PER_CU))) void k_fir_exact12(const float2* __restrict__ in,
                                                    const float2* __restrict__ hist_in,
                                                    float2* __restrict__ out,
                                                    const float4* __restrict__ timg32, // exact-fp32 tile taps [4][TWF]
                                                    const float* __restrict__ taps,
                                                    const unsigned* __restrict__ xq, // this launch's set
                                                    unsigned* __restrict__ xq_next,  // the next launch's set
                                                    int64_t subcap,
                                                    int L,
                                                    int64_t n_out)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    static_assert(XQ_N == 64, "one sub-queue counter per lane");
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    if (blockIdx.x == 0 && tid < 64) // the next launch's counters (vector stores, one lane each)
        __hip_atomic_store(xq_next + XQ_LINE * tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every wave: the XQ_N counters (one per lane) and their inclusive prefix sum
    unsigned incl = __hip_atomic_load(xq + XQ_LINE * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a sub-queue that counted more appends than it holds lost entries (never on a queue whose
    // counters were zeroed: xq_reset after a failed call): then every chunk of the
    // launch is filtered again here in the fp32 direct form -- slow, but no output is left unwritten
    const bool over = __ballot(incl > (unsigned)subcap) != 0;
    incl = min(incl, (unsigned)subcap); // entries past a sub-queue's capacity were never written
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    const int64_t nchunks = (n_out + geom12<Q>::CHUNK - 1) / geom12<Q>::CHUNK;
    const unsigned cnt = over ? (unsigned)nchunks : __builtin_amdgcn_readlane(incl, 63);
    if (cnt == 0) return; // nothing queued (the common case)
    auto entry = [&](unsigned i) {
        if (over) return (i << 1) | 1u; // chunk i, direct form
        const int k = __popcll(__ballot(incl <= i)); // sub-queue holding queued chunk i (prefix sums ascend)
        const unsigned start = k ? __shfl(incl, k - 1) : 0u;
        return __hip_atomic_load(xq + XQ_E + k * subcap + (i - start), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    for (unsigned i = blockIdx.x; i < cnt; i += gridDim.x) {
        const unsigned e = entry(i);
        if ((int64_t)(e >> 1) >= nchunks) continue; // never for a queue this launch filled (defensive)
        float4 v[4], hv;
        load12<Q>(in, hist_in, L, n_out, e >> 1, v, hv);
        exact_chunk12<Q>(lds, out, timg32, taps, L, n_out, e >> 1, v, hv, NSH_V12_F32T && !(e & 1u));
    }
}

// k_fir_mfma11's LDS with the exact-fp32 tile: a finite chunk whose range the split cannot hold is
// filtered as if undecimated by k_fir_f32mfma's tile (nsh_fir_f32_tile.hpp, QF = HR + 1 tap blocks
// of 16 over the chunk's D H-sample halo) and every D-th output kept -- the same fp32 matrix work per
// input sample as at decim 1, no polyphase form. Each plane buffer holds the tile's two fp32 planes
// (at <2,5> and <4,3> they fit the split's buffer; other forms may grow it); the tile's taps (one
// copy, loaded once per workgroup) and a per-wave output scratch (the tile's lane map -> the split
// path's, for the common store) follow the stash. LDS stays within 2 resident workgroups per CU
// (the kernel's occupancy).
template <int D, int QH>
struct geom11x : geom11<D, QH> {
    using B = geom11<D, QH>;
    static constexpr int HRF = D * (QH - 1);                     // tile halo rows (16 samples)
    static constexpr int QF = HRF + 1;
    using GF = nsh_f32t::geom<HRF, QF>;
    static constexpr int BUF = (B::BUF > 2 * GF::PLANE ? B::BUF : 2 * GF::PLANE);
    static constexpr int STASH_AT = 2 * BUF;
    static constexpr int TAPF = STASH_AT + 2 * B::STASH;          // tile taps
    static constexpr int SCR = TAPF + (GF::TAPS + 255) / 256 * 256; // [4 waves][WAVE_OUT] float2
    static constexpr int SLOTS = SCR + 4 * B::WAVE_OUT * 8;
    static constexpr int LDS = SLOTS + 64;
    static_assert(GF::H == D * B::H && BUF % 256 == 0, "tile halo = the chunk's halo");
    static_assert(2 * LDS <= 160 * 1024, "2 workgroups per CU");
};

template <int D, int QH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma11(const float2* __restrict__ in,
                                                      const float2* __restrict__ hist_in,
                                                      float2* __restrict__ hist_out,
                                                      float2* __restrict__ out,
                                                      const _Float16* __restrict__ frag, // per phase: [2][KS][64] x8, [2][64] x4
                                                      const float4* __restrict__ timg32, // tile taps [4][TWF]
                                                      const float* __restrict__ taps,
                                                      int L,
                                                      int sh,
                                                      int64_t n_out)
{
    using G = geom11x<D, QH>;
    using GF = typename G::GF;
    constexpr int KS = G::KS;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* stash = reinterpret_cast<float4*>(lds + G::STASH_AT); // [2][HP] raw halo sources
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    unsigned* slot_mnz = slot_max + 8;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out * D;
    {   // the tile's taps, once per workgroup (read after the prologue's barriers)
        float4 t32[2];
        nsh_f32t::load_taps<GF>(timg32, t32, tid, G::NT);
        nsh_f32t::put_taps_at<GF>(lds + G::TAPF, t32, tid, G::NT);
    }

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
            for (int f = 0; f < D; ++f) {
                const nsh::buf_f4 t = __builtin_bit_cast(
                    nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, ((tid + G::NT * u) * D + f) * 16, 0, D == 2 ? NSH_V11_AUX2 : NSH_V11_AUX4));
                v[u * D + f] = make_float4(t.x, t.y, t.z, t.w);
            }
    };
    auto stash_tail = [&](float4* st, const float4 (&v)[4]) {
        if (tail_owner) {
#pragma unroll
            for (int f = 0; f < D; ++f) st[(tid - (G::NT - G::H / 2)) * D + f] = v[(G::UNITS - 1) * D + f];
        }
    };
    // chunk -> buffer: raw fp32 (halo float4 [0, HP), chunk float4 HP + j) or split phase planes
    auto put_chunk = [&](unsigned char* buf, const float4* hsrc, const float4 (&v)[4], bool raw, bool f32t, int sc) {
        if (__builtin_expect(f32t, 0)) { // the tile's fp32 planes (16-sample rows), halo first
            if (tid < G::HP) nsh_f32t::put<GF>(buf, hsrc[tid], 2 * tid);
#pragma unroll
            for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
                for (int f = 0; f < D; ++f) nsh_f32t::put<GF>(buf, v[u * D + f], GF::H + 2 * ((tid + G::NT * u) * D + f));
            return;
        }
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
                // single ds_read_b64 (the empty asm keeps the compiler from pairing the tiles'
                // reads into ds_read2_b64, whose 16-lane groups see the re and im rows 4 apart on
                // one bank: 4-way, 43-50 % of the kernel's LDS cycles in profiles/r03o_pmc_decim.json;
                // as ds_read_b64, 2-way)
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - (QH - 1) * 32 + g * 8;
                    const f16x4 A0 = *reinterpret_cast<const f16x4*>(ph + off);
                    asm volatile("" ::: "memory");
                    const f16x4 A1 = *reinterpret_cast<const f16x4*>(ph + off + G::PLANE);
                    asm volatile("" ::: "memory");
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
    // the tile's outputs n = 16 (32 wave + 8 t + 2 g + u) + i (undecimated), the lanes with
    // i mod D = 0 keeping theirs (m = n / D), through the wave's LDS scratch into the split
    // path's lane map (the wave's own outputs: a wave barrier, no workgroup barrier)
    auto f32_tile = [&](const unsigned char* cur, nf2 (&o)[2 * G::TILES]) {
        f32x4 acc[4];
        nsh_f32t::tile_at<GF, G::QF>(cur, lds + G::TAPF, wave, lane, acc);
        nf2* scr = reinterpret_cast<nf2*>(lds + G::SCR) + wave * G::WAVE_OUT;
        const int i = lane & 15;
        if (i % D == 0) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int u = 0; u < 2; ++u) scr[(16 * (8 * t + 2 * g + u) + i) / D] = nf2{ acc[t][2 * u], acc[t][2 * u + 1] };
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi) o[oi] = scr[((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase];
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
    bool f32_cur = ex_cur && m_prev < 0x7f800000u; // finite: the exact-fp32 tile
    put_chunk(lds, stash + G::HP, va, ex_cur, f32_cur, s_cur);
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
        const bool f32_nxt = ex_nxt && m2 < 0x7f800000u;
        load(ld, clamp(ch + 3));
        put_chunk(nbuf, stash + pi * G::HP, nxt, ex_nxt, f32_nxt, s_nxt);
        stash_tail(stash + pn * G::HP, nxt);
        nf2 o[2 * G::TILES];
        if (__builtin_expect(ex_cur, 0)) {
            if (f32_cur)
                f32_tile(cur, o);
            else
                direct_tile(cur, o);
        } else {
            mfma_tile(cur, -(s_cur + sh), o);
        }
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
        f32_cur = f32_nxt;
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

// ---- k_fir_mfma13: the decimators' lockstep walk, exact chunks queued (round 5) ------------
#ifndef NSH_V13_AUX // chunk loads' cache policy: nontemporal on whole-line loads (no line is read twice)
#define NSH_V13_AUX (NSH_V13_CLOAD ? 2 : D == 2 ? NSH_V11_AUX2 : NSH_V11_AUX4)
#endif
// k_fir_mfma11's per-chunk work (polyphase split at a per-chunk scale, the same MFMA tile) in a
// different walk: the persistent workgroups of an XCD (x = blockIdx mod 8, W of them) take its
// eighth of the chunks in lockstep -- at step i workgroup k of XCD x filters chunk
// x per_x + k + i W -- so each XCD streams one contiguous window of W chunks at a time instead of
// W separate ranges (profiles/r04zw_v11_xcd_ab.log: D = 4 9.5 % faster, bit-identical). Each
// chunk's halo (the D H input samples before it, the tail of the chunk its neighbour filters in the
// same step: an L2 hit) is loaded with it and staged raw in an LDS stash, one step ahead, for the
// split; scale and exact-path test cover the chunk and its halo (k_fir_mfma11's scale covered the
// whole previous chunk: outputs match it within the split's rounding, bit for bit wherever both
// pick the same scale). Chunks the split cannot carry are not filtered here: the workgroup appends
// them to the launch's exact queue and k_fir_exact13 (same stream, right after) filters them -- so a
// periodic pattern of exact chunks, which the lockstep walk would put on one workgroup per XCD,
// cannot unbalance it (r04zw: every 64th chunk exact 968 vs 548 us with the exact forms inline).
// the chunk's float4 (2 input samples) a lane loads as its unit u, instruction f: the wave's
// 64 D float4 of unit u in D contiguous 1 KiB runs
template <int D>
__device__ __forceinline__ int q13(int u, int f)
{
    return 64 * D * ((int)(threadIdx.x >> 6) + 4 * u) + 64 * f + (int)(threadIdx.x & 63);
}
template <int D, int QH>
__device__ __forceinline__ void load13(const float2* __restrict__ in, const float2* __restrict__ hist_in, int L, int64_t n_in,
                                       int64_t ch, float4 (&v)[4], float4& hv)
{
    using G = geom11<D, QH>;
    const int tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK_IN>(in, ch, n_in);
#pragma unroll
    for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
        for (int f = 0; f < D; ++f) {
            // NSH_V13_CLOAD: float4 q13(u, f) of the chunk (each instruction 1 KiB contiguous), else
            // (tid + NT u) D + f (a thread's D float4 adjacent, each instruction spread over D KiB)
            const int q = NSH_V13_CLOAD ? q13<D>(u, f) : (tid + G::NT * u) * D + f;
            const nsh::buf_f4 t = __builtin_bit_cast(nsh::buf_f4, __builtin_amdgcn_raw_buffer_load_b128(r, q * 16, 0, NSH_V13_AUX));
            v[u * D + f] = make_float4(t.x, t.y, t.z, t.w);
        }
    // the halo: input samples [ch CHUNK_IN - 2 HP, ch CHUNK_IN), two per thread tid < HP, from `in`
    // (ch > 0) or the history (ch = 0: element g + L - 1; out-of-range lanes and a null history read
    // zeros); one buffer resource either way, no branch between the loads. A chunk index past the
    // stream (an empty prefetch) reads zeros.
    __amdgpu_buffer_rsrc_t hr;
    int off0, off1;
    if (ch > 0) {
        hr = chunk_rsrc<2 * G::HP>(in + ch * G::CHUNK_IN - 2 * G::HP, 0, ch * G::CHUNK_IN <= n_in ? 2 * G::HP : 0);
        off0 = 16 * tid;
        off1 = off0 + 8;
    } else {
        hr = chunk_rsrc<1 << 20>(hist_in, 0, hist_in ? L - 1 : 0);
        const int e = 2 * tid - 2 * G::HP + (L - 1);
        off0 = e >= 0 ? 8 * e : 1 << 30;
        off1 = e + 1 >= 0 ? 8 * (e + 1) : 1 << 30;
    }
    hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < G::HP) {
        const nsh::buf_f2 a = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off0, 0, 0));
        const nsh::buf_f2 b = __builtin_bit_cast(nsh::buf_f2, __builtin_amdgcn_raw_buffer_load_b64(hr, off1, 0, 0));
        hv = make_float4(a.x, a.y, b.x, b.y);
    }
}

template <int D, int QH>
__global__ __launch_bounds__(256, 2) void k_fir_mfma13(const float2* __restrict__ in,
                                                      const float2* __restrict__ hist_in,
                                                      float2* __restrict__ hist_out,
                                                      float2* __restrict__ out,
                                                      const _Float16* __restrict__ frag, // per phase: [2][KS][64] x8, [2][64] x4
                                                      unsigned* __restrict__ xq,         // this launch's exact-queue set
                                                      int64_t subcap,
                                                      int L,
                                                      int sh,
                                                      int64_t n_out,
                                                      int64_t per_x)
{
    using G = geom11<D, QH>;
    constexpr int KS = G::KS;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    float4* stash = reinterpret_cast<float4*>(lds + 2 * G::BUF); // [2][HP] raw halos, one step ahead
    unsigned* slot_max = reinterpret_cast<unsigned*>(lds + G::SLOTS);
    unsigned* slot_mnz = slot_max + 8;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t n_in = n_out * D;
    if (blockIdx.x == 0)
        for (int j = tid; j < L - 1; j += G::NT) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);

    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int W = (int)(gridDim.x >> 3);
    const int64_t xb = (int64_t)(blockIdx.x & 7) * per_x;
    const int64_t xe = xb + per_x < nchunks ? xb + per_x : nchunks;
    const int64_t c_first = xb + (blockIdx.x >> 3), hop = W;
    if (c_first >= xe) return; // whole workgroup, before any barrier
    // the workgroup's i-th chunk; past its range an empty buffer range (loads return 0)
    auto chunk_at = [&](int64_t i) { const int64_t c = c_first + i * hop; return c < xe ? c : nchunks; };
    const int64_t n_steps = (xe - c_first + hop - 1) / hop;

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

    const int rho = lane & 15;
    const int c = rho & 1, b = rho >> 1;
    const int g = lane >> 4;
    const int phase = lane & 15;
    const int row_base = c * G::IM_OFF + (G::HR + wave * (G::WAVE_OUT / 16) + b) * 32;
    auto reduce = [&](const float4 (&v)[4], const float4& hv, unsigned& m, unsigned& z) {
        float mf = max_abs4(hv);
        z = min_nz1(hv);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mf = __builtin_elementwise_maximum(mf, max_abs4(v[u]));
            z = min(z, min_nz1(v[u]));
        }
        m = wave_max(__float_as_uint(mf));
        z = wave_min(z);
    };
    auto put_halo = [&](float4* st, const float4& hv) {
        if (tid < G::HP) st[tid] = hv;
    };
    // chunk + its raw halo (stash) -> the split phase planes
    auto put_split = [&](unsigned char* buf, const float4* hsrc, const float4 (&v)[4], int sc) {
        if (tid < D * (G::H / 2)) { // halo: phase r, pair pi from the raw halo samples
            const int r = tid / (G::H / 2), pi = tid % (G::H / 2);
            const int sr = r == 0 ? 0 : D - r;
            const int pa = D * (2 * pi) + sr, pb = D * (2 * pi + 1) + sr;
            const float2 a = f4_sample(hsrc[pa >> 1], pa & 1), bb = f4_sample(hsrc[pb >> 1], pb & 1);
            store_pair11<D, QH>(buf, r, 2 * pi, a.x, bb.x, a.y, bb.y, sc);
        }
#if NSH_V13_CLOAD
        // float4 q holds samples 2q, 2q + 1: phase offsets 2q mod D (+1) at time 2q / D, the pair
        // 2q / 2D, its time bit k = q & (D / 2). Lanes q and q ^ (D / 2) hold the same offsets at the
        // pair's two times: each keeps offset k and takes the partner's (one DPP exchange per float),
        // then stores one phase pair -- all D phases in each store instruction (PH padded for it)
        constexpr int XCHG = D == 4 ? 0x4e : 0xb1; // quad_perm [2,3,0,1] / [1,0,3,2]: lane ^ (D / 2)
#pragma unroll
        for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
            for (int f = 0; f < D; ++f) {
                const int q = q13<D>(u, f);
                const bool k = (q & (D / 2)) != 0;
                const float4 x = v[u * D + f];
                const float kre = k ? x.z : x.x, kim = k ? x.w : x.y; // offset k: kept
                const float sre = k ? x.x : x.z, sim = k ? x.y : x.w; // offset 1 - k: the partner's
                const float rre = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sre), XCHG, 0xf, 0xf, true));
                const float rim = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(sim), XCHG, 0xf, 0xf, true));
                const int sr = D == 4 ? 2 * (q & 1) + (int)k : (int)k;
                const int r = sr == 0 ? 0 : D - sr;
                const int s = G::H + 2 * (q / D);
                if (k)
                    store_pair11<D, QH>(buf, r, s, rre, kre, rim, kim, sc);
                else
                    store_pair11<D, QH>(buf, r, s, kre, rre, kim, rim, sc);
            }
#else
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
#endif
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
            if constexpr (G::TAIL) { // separate accumulators, single ds_read_b64 (k_fir_mfma11)
#pragma unroll
                for (int t = 0; t < G::TILES; ++t) {
                    const int off = row_base + t * 8 * 32 - (QH - 1) * 32 + g * 8;
                    const f16x4 A0 = *reinterpret_cast<const f16x4*>(ph + off);
                    asm volatile("" ::: "memory");
                    const f16x4 A1 = *reinterpret_cast<const f16x4*>(ph + off + G::PLANE);
                    asm volatile("" ::: "memory");
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
    auto store_tile = [&](int64_t ch, const nf2 (&o)[2 * G::TILES]) {
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK>(out, ch, n_out);
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi)
            buf_store_f2(r, (wave * G::WAVE_OUT + ((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase) * 8, o[oi]);
    };
    // the workgroup's decision for a chunk from its slot set (SGPRs: scalar branches on it)
    struct decision {
        int s;
        bool ex;
    };
    auto decide = [&](int par, int64_t ch) {
        const unsigned m = __builtin_amdgcn_readfirstlane(
            max(max(slot_max[4 * par], slot_max[4 * par + 1]), max(slot_max[4 * par + 2], slot_max[4 * par + 3])));
        const unsigned z = __builtin_amdgcn_readfirstlane(
            min(min(slot_mnz[4 * par], slot_mnz[4 * par + 1]), min(slot_mnz[4 * par + 2], slot_mnz[4 * par + 3])));
        const int s = scale_of(m);
        const bool ex = chunk_needs_exact(m, z, s);
        if (ex && tid == 0 && ch < nchunks) { // to k_fir_exact13 (a vector atomic and a vector store from one lane)
            const unsigned k = blockIdx.x % XQ_N;
            const unsigned i = __hip_atomic_fetch_add(xq + XQ_LINE * k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (i < (unsigned)subcap)
                __hip_atomic_store(xq + XQ_E + k * subcap + i, (unsigned)(ch << 1) | (m >= 0x7f800000u ? 1u : 0u),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return decision{ s, ex };
    };

    // ---- prologue: chunk 0 (+ halo) staged; chunks 1, 2 in flight, chunk 1 reduced
    float4 va[4], vb[4], vc[4];
    float4 ha, hb, hc;
    load13<D, QH>(in, hist_in, L, n_in, chunk_at(0), va, ha);
    {
        unsigned m, z;
        reduce(va, ha, m, z);
        put_halo(stash + G::HP, ha);
        if (lane == 0) {
            slot_max[wave] = m;
            slot_mnz[wave] = z;
        }
    }
    nsh::lds_barrier();
    decision d_cur = decide(0, chunk_at(0));
    if (!d_cur.ex) put_split(lds, stash + G::HP, va, d_cur.s);
    load13<D, QH>(in, hist_in, L, n_in, chunk_at(1), va, ha);
    load13<D, QH>(in, hist_in, L, n_in, chunk_at(2), vb, hb);
    {
        unsigned m, z;
        reduce(va, ha, m, z);
        nsh::lds_barrier(); // slots [0..3] and stash[1] read above
        put_halo(stash, ha);
        if (lane == 0) {
            slot_max[4 + wave] = m;
            slot_mnz[4 + wave] = z;
        }
    }
    nsh::lds_barrier();

    // step i: chunk i+1 (nxt, its halo in stash[i & 1]) split into the other buffer, chunk i filtered
    // from this one, chunk i+2 (nn) reduced and its halo stashed, chunk i+3 requested into ld
    auto step = [&](float4 (&nxt)[4], float4 (&nn)[4], float4& hnn, float4 (&ld)[4], float4& hld, int64_t i) {
        const int pi = (int)(i & 1), pn = pi ^ 1;
        const unsigned char* cur = lds + pi * G::BUF;
        unsigned char* nbuf = lds + pn * G::BUF;
        const decision d_nxt = decide(pn, chunk_at(i + 1));
        load13<D, QH>(in, hist_in, L, n_in, chunk_at(i + 3), ld, hld);
        if (!d_nxt.ex) put_split(nbuf, stash + pi * G::HP, nxt, d_nxt.s);
        if (!d_cur.ex) {
            nf2 o[2 * G::TILES];
            mfma_tile(cur, -(d_cur.s + sh), o);
            store_tile(chunk_at(i), o);
        }
        unsigned m, z;
        reduce(nn, hnn, m, z);
        put_halo(stash + pn * G::HP, hnn);
        if (lane == 0) {
            slot_max[4 * pi + wave] = m;
            slot_mnz[4 * pi + wave] = z;
        }
        d_cur = d_nxt;
        nsh::lds_barrier();
    };
    int64_t i = 0;
    for (; i + 2 < n_steps; i += 3) {
        step(va, vb, hb, vc, hc, i);
        step(vb, vc, hc, va, ha, i + 1);
        step(vc, va, ha, vb, hb, i + 2);
    }
    if (i < n_steps) step(va, vb, hb, vc, hc, i++);
    if (i < n_steps) step(vb, vc, hc, va, ha, i);
}

// The chunks k_fir_mfma13 queued, on the exact forms of k_fir_mfma11: finite -> the exact-fp32 tile
// (filtered undecimated, every D-th output kept), inf/NaN -> the fp32 direct form. A persistent walk
// over the queue (NSH_X12_PER_CU workgroups per CU), one chunk per workgroup step; it zeroes the next
// launch's counters (k_fir_exact12's protocol).
template <int D, int QH>
__global__ __launch_bounds__(256) void k_fir_exact13(const float2* __restrict__ in,
                                                    const float2* __restrict__ hist_in,
                                                    float2* __restrict__ out,
                                                    const float4* __restrict__ timg32, // tile taps [4][TWF]
                                                    const float* __restrict__ taps,
                                                    const unsigned* __restrict__ xq, // this launch's set
                                                    unsigned* __restrict__ xq_next,  // the next launch's set
                                                    int64_t subcap,
                                                    int L,
                                                    int64_t n_out)
{
    using G = geom11x<D, QH>;
    using GF = typename G::GF;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = lane >> 4;
    const int phase = lane & 15;
    if (blockIdx.x == 0 && tid < 64)
        __hip_atomic_store(xq_next + XQ_LINE * tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned incl = __hip_atomic_load(xq + XQ_LINE * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool over = __ballot(incl > (unsigned)subcap) != 0; // lost entries: every chunk again (k_fir_exact12)
    incl = min(incl, (unsigned)subcap);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    const unsigned cnt = over ? (unsigned)((n_out + G::CHUNK - 1) / G::CHUNK) : __builtin_amdgcn_readlane(incl, 63);
    if (cnt == 0) return; // nothing queued (the common case)
    auto entry = [&](unsigned i) {
        if (over) return (i << 1) | 1u; // chunk i, direct form
        const int k = __popcll(__ballot(incl <= i));
        const unsigned start = k ? __shfl(incl, k - 1) : 0u;
        return __hip_atomic_load(xq + XQ_E + k * subcap + (i - start), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    {   // the tile's taps, once per workgroup (read after the first chunk's barrier)
        float4 t32[2];
        nsh_f32t::load_taps<GF>(timg32, t32, tid, G::NT);
        nsh_f32t::put_taps_at<GF>(lds + G::TAPF, t32, tid, G::NT);
    }
    const int64_t n_in = n_out * D;
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    for (unsigned i = blockIdx.x; i < cnt; i += gridDim.x) {
        const unsigned e = entry(i);
        const int64_t ch = (int64_t)(e >> 1);
        if (ch >= nchunks) continue; // never for a queue this launch filled (defensive)
        const bool f32t = !(e & 1u);
        float4 v[4], hv;
        load13<D, QH>(in, hist_in, L, n_in, ch, v, hv);
        auto q_of = [&](int u, int f) { return NSH_V13_CLOAD ? q13<D>(u, f) : (tid + G::NT * u) * D + f; }; // load13's float4
        nsh::lds_barrier(); // the previous chunk's reads of LDS are done
        if (f32t) {
            if (tid < G::HP) nsh_f32t::put<GF>(lds, hv, 2 * tid);
#pragma unroll
            for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
                for (int f = 0; f < D; ++f) nsh_f32t::put<GF>(lds, v[u * D + f], GF::H + 2 * q_of(u, f));
        } else {
            float4* rb = reinterpret_cast<float4*>(lds);
            if (tid < G::HP) rb[tid] = hv;
#pragma unroll
            for (int u = 0; u < G::UNITS; ++u)
#pragma unroll
                for (int f = 0; f < D; ++f) rb[G::HP + q_of(u, f)] = v[u * D + f];
        }
        nsh::lds_barrier();
        nf2 o[2 * G::TILES];
        if (f32t) {
            typedef float f32x4 __attribute__((ext_vector_type(4)));
            f32x4 acc[4];
            nsh_f32t::tile_at<GF, G::QF>(lds, lds + G::TAPF, wave, lane, acc);
            nf2* scr = reinterpret_cast<nf2*>(lds + G::SCR) + wave * G::WAVE_OUT;
            const int ii = lane & 15;
            if (ii % D == 0) {
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int u = 0; u < 2; ++u) scr[(16 * (8 * t + 2 * g + u) + ii) / D] = nf2{ acc[t][2 * u], acc[t][2 * u + 1] };
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int oi = 0; oi < 2 * G::TILES; ++oi) o[oi] = scr[((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase];
        } else if constexpr (D == 4 || NSH_DECIM2_SHARED) {
#pragma unroll 1
            for (int t = 0; t < G::TILES; ++t) {
                nf2 acc[2];
                direct_group<2, 16 * D, D * G::H, D * (G::H - 16)>(
                    reinterpret_cast<const nf2*>(lds), D * G::H + D * (wave * G::WAVE_OUT + (8 * t + 2 * g) * 16 + phase), taps, L, acc);
                if (t == 0) {
                    o[0] = acc[0];
                    o[1] = acc[1];
                } else {
                    o[2 * G::TILES - 2] = acc[0];
                    o[2 * G::TILES - 1] = acc[1];
                }
            }
        } else {
            const float2* raw = reinterpret_cast<const float2*>(lds);
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
        const __amdgpu_buffer_rsrc_t r = chunk_rsrc<G::CHUNK>(out, ch, n_out);
#pragma unroll
        for (int oi = 0; oi < 2 * G::TILES; ++oi)
            buf_store_f2(r, (wave * G::WAVE_OUT + ((oi >> 1) * 8 + 2 * g + (oi & 1)) * 16 + phase) * 8, o[oi]);
    }
}

// The plan's exact queue for stream s: two sets of at least `words` u32 each (stride returned), and
// the set this launch uses (the stream's launch count & 1). Grown (rare: the first call with more
// chunks than any before on this stream) after the stream has drained, so no launch still uses the
// old one; a new queue starts with both sets' counters zero, in stream order.
unsigned* exact_queue(const nsh_fir_plan* p, hipStream_t s, int64_t words, int64_t& stride, int& set, hipError_t& e)
{
    e = hipSuccess;
    std::lock_guard<std::mutex> g(p->xq_mu);
    nsh_fir_plan::xqueue* q = nullptr;
    for (auto& x : p->xq)
        if (x.s == s) q = &x;
    if (!q || q->stride < words) {
        int64_t st = XQ_E + 1024;
        while (st < words) st *= 2;
        if (q) {
            if ((e = hipStreamSynchronize(s)) != hipSuccess) return nullptr;
            (void)hipFree(q->d);
            q->d = nullptr;
            q->stride = 0;
        } else {
            p->xq.push_back({ s, nullptr, 0, 0 });
            q = &p->xq.back();
        }
        unsigned* d = nullptr;
        if ((e = hipMalloc(&d, (size_t)(2 * st) * sizeof(unsigned))) != hipSuccess) return nullptr;
        if ((e = hipMemsetAsync(d, 0, XQ_E * sizeof(unsigned), s)) == hipSuccess)
            e = hipMemsetAsync(d + st, 0, XQ_E * sizeof(unsigned), s);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return nullptr;
        }
        q->d = d;
        q->stride = st;
    }
    stride = q->stride;
    set = (int)(q->launches++ & 1);
    return q->d;
}

// After a failed launch in the k_fir_mfma12 / k_fir_exact12 pair the queue's parity no longer
// matches what ran (the set k_fir_exact12 should have zeroed still holds counts): zero both sets'
// counters in stream order (behind anything the failed call did enqueue) and restart the parity,
// so the next call appends to a clean set.
void xq_reset(const nsh_fir_plan* p, hipStream_t s)
{
    std::lock_guard<std::mutex> g(p->xq_mu);
    for (auto& q : p->xq)
        if (q.s == s && q.d) {
            (void)hipMemsetAsync(q.d, 0, XQ_E * sizeof(unsigned), s);
            (void)hipMemsetAsync(q.d + q.stride, 0, XQ_E * sizeof(unsigned), s);
            q.launches = 0;
        }
}

template <int D, int QH>
int launch_v11(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geom11x<D, QH>;
    if (p->QFT != G::QF) return nsh::fail_msg("nsh_fir_ccf(mfma decim): tile tap image does not match the kernel");
    NSH_CK(set_lds_attr((const void*)k_fir_mfma11<D, QH>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int64_t max_grid = (int64_t)n_cu * 2; // launch_v9's longer grids measured 4-7 % slower here
    const unsigned grid = (unsigned)(nchunks < max_grid ? nchunks : max_grid);
    nsh::launch((k_fir_mfma11<D, QH>), dim3(grid), dim3(G::NT), G::LDS, s, in, hin, hout, out,
                       (const _Float16*)p->fragd8_dev, (const float4*)p->tf32q_dev, (const float*)p->taps_dev, p->L, p->sh8,
                       n_out);
    NSH_CK_LAUNCH("nsh_fir_ccf(mfma decim fp16x2)");
    return 0;
}

// The lockstep walk (k_fir_mfma13 + k_fir_exact13) for decim D, the contiguous walk
// (k_fir_mfma11, exact forms inline) otherwise: bit D of the plan's dec_walk, set at plan creation
// from NSH_DEC_WALK_MASK (environment; default below: D = 2 and 4) -- tests run both walks.
template <int D, int QH>
int launch_v13(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geom11<D, QH>;
    using GX = geom11x<D, QH>;
    if (p->QFT != GX::QF) return nsh::fail_msg("nsh_fir_ccf(mfma decim): tile tap image does not match the kernel");
    NSH_CK(set_lds_attr((const void*)k_fir_mfma13<D, QH>, G::LDS, p->dev));
    NSH_CK(set_lds_attr((const void*)k_fir_exact13<D, QH>, GX::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int n_cu = plan_cus(p);
    const int W = n_cu * p->walk_wgpc / 8 > 0 ? n_cu * p->walk_wgpc / 8 : 1; // one lockstep row per XCD
    const int64_t per_x = (nchunks + 7) / 8;
    const int64_t grid = 8 * (int64_t)W;
    const int64_t steps = (per_x + W - 1) / W;
    const int64_t subcap = xq_subcap(grid) * steps; // a sub-queue's workgroups can queue every chunk they walk
    hipError_t e;
    int64_t stride = 0;
    int set = 0;
    unsigned* xq = exact_queue(p, s, XQ_E + XQ_N * subcap, stride, set, e);
    if (!xq) return nsh::fail(e, "nsh_fir_ccf(mfma decim): exact queue");
    unsigned* cur = xq + set * stride;
    unsigned* nxt = xq + (set ^ 1) * stride;
    const nsh::launch_events t = nsh::take_launch_events(); // one pair over both kernels
    nsh::launch_timed((k_fir_mfma13<D, QH>), dim3((unsigned)grid), dim3(G::NT), G::LDS, s, t.start, (hipEvent_t) nullptr, in,
                      hin, hout, out, (const _Float16*)p->fragd8_dev, cur, subcap, p->L, p->sh8, n_out, per_x);
    if ((e = hipGetLastError()) != hipSuccess) {
        xq_reset(p, s);
        return nsh::fail(e, "nsh_fir_ccf(mfma decim v13)");
    }
    const int64_t xcap = (int64_t)n_cu * NSH_X12_PER_CU;
    nsh::launch_timed((k_fir_exact13<D, QH>), dim3((unsigned)(nchunks < xcap ? nchunks : xcap)), dim3(G::NT), GX::LDS, s,
                      (hipEvent_t) nullptr, t.stop, in, hin, out, (const float4*)p->tf32q_dev, (const float*)p->taps_dev,
                      (const unsigned*)cur, nxt, subcap, p->L, n_out);
    if ((e = hipGetLastError()) != hipSuccess) {
        xq_reset(p, s);
        return nsh::fail(e, "nsh_fir_ccf(mfma decim v13 exact chunks)");
    }
    return 0;
}

template <int D, int QH>
int launch_walk(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
                hipStream_t s)
{
    if (p->dec_walk & (1 << D)) return launch_v13<D, QH>(p, in, hin, hout, out, n_out, s);
    return launch_v11<D, QH>(p, in, hin, hout, out, n_out, s);
}

template <int D>
int launch_dec(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    switch (p->QHD) {
    case 2: return launch_walk<D, 2>(p, in, hin, hout, out, n_out, s);
    case 3: return launch_walk<D, 3>(p, in, hin, hout, out, n_out, s);
    case 4: return launch_walk<D, 4>(p, in, hin, hout, out, n_out, s);
    case 5: return launch_walk<D, 5>(p, in, hin, hout, out, n_out, s);
    case 6: return launch_walk<D, 6>(p, in, hin, hout, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma decim): unsupported tap count");
    }
}

template <int Q>
int launch_v12(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out,
               hipStream_t s)
{
    using G = geom12<Q>;
    NSH_CK(set_lds_attr((const void*)k_fir_mfma12<Q>, G::LDS, p->dev));
    NSH_CK(set_lds_attr((const void*)k_fir_exact12<Q>, G::LDS, p->dev));
    const int64_t nchunks = (n_out + G::CHUNK - 1) / G::CHUNK;
    const int64_t per_x = (nchunks + 7) / 8; // workgroups (= chunks) per XCD
    const int64_t grid = per_x * 8;
    if (grid > 0x7fffffff) return nsh::fail_msg("nsh_fir_ccf(mfma v12): stream too long for one launch");
    hipError_t e;
    const int64_t subcap = xq_subcap(grid);
    int64_t stride = 0;
    int set = 0;
    unsigned* xq = exact_queue(p, s, XQ_E + XQ_N * subcap, stride, set, e);
    if (!xq) return nsh::fail(e, "nsh_fir_ccf(mfma v12): exact queue");
    unsigned* cur = xq + set * stride;
    unsigned* nxt = xq + (set ^ 1) * stride;
    // a timed call is timed as one: start with k_fir_mfma12's dispatch, stop with k_fir_exact12's
    // (the follow-up launch and every exact chunk are inside the pair)
    const nsh::launch_events t = nsh::take_launch_events();
    nsh::launch_timed((k_fir_mfma12<Q>), dim3((unsigned)grid), dim3(G::NT), G::LDS, s, t.start, (hipEvent_t) nullptr, in,
                      hin, hout, out, (const uint4*)p->frag12_dev, cur, p->L, p->sh8, n_out, per_x);
    if ((e = hipGetLastError()) != hipSuccess) {
        xq_reset(p, s);
        return nsh::fail(e, "nsh_fir_ccf(mfma fp16x2 v12)");
    }
    const int64_t xcap = (int64_t)plan_cus(p) * NSH_X12_PER_CU;
    nsh::launch_timed((k_fir_exact12<Q>), dim3((unsigned)(nchunks < xcap ? nchunks : xcap)), dim3(G::NT), G::LDS, s,
                      (hipEvent_t) nullptr, t.stop, in, hin, out, (const float4*)p->tf32q_dev, (const float*)p->taps_dev,
                      (const unsigned*)cur, nxt, subcap, p->L, n_out);
    if ((e = hipGetLastError()) != hipSuccess) {
        xq_reset(p, s);
        return nsh::fail(e, "nsh_fir_ccf(mfma v12 exact chunks)");
    }
    return 0;
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

// the exact-fp32 tile's taps (finite chunks the split cannot hold): R[m] = h[16 QF - 1 - m], QF tap
// blocks of 16 (zero-padded past L), 4 copies shifted by 0..3 floats (nsh_fir_f32_tile.hpp)
static hipError_t f32_tile_image(nsh_fir_plan* p, int QF)
{
    const int TWF = 16 * QF + 16, P = 16 * QF - 1;
    std::vector<float> img((size_t)4 * TWF, 0.f);
    for (int d = 0; d < 4; ++d)
        for (int k = 0; k < TWF; ++k) {
            const int t = P - (k + d);
            img[(size_t)d * TWF + k] = (t >= 0 && t < p->L) ? p->taps_host[t] : 0.f;
        }
    p->QFT = QF;
    hipError_t e = hipMalloc(&p->tf32q_dev, img.size() * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(p->tf32q_dev, img.data(), img.size() * sizeof(float), hipMemcpyHostToDevice);
    return e;
}

// bit D: decim D on the lockstep walk (k_fir_mfma13) -- D = 4 since round 5 (r05b), D = 2 since its
// whole-line loads (1.6 % faster, also with exact chunks every 4th / 64th chunk, bit-identical on
// finite input, r05zzg, r05zzh); 0 selects the contiguous walk k_fir_mfma11 (tests run both)
#ifndef NSH_DEC_WALK_MASK
#define NSH_DEC_WALK_MASK 20
#endif
int nsh_fir_mfma_prepare_decim(nsh_fir_plan* p)
{
    const char* wm = std::getenv("NSH_DEC_WALK_MASK");
    p->dec_walk = wm && *wm ? std::atoi(wm) : NSH_DEC_WALK_MASK;
    const char* wg = std::getenv("NSH_WALK_WGPC"); // probes: resident workgroups per CU of the walk
    p->walk_wgpc = wg && std::atoi(wg) >= 1 && std::atoi(wg) <= 4 ? std::atoi(wg) : 2;
    // polyphase taps h'_0[j] = h[D j], h'_r[j] = h[D (j - 1) + r] (r >= 1, j >= 1)
    const int D = p->D, QH = decim_qh(p), KS = QH / 2;
    const bool tail = QH % 2;
    p->QHD = QH;
    auto tap = [&](int r, int j) -> float {
        const int k = r == 0 ? D * j : (j >= 1 ? D * (j - 1) + r : -1);
        return (k >= 0 && k < p->L) ? p->taps_host[k] : 0.f;
    };
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
    NSH_CK(f32_tile_image(p, D * (QH - 1) + 1)); // geom11x::QF: the whole D H-sample halo
    return 0;
}

int nsh_fir_mfma_prepare(nsh_fir_plan* p)
{
    if (p->D > 1) return nsh_fir_mfma_prepare_decim(p);
    const int Q = (p->L + 30) / 32 + 1;
    p->Q = Q;
    p->S = 2 * Q;
    // taps scaled by 2^sh8 (max |h| * 2^sh8 in [2^14, 2^15)) and split into two fp16 terms (RNE). A
    // tap far below the largest (e.g. firwin's ~1e-18 taps at the sinc zeros) lands in fp16's
    // subnormal range or flushes: it is then exact to 2^-39 of the largest tap, which moves an
    // output by at most 2^-39 max|h| sum|x|, far below fp32's own rounding of the sum. So every
    // finite tap set qualifies.
    unsigned maxbits = 0;
    for (float t : p->taps_host) {
        unsigned u;
        std::memcpy(&u, &t, 4);
        maxbits = std::max(maxbits, u & 0x7fffffffu);
    }
    const int sh = 141 - (int)(maxbits >> 23);
    p->sh8 = sh;
    {
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
    }
    NSH_CK(f32_tile_image(p, 2 * Q - 1)); // k_fir_mfma12's tile: v12's 32 (Q - 1)-sample halo
    return 0;
}

std::string nsh_fir_mfma_kernel_name(const nsh_fir_plan* p)
{
    auto t = [](const char* k, int a, int b = -1) {
        return std::string(k) + "<" + std::to_string(a) + (b >= 0 ? "," + std::to_string(b) : std::string()) + ">";
    };
    if (p->D > 1) return t((p->dec_walk & (1 << p->D)) ? "k_fir_mfma13" : "k_fir_mfma11", p->D, p->QHD);
    return t("k_fir_mfma12", p->Q);
}

int nsh_fir_mfma_run(const nsh_fir_plan* p, const float2* in, const float2* hist_in, float2* hist_out, float2* out, int64_t n_out, hipStream_t s)
{
    if (p->D == 2) return launch_dec<2>(p, in, hist_in, hist_out, out, n_out, s);
    if (p->D == 4) return launch_dec<4>(p, in, hist_in, hist_out, out, n_out, s);
    switch (p->Q) {
    case 1: return launch_v12<1>(p, in, hist_in, hist_out, out, n_out, s);
    case 2: return launch_v12<2>(p, in, hist_in, hist_out, out, n_out, s);
    case 3: return launch_v12<3>(p, in, hist_in, hist_out, out, n_out, s);
    case 4: return launch_v12<4>(p, in, hist_in, hist_out, out, n_out, s);
    case 5: return launch_v12<5>(p, in, hist_in, hist_out, out, n_out, s);
    case 6: return launch_v12<6>(p, in, hist_in, hist_out, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(mfma): unsupported tap count");
    }
}
