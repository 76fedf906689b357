// libnsh_hip.so: fir_filter_ccf (complex fp32 stream, real fp32 taps, optional decimation).
//
//   y[m] = sum_{k<L} h[k] * x[m*D - k]          (GNU Radio fir_filter_ccf convention with
//                                                 zero initial history)
//
// The reference has no FIR block; its block API has no history
// (runtime/include/gnuradio/sync_block.hpp:36-86), so each call receives the L-1 samples
// that precede in[0] (hist_in) and hands the next call its own (hist_out).
//
// Two algorithms (nsh_fir_algo):
//  * DIRECT -- fp32 VALU direct form. A 256-thread workgroup stages its input window
//    (T-1)*D + Lp samples in LDS (one HBM read per sample), each thread keeps R
//    consecutive outputs in registers and slides an 8-tap register window over the
//    staged samples; taps come from the scalar cache (s_load, uniform index). LDS rows
//    are padded by one sample every R*D samples so the per-lane ds_read_b64 of the window
//    is bank-conflict-free. Exact fp32 products, fp32 accumulation in tap order.
//  * MFMA -- split-precision Toeplitz MFMA (nsh_fir_mfma.hip): decim 1 on 32-sample blocks as
//    scaled fp16x2 (k_fir_mfma12), decim 2 and 4 as the polyphase fp16x2 form (k_fir_mfma11).
//  * MFMA_F32 -- exact fp32 Toeplitz MFMA (nsh_fir_f32.hip); PFFT -- decim 8 / 16 by
//    polyphase-FFT overlap-save (nsh_fir_pfft.hip). Decim 8 otherwise: DIRECT.
//  NSH_FIR_MFMA16 / NSH_FIR_MFMA_BF16X3 name kernels retired in round 4 (DESIGN.md section 4
//  keeps their measurements): plan creation refuses them.
#include "nsh_common.hpp"

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "nsh_fir_plan.hpp"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float2 virt(const float2* __restrict__ in,
                                       const float2* __restrict__ hist,
                                       int64_t g,
                                       int64_t n_in,
                                       int L)
{
    if (g >= 0) return g < n_in ? in[g] : make_float2(0.f, 0.f);
    if (g >= -(int64_t)(L - 1)) return hist ? hist[g + (L - 1)] : make_float2(0.f, 0.f); // null: zeros
    return make_float2(0.f, 0.f);
}

template <int D, int R>
__global__ __launch_bounds__(kThreads) void k_fir_direct(const float2* __restrict__ in,
                                                         const float2* __restrict__ hist_in,
                                                         float2* __restrict__ hist_out,
                                                         float2* __restrict__ out,
                                                         const float* __restrict__ taps, // Lp, zero padded
                                                         int L,
                                                         int Lp,
                                                         int64_t n_out)
{
    extern __shared__ __attribute__((aligned(16))) float2 xs[];
    constexpr int T = kThreads * R;          // outputs per workgroup
    constexpr int W = 8 + (R - 1) * D;       // register window (samples)
    constexpr int PAD = R * D;               // one pad sample every PAD samples
    const int tid = threadIdx.x;
    const int64_t n_in = n_out * D;
    const int64_t m0 = (int64_t)blockIdx.x * T;
    const int64_t g0 = m0 * D - (Lp - 1);    // global index of staged sample 0
    const int count = (T - 1) * D + Lp;

    for (int i = tid; i < count; i += kThreads) xs[i + i / PAD] = virt(in, hist_in, g0 + i, n_in, L);

    if (blockIdx.x == 0) { // history for the next call: the L-1 samples before in[n_in]
        for (int j = tid; j < L - 1; j += kThreads) hist_out[j] = virt(in, hist_in, n_in - (L - 1) + j, n_in, L);
    }
    __syncthreads();

    float2 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = make_float2(0.f, 0.f);

    // window w[o] = xs[t*R*D + Lp - 8 - 8*kb + o]
    int base = tid * R * D + Lp - 8;
    float2 w[W];
#pragma unroll
    for (int o = 0; o < W; ++o) {
        const int s = base + o;
        w[o] = xs[s + s / PAD];
    }
    // The last block's padded taps (k >= L) are skipped, not multiplied: 0 x inf / NaN would
    // put a NaN where the L-tap sum has none (a sample L or more back is outside the window).
    const int nkb = Lp / 8;
    for (int kb = 0; kb < nkb; ++kb) {
        const int jn = kb + 1 < nkb ? 8 : L - 8 * kb; // uniform
        float h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = taps[8 * kb + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j >= jn) break;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float2 x = w[r * D + 7 - j];
                acc[r].x = __builtin_fmaf(h[j], x.x, acc[r].x);
                acc[r].y = __builtin_fmaf(h[j], x.y, acc[r].y);
            }
        }
        if (kb + 1 < nkb) {
#pragma unroll
            for (int o = W - 1; o >= 8; --o) w[o] = w[o - 8];
            base -= 8;
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                const int s = base + o;
                w[o] = xs[s + s / PAD];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t m = m0 + (int64_t)tid * R + r;
        if (m < n_out) out[m] = acc[r];
    }
}

template <int D, int R>
int launch_direct(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out, hipStream_t s)
{
    constexpr int T = kThreads * R;
    const int count = (T - 1) * D + p->Lp;
    const size_t lds = (size_t)(count + count / (R * D) + 1) * sizeof(float2);
    const int64_t grid = (n_out + T - 1) / T;
    if (grid > 0x7fffffff) return nsh::fail_msg("nsh_fir_ccf: too many outputs for one call");
    nsh::launch((k_fir_direct<D, R>), dim3((unsigned)grid), dim3(kThreads), lds, s,
                       in, hin, hout, out, p->taps_dev, p->L, p->Lp, n_out);
    NSH_CK_LAUNCH("nsh_fir_ccf(direct)");
    return 0;
}

// History-only update for n_out == 0 calls is a no-op: no input consumed.
int run_direct(const nsh_fir_plan* p, const float2* in, const float2* hin, float2* hout, float2* out, int64_t n_out, hipStream_t s)
{
    switch (p->D) {
    case 1: return launch_direct<1, 8>(p, in, hin, hout, out, n_out, s);
    case 2: return launch_direct<2, 8>(p, in, hin, hout, out, n_out, s);
    case 4: return launch_direct<4, 4>(p, in, hin, hout, out, n_out, s);
    case 8: return launch_direct<8, 2>(p, in, hin, hout, out, n_out, s);
    default: return nsh::fail_msg("nsh_fir_ccf(direct): decimation must be 1, 2, 4 or 8");
    }
}

} // namespace

extern "C" {

int nsh_fir_plan_create(int dev, const float* taps_host, int ntaps, int decim, int algo, void** plan)
{
    if (ntaps < 1 || ntaps > 4096) return nsh::fail_msg("nsh_fir_plan_create: ntaps must be in [1, 4096]");
    if (decim != 1 && decim != 2 && decim != 4 && decim != 8 && decim != 16)
        return nsh::fail_msg("nsh_fir_plan_create: decimation must be 1, 2, 4, 8 or 16");
    NSH_CK(hipSetDevice(dev));
    auto* p = new nsh_fir_plan();
    p->dev = dev;
    if (hipDeviceGetAttribute(&p->n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) p->n_cu = 256;
    p->L = ntaps;
    p->D = decim;
    p->Lp = (ntaps + 7) / 8 * 8;
    p->taps_host.assign(taps_host, taps_host + ntaps);
    std::vector<float> padded(p->Lp, 0.f);
    std::copy(taps_host, taps_host + ntaps, padded.begin());
    hipError_t e = hipMalloc(&p->taps_dev, p->Lp * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(p->taps_dev, padded.data(), p->Lp * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        delete p;
        return nsh::fail(e, "nsh_fir_plan_create: taps upload");
    }
    if (algo < NSH_FIR_AUTO || algo > NSH_FIR_PFFT) {
        (void)hipFree(p->taps_dev);
        delete p;
        return nsh::fail_msg("nsh_fir_plan_create: unknown algorithm");
    }
    if (algo == NSH_FIR_MFMA16 || algo == NSH_FIR_MFMA_BF16X3) {
        (void)hipFree(p->taps_dev);
        delete p;
        return nsh::fail_msg("nsh_fir_plan_create: the MFMA16 / MFMA_BF16X3 kernels were retired (use NSH_FIR_MFMA or "
                             "NSH_FIR_MFMA_F32)");
    }
    int resolved = algo;
    // decim 8 and 16: the polyphase-FFT kernel (k_fir_pfft; 2x the direct form at 127 taps, 5x at
    // 511) when the filter fits its 256 overlap rows, else the direct form (decim 8 only)
    const bool pfft_ok = (decim == 8 || decim == 16) && (ntaps - 1 + decim - 1) / decim <= 256 &&
                         std::all_of(taps_host, taps_host + ntaps, [](float v) { return std::isfinite(v); });
    if (algo == NSH_FIR_AUTO)
        resolved = pfft_ok ? NSH_FIR_PFFT : (nsh_fir_mfma_supported(p) ? NSH_FIR_MFMA : NSH_FIR_DIRECT);
    if ((resolved == NSH_FIR_PFFT && !pfft_ok) || (decim == 16 && resolved != NSH_FIR_PFFT)) {
        (void)hipFree(p->taps_dev);
        delete p;
        return nsh::fail_msg("nsh_fir_plan_create: PFFT needs decim 8 or 16, finite taps and ntaps <= 256 decim + 1; "
                             "decim 16 needs PFFT");
    }
    if (resolved == NSH_FIR_PFFT) {
        const float* tp[1] = { taps_host };
        const int nt[1] = { ntaps }, dc[1] = { decim };
        const int rc = nsh_fir_cascade_plan_create(dev, tp, nt, dc, 1, &p->casc);
        if (rc) {
            (void)hipFree(p->taps_dev);
            delete p;
            return rc;
        }
        p->algo = NSH_FIR_PFFT;
        p->kernel = nsh_fir_cascade_kernel(p->casc);
        *plan = p;
        return 0;
    }
    if (resolved == NSH_FIR_MFMA_F32) {
        const int rc = nsh_fir_f32_supported(p) ? nsh_fir_f32_prepare(p)
                                                : nsh::fail_msg("nsh_fir_plan_create: MFMA_F32 form needs decim 1, finite taps and ntaps <= 257");
        if (rc) {
            if (p->tf32_dev) (void)hipFree(p->tf32_dev);
            (void)hipFree(p->taps_dev);
            delete p;
            return rc;
        }
    }
    if (resolved == NSH_FIR_MFMA) {
        if (!nsh_fir_mfma_supported(p)) {
            (void)hipFree(p->taps_dev);
            delete p;
            return nsh::fail_msg("nsh_fir_plan_create: MFMA form needs finite taps and decim 1 with ntaps <= 161, "
                                 "decim 2 with ntaps <= 160 or decim 4 with ntaps <= 320");
        }
        const int rc = nsh_fir_mfma_prepare(p);
        if (rc) {
            (void)hipFree(p->taps_dev);
            delete p;
            return rc;
        }
    }
    p->algo = resolved;
    if (resolved == NSH_FIR_DIRECT) {
        static const int R[9] = { 0, 8, 8, 0, 4, 0, 0, 0, 2 };
        p->kernel = "k_fir_direct<" + std::to_string(p->D) + "," + std::to_string(R[p->D]) + ">";
    } else if (resolved == NSH_FIR_MFMA_F32) {
        // named by nsh_fir_f32_prepare
    } else {
        p->kernel = nsh_fir_mfma_kernel_name(p);
    }
    *plan = p;
    return 0;
}

int nsh_fir_plan_destroy(void* plan)
{
    auto* p = static_cast<nsh_fir_plan*>(plan);
    if (!p) return 0;
    if (p->taps_dev) (void)hipFree(p->taps_dev);
    if (p->frag12_dev) (void)hipFree(p->frag12_dev);
    if (p->tf32_dev) (void)hipFree(p->tf32_dev);
    if (p->tf32q_dev) (void)hipFree(p->tf32q_dev);
    if (p->fragd8_dev) (void)hipFree(p->fragd8_dev);
    if (p->casc) nsh_fir_cascade_plan_destroy(p->casc);
    for (auto& q : p->xq) (void)hipFree(q.d);
    delete p;
    return 0;
}

int nsh_fir_plan_algo(void* plan) { return plan ? static_cast<nsh_fir_plan*>(plan)->algo : 0; }
const char* nsh_fir_plan_kernel(void* plan) { return plan ? static_cast<nsh_fir_plan*>(plan)->kernel.c_str() : ""; }

int nsh_fir_ccf(void* plan, const float* in, const float* hist_in, float* hist_out, float* out, int64_t n_out, void* stream)
{
    nsh::launch_events_guard timing_guard; // the armed event pair never outlives this call
    auto* p = static_cast<nsh_fir_plan*>(plan);
    if (!p) return nsh::fail_msg("nsh_fir_ccf: null plan");
    if (n_out <= 0) return 0;
    if (!in || !out) return nsh::fail_msg("nsh_fir_ccf: null input or output");
    if (hist_in == hist_out && p->L > 1) return nsh::fail_msg("nsh_fir_ccf: hist_out must not alias hist_in");
    hipStream_t s = nsh::S(stream);
    if (p->algo == NSH_FIR_PFFT) return nsh_fir_cascade_ccf(p->casc, in, hist_in, hist_out, out, n_out, stream);
    // every kernel but the polyphase-FFT one writes the next call's history unconditionally
    if (!hist_out && p->L > 1) return nsh::fail_msg("nsh_fir_ccf: hist_out is required (ntaps-1 samples)");
    if (p->algo == NSH_FIR_MFMA)
        return nsh_fir_mfma_run(p, (const float2*)in, (const float2*)hist_in, (float2*)hist_out, (float2*)out, n_out, s);
    if (p->algo == NSH_FIR_MFMA_F32)
        return nsh_fir_f32_run(p, (const float2*)in, (const float2*)hist_in, (float2*)hist_out, (float2*)out, n_out, s);
    return run_direct(p, (const float2*)in, (const float2*)hist_in, (float2*)hist_out, (float2*)out, n_out, s);
}

} // extern "C"
