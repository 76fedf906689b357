/*
 * nsh_oracle.c -- CPU ORACLE for the newsched block-execution hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker. The product path
 * (newsched_amd/) never links, loads or calls it, and has no CPU fallback.
 *
 * Parity status:
 *   copy / multiply_const_cc / multiply_const_ff: pinned by the reference's own test
 *     vectors (schedulers/mt/test/qa_scheduler_mt.cpp:79-135 BlockFanout,
 *     qa_block_grouping.cpp:15-66, test/cuda/qa_scheduler_mt_cuda_copy.cpp:20-86 CudaCopy*);
 *     non-identity constants follow the std::complex / VOLK generic formula
 *     (blocklib/blocks/lib/multiply_const.cpp:33-46 -> volk_32fc_s32fc_multiply_32fc,
 *     VOLK v2.2.1 per .github/workflows/build_and_test.yml:18, not vendored).
 *   fir_filter_ccf (+decim), fft 1024, add_cc, multiply_cc, channelizer: ABSENT from the
 *     reference, so reference parity is UNPINNED; these restate the GNU
 *     Radio conventions of SURVEY.md §8a a19 and are pinned instead to scipy.signal.lfilter
 *     and numpy.fft fixtures generated in this container (oracle/gen_golden.py ->
 *     tests/golden/).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; contraction off so products round
 * exactly as the reference's non-FMA VOLK kernels do).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* Counter-based synthetic stream, BASELINE.md §2: x[i] = (u(2i), u(2i+1)),
 * u(j) = ((splitmix64(seed ^ j) >> 40) * 2^-23) - 1, exactly representable in fp32. */
static uint64_t splitmix64(uint64_t x)
{
    uint64_t z;
    x += 0x9E3779B97F4A7C15ull;
    z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_synth_cf32(float* out, int64_t n, uint64_t first_index, uint64_t seed)
{
    for (int64_t i = 0; i < n; ++i) {
        const uint64_t g = 2 * (first_index + (uint64_t)i);
        out[2 * i] = (float)(int)(splitmix64(seed ^ g) >> 40) * (1.0f / 8388608.0f) - 1.0f;
        out[2 * i + 1] = (float)(int)(splitmix64(seed ^ (g + 1)) >> 40) * (1.0f / 8388608.0f) - 1.0f;
    }
}

/* blocks::copy::work -- memcpy of n_items*itemsize (blocklib/blocks/include/gnuradio/
 * blocklib/blocks/copy.hpp:33-44). */
void orc_copy(const void* in, void* out, size_t bytes) { memcpy(out, in, bytes); }

/* blocks::multiply_const<gr_complex>::work (blocklib/blocks/lib/multiply_const.cpp:33-46):
 * out[i] = in[i] * k, std::complex<float> product = (ar kr - ai ki, ar ki + ai kr). */
void orc_mul_const_cc(const float* in, float* out, int64_t n, float kr, float ki)
{
    for (int64_t i = 0; i < n; ++i) {
        const float ar = in[2 * i], ai = in[2 * i + 1];
        const float p0 = ar * kr, p1 = ai * ki, p2 = ar * ki, p3 = ai * kr;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}

/* blocks::multiply_const<float>::work (multiply_const.cpp:17-31). */
void orc_mul_const_ff(const float* in, float* out, int64_t n, float k)
{
    for (int64_t i = 0; i < n; ++i) out[i] = in[i] * k;
}

/* m chained multiply_const_cc blocks (BASELINE config C2), each stage rounded. */
void orc_mul_const_chain_cc(const float* in, float* out, int64_t n, const float* k, int m)
{
    if (in != out) memcpy(out, in, (size_t)n * 8);
    for (int s = 0; s < m; ++s) orc_mul_const_cc(out, out, n, k[2 * s], k[2 * s + 1]);
}

/* add_cc / multiply_cc: GNU Radio add_cc, multiply_cc (no reference counterpart). */
void orc_add_cc(const float* a, const float* b, float* out, int64_t n)
{
    for (int64_t i = 0; i < 2 * n; ++i) out[i] = a[i] + b[i];
}
void orc_mul_cc(const float* a, const float* b, float* out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        const float ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
        const float p0 = ar * br, p1 = ai * bi, p2 = ar * bi, p3 = ai * br;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}

/* fir_filter_ccf with decimation D, GNU Radio convention:
 *   y[m] = sum_{k<L} h[k] x[m D - k], x[<0] taken from hist (L-1 samples, hist[L-2] is
 *   the sample just before x[0]); accumulated in double, rounded once to fp32.
 * n_out outputs consume n_out*D inputs; hist_out (may be NULL) receives the L-1 samples
 * preceding the next call's x[0]. */
void orc_fir_ccf(const float* x, const float* hist, float* hist_out, float* y, int64_t n_out,
                 const float* h, int L, int D)
{
    const int64_t n_in = n_out * D;
    for (int64_t m = 0; m < n_out; ++m) {
        double ar = 0.0, ai = 0.0;
        for (int k = 0; k < L; ++k) {
            const int64_t g = m * D - k;
            float xr, xi;
            if (g >= 0) {
                xr = x[2 * g];
                xi = x[2 * g + 1];
            } else if (hist) {
                xr = hist[2 * (g + L - 1)];
                xi = hist[2 * (g + L - 1) + 1];
            } else {
                xr = 0.f;
                xi = 0.f;
            }
            ar += (double)h[k] * (double)xr;
            ai += (double)h[k] * (double)xi;
        }
        y[2 * m] = (float)ar;
        y[2 * m + 1] = (float)ai;
    }
    if (hist_out) {
        for (int j = 0; j < L - 1; ++j) {
            const int64_t g = n_in - (L - 1) + j;
            float xr = 0.f, xi = 0.f;
            if (g >= 0) {
                xr = x[2 * g];
                xi = x[2 * g + 1];
            } else if (hist) {
                xr = hist[2 * (g + L - 1)];
                xi = hist[2 * (g + L - 1) + 1];
            }
            hist_out[2 * j] = xr;
            hist_out[2 * j + 1] = xi;
        }
    }
}

/* 1024-point DFT in double (iterative radix-2), forward e^{-i}, inverse e^{+i},
 * unnormalised both ways. One frame at a time. */
static void dft1024_d(const float* in, double* re, double* im, int inverse)
{
    const int N = 1024;
    for (int i = 0; i < N; ++i) {
        int r = 0;
        for (int b = 0; b < 10; ++b)
            if (i & (1 << b)) r |= 1 << (9 - b);
        re[r] = in[2 * i];
        im[r] = in[2 * i + 1];
    }
    for (int len = 2; len <= N; len <<= 1) {
        const double ang = (inverse ? 2.0 : -2.0) * M_PI / len;
        for (int i = 0; i < N; i += len)
            for (int j = 0; j < len / 2; ++j) {
                const double wr = cos(ang * j), wi = sin(ang * j);
                const int a = i + j, b = i + j + len / 2;
                const double tr = re[b] * wr - im[b] * wi, ti = re[b] * wi + im[b] * wr;
                re[b] = re[a] - tr;
                im[b] = im[a] - ti;
                re[a] += tr;
                im[a] += ti;
            }
    }
}

void orc_fft1024(const float* in, float* out, int64_t nframes, int inverse)
{
    double re[1024], im[1024];
    for (int64_t f = 0; f < nframes; ++f) {
        dft1024_d(in + f * 2048, re, im, inverse);
        for (int i = 0; i < 1024; ++i) {
            out[f * 2048 + 2 * i] = (float)re[i];
            out[f * 2048 + 2 * i + 1] = (float)im[i];
        }
    }
}

/* fft1024 -> multiply by w (complex) -> ifft1024, in double between the transforms. */
void orc_channelizer1024(const float* in, float* out, const float* w, int64_t nframes)
{
    double re[1024], im[1024], re2[1024], im2[1024];
    for (int64_t f = 0; f < nframes; ++f) {
        dft1024_d(in + f * 2048, re, im, 0);
        for (int i = 0; i < 1024; ++i) { /* spectrum * w, bit-reversed for the inverse */
            int r = 0;
            for (int b = 0; b < 10; ++b)
                if (i & (1 << b)) r |= 1 << (9 - b);
            re2[r] = re[i] * w[2 * i] - im[i] * w[2 * i + 1];
            im2[r] = re[i] * w[2 * i + 1] + im[i] * w[2 * i];
        }
        for (int len = 2; len <= 1024; len <<= 1) {
            const double ang = 2.0 * M_PI / len;
            for (int i = 0; i < 1024; i += len)
                for (int j = 0; j < len / 2; ++j) {
                    const double wr = cos(ang * j), wi = sin(ang * j);
                    const int a = i + j, b = i + j + len / 2;
                    const double tr = re2[b] * wr - im2[b] * wi, ti = re2[b] * wi + im2[b] * wr;
                    re2[b] = re2[a] - tr;
                    im2[b] = im2[a] - ti;
                    re2[a] += tr;
                    im2[a] += ti;
                }
        }
        for (int i = 0; i < 1024; ++i) {
            out[f * 2048 + 2 * i] = (float)re2[i];
            out[f * 2048 + 2 * i + 1] = (float)im2[i];
        }
    }
}
