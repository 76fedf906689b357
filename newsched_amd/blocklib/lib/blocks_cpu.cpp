// CPU block implementations (reference blocklib/blocks/lib/*.cpp semantics).
#include <gnuradio/blocklib/blocks/arith.hpp>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/multiply_const.hpp>

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace gr {
namespace blocks {

namespace {
// Function multiversioning by ISA FEATURE. GCC's target_clones("arch=skylake-avx512", "arch=haswell",
// "default") -- what this file used up to round 5 -- dispatches "arch=" clones with
// __builtin_cpu_is(<model>), which is false on every AMD EPYC and on Intel parts GCC does not name
// that way (this container's Xeon included), so the baseline ran the SSE2 default clone. The clones
// below are chosen with __builtin_cpu_supports on the features each one is compiled for.
enum class isa { avx512, avx2, base };
isa detect_isa()
{
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("fma")) return isa::avx512;
    if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return isa::avx2;
    return isa::base;
}
const isa g_isa = detect_isa();
#define NSR_AVX512 __attribute__((target("avx512f,avx512vl,avx512dq,avx512bw,avx2,fma")))
#define NSR_AVX2 __attribute__((target("avx2,fma")))

// (ar kr - ai ki, ar ki + ai kr) with every product rounded: FMA contraction is switched
// off for these two functions only, to match the reference formula bit for bit.
#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
static inline __attribute__((always_inline)) void cmul_const_body(const float* in, float* out, size_t n, float kr, float ki)
{
    for (size_t i = 0; i < n; ++i) {
        const float ar = in[2 * i], ai = in[2 * i + 1];
        const float p0 = ar * kr, p1 = ai * ki, p2 = ar * ki, p3 = ai * kr;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}
static inline __attribute__((always_inline)) void cmul_vec_body(const float* a, const float* b, float* out, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        const float ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
        const float p0 = ar * br, p1 = ai * bi, p2 = ar * bi, p3 = ai * br;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}
NSR_AVX512 void cmul_const_avx512(const float* in, float* out, size_t n, float kr, float ki) { cmul_const_body(in, out, n, kr, ki); }
NSR_AVX2 void cmul_const_avx2(const float* in, float* out, size_t n, float kr, float ki) { cmul_const_body(in, out, n, kr, ki); }
void cmul_const_base(const float* in, float* out, size_t n, float kr, float ki) { cmul_const_body(in, out, n, kr, ki); }
NSR_AVX512 void cmul_vec_avx512(const float* a, const float* b, float* out, size_t n) { cmul_vec_body(a, b, out, n); }
NSR_AVX2 void cmul_vec_avx2(const float* a, const float* b, float* out, size_t n) { cmul_vec_body(a, b, out, n); }
void cmul_vec_base(const float* a, const float* b, float* out, size_t n) { cmul_vec_body(a, b, out, n); }
#pragma GCC pop_options

void cmul_const(const float* in, float* out, size_t n, float kr, float ki)
{
    switch (g_isa) {
    case isa::avx512: return cmul_const_avx512(in, out, n, kr, ki);
    case isa::avx2: return cmul_const_avx2(in, out, n, kr, ki);
    default: return cmul_const_base(in, out, n, kr, ki);
    }
}
void cmul_vec(const float* a, const float* b, float* out, size_t n)
{
    switch (g_isa) {
    case isa::avx512: return cmul_vec_avx512(a, b, out, n);
    case isa::avx2: return cmul_vec_avx2(a, b, out, n);
    default: return cmul_vec_base(a, b, out, n);
    }
}

// Decim-1 rows: NV x 8 complex outputs (NV vectors of 16 interleaved floats) per step, fp32
// accumulation: out[m] = sum_k h[k] * x[m - k], x = ext shifted by L-1. The taps go by residue
// rho = k mod 8: tap rho + 8t at output vector r reads the input vector W[r - t] (one vector = 8
// complex samples = the 8-tap stride), so for one residue each input vector is loaded ONCE, aligned
// to the 8-sample grid of its residue, and feeds up to NV FMAs from a rolling window of NV
// registers -- instead of one cache-line-splitting load per FMA. NV = 8 on AVX-512 (two FMA
// pipes x four cycles of latency), 4 on AVX2 (the same registers in 256-bit halves).
typedef float v16f __attribute__((vector_size(64)));

template <int NV, int P>
static inline __attribute__((always_inline)) void fir_step(v16f* a, v16f* w, float hk)
{
    for (int r = 0; r < NV; ++r) a[r] += hk * w[(r - P + 8 * NV) % NV];
}

template <int NV>
static inline __attribute__((always_inline)) void fir_rows_body(const float* ext, const float* h, int L, int D, float* out,
                                                                size_t n_out)
{
    size_t m = 0;
    if (D == 1) {
        for (; m + 8 * NV <= n_out; m += 8 * NV) {
            v16f a[NV] = {};
            const float* base = ext + 2 * (m + (size_t)(L - 1));
            for (int rho = 0; rho < 8 && rho < L; ++rho) {
                const float* W = base - 2 * rho; // W[j] = W + 16 j
                const int T = (L - rho + 7) / 8;  // taps rho, rho + 8, ... < L
                v16f w[NV];                       // W[j] in slot j mod NV
                for (int r = 0; r < NV; ++r) std::memcpy(&w[r], W + 16 * r, 64);
                // step t: a[r] += h[rho + 8t] W[r - t]; then W[-(t+1)] replaces W[NV-1-t]
#define NSR_FIR_STEP(P)                                                                      \
    if (t + P < T) {                                                                         \
        fir_step<NV, P % NV>(a, w, h[rho + 8 * (t + P)]);                                    \
        if (t + P + 1 < T) std::memcpy(&w[(NV - 1 - P % NV) % NV], W - 16 * (t + P + 1), 64); \
    }
                for (int t = 0; t < T; t += 8) {
                    NSR_FIR_STEP(0) NSR_FIR_STEP(1) NSR_FIR_STEP(2) NSR_FIR_STEP(3)
                    NSR_FIR_STEP(4) NSR_FIR_STEP(5) NSR_FIR_STEP(6) NSR_FIR_STEP(7)
                }
#undef NSR_FIR_STEP
            }
            for (int r = 0; r < NV; ++r) std::memcpy(out + 2 * m + 16 * r, &a[r], 64);
        }
    }
    for (; m < n_out; ++m) {
        float ar = 0.f, ai = 0.f;
        for (int k = 0; k < L; ++k) {
            const float* x = ext + 2 * (m * (size_t)D + (size_t)(L - 1 - k));
            ar += h[k] * x[0];
            ai += h[k] * x[1];
        }
        out[2 * m] = ar;
        out[2 * m + 1] = ai;
    }
}
NSR_AVX512 void fir_rows_avx512(const float* ext, const float* h, int L, int D, float* out, size_t n)
{
    fir_rows_body<8>(ext, h, L, D, out, n);
}
NSR_AVX2 void fir_rows_avx2(const float* ext, const float* h, int L, int D, float* out, size_t n)
{
    fir_rows_body<4>(ext, h, L, D, out, n);
}
void fir_rows_base(const float* ext, const float* h, int L, int D, float* out, size_t n) { fir_rows_body<4>(ext, h, L, D, out, n); }
void fir_rows(const float* ext, const float* h, int L, int D, float* out, size_t n_out)
{
    switch (g_isa) {
    case isa::avx512: return fir_rows_avx512(ext, h, L, D, out, n_out);
    case isa::avx2: return fir_rows_avx2(ext, h, L, D, out, n_out);
    default: return fir_rows_base(ext, h, L, D, out, n_out);
    }
}
} // namespace

template <class T>
work_return_code_t multiply_const<T>::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const T* iptr = static_cast<const T*>(in[0].buffer->read_ptr());
    T* optr = static_cast<T*>(out[0].buffer->write_ptr());
    const size_t n = (size_t)out[0].n_items * d_vlen;
    if constexpr (std::is_same_v<T, gr_complex>) {
        cmul_const(reinterpret_cast<const float*>(iptr), reinterpret_cast<float*>(optr), n, d_k.real(), d_k.imag());
    } else {
        for (size_t i = 0; i < n; ++i) optr[i] = iptr[i] * d_k;
    }
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}
template class multiply_const<int16_t>;
template class multiply_const<int32_t>;
template class multiply_const<float>;
template class multiply_const<gr_complex>;

template <int OP>
work_return_code_t arith_cc<OP>::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const size_t n = (size_t)out[0].n_items * _vlen;
    float* o = static_cast<float*>(out[0].buffer->write_ptr());
    const float* a = static_cast<const float*>(in[0].buffer->read_ptr());
    if (_nports == 1) {
        if (o != a) std::memmove(o, a, n * 8);
    }
    for (size_t p = 1; p < _nports; ++p) {
        const float* b = static_cast<const float*>(in[p].buffer->read_ptr());
        const float* src = p == 1 ? a : o;
        if constexpr (OP == 0) {
            for (size_t i = 0; i < 2 * n; ++i) o[i] = src[i] + b[i];
        } else {
            cmul_vec(src, b, o, n);
        }
    }
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}
template class arith_cc<0>;
template class arith_cc<1>;

fir_filter_ccf::fir_filter_ccf(const std::vector<float>& taps, int decim)
    : decim_block("fir_filter_ccf", (unsigned)decim), _taps(taps), _decim(decim)
{
    if (taps.empty()) throw std::invalid_argument("fir_filter_ccf: no taps");
    if (decim < 1) throw std::invalid_argument("fir_filter_ccf: decimation < 1");
}

bool fir_filter_ccf::start()
{
    _ext.assign(_taps.size() - 1, gr_complex(0, 0)); // zero history at stream start
    return block::start();
}

void fir_filter_ccf::filter(const gr_complex* x, gr_complex* y, int n_out)
{
    const int L = (int)_taps.size();
    const size_t n_in = (size_t)n_out * _decim;
    if (_ext.size() < (size_t)(L - 1)) _ext.assign((size_t)(L - 1), gr_complex(0, 0)); // not started: zeros
    _ext.resize((size_t)(L - 1) + n_in);
    std::memcpy(_ext.data() + (L - 1), x, n_in * sizeof(gr_complex));
    fir_rows(reinterpret_cast<const float*>(_ext.data()), _taps.data(), L, _decim, reinterpret_cast<float*>(y), (size_t)n_out);
    // keep the last L-1 inputs as history
    std::memmove(_ext.data(), _ext.data() + n_in, (size_t)(L - 1) * sizeof(gr_complex));
    _ext.resize((size_t)(L - 1));
}

work_return_code_t fir_filter_ccf::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const int n_out = out[0].n_items; // decim_block::do_work: in[0].n_items == D * n_out
    filter(static_cast<const gr_complex*>(in[0].buffer->read_ptr()), static_cast<gr_complex*>(out[0].buffer->write_ptr()),
           n_out);
    out[0].n_produced = n_out;
    return work_return_code_t::WORK_OK;
}

const char* cpu_isa()
{
    switch (g_isa) {
    case isa::avx512: return "avx512f+fma";
    case isa::avx2: return "avx2+fma";
    default: return "x86-64 baseline (sse2)";
    }
}

} // namespace blocks
} // namespace gr
