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
// (ar kr - ai ki, ar ki + ai kr) with every product rounded: FMA contraction is switched
// off for these two functions only, to match the reference formula bit for bit.
#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
__attribute__((target_clones("arch=skylake-avx512", "arch=haswell", "default"))) void
cmul_const(const float* in, float* out, size_t n, float kr, float ki)
{
    for (size_t i = 0; i < n; ++i) {
        const float ar = in[2 * i], ai = in[2 * i + 1];
        const float p0 = ar * kr, p1 = ai * ki, p2 = ar * ki, p3 = ai * kr;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}
__attribute__((target_clones("arch=skylake-avx512", "arch=haswell", "default"))) void
cmul_vec(const float* a, const float* b, float* out, size_t n)
{
    for (size_t i = 0; i < n; ++i) {
        const float ar = a[2 * i], ai = a[2 * i + 1], br = b[2 * i], bi = b[2 * i + 1];
        const float p0 = ar * br, p1 = ai * bi, p2 = ar * bi, p3 = ai * br;
        out[2 * i] = p0 - p1;
        out[2 * i + 1] = p2 + p3;
    }
}
#pragma GCC pop_options

// Decim-1 rows: 32 complex outputs (4 x 16 interleaved floats) per step, taps broadcast,
// fp32 FMA in tap order: out[m] = sum_k h[k] * x[m - k], x = ext shifted by L-1.
typedef float v16f __attribute__((vector_size(64)));

__attribute__((target_clones("arch=skylake-avx512", "arch=haswell", "default"))) void
fir_rows(const float* ext, const float* h, int L, int D, float* out, size_t n_out)
{
    size_t m = 0;
    if (D == 1) {
        for (; m + 32 <= n_out; m += 32) {
            v16f a0 = {}, a1 = {}, a2 = {}, a3 = {};
            const float* base = ext + 2 * (m + (size_t)(L - 1));
            for (int k = 0; k < L; ++k) {
                const float* x = base - 2 * k;
                v16f x0, x1, x2, x3;
                std::memcpy(&x0, x, 64);
                std::memcpy(&x1, x + 16, 64);
                std::memcpy(&x2, x + 32, 64);
                std::memcpy(&x3, x + 48, 64);
                const float hk = h[k];
                a0 += hk * x0;
                a1 += hk * x1;
                a2 += hk * x2;
                a3 += hk * x3;
            }
            std::memcpy(out + 2 * m, &a0, 64);
            std::memcpy(out + 2 * m + 16, &a1, 64);
            std::memcpy(out + 2 * m + 32, &a2, 64);
            std::memcpy(out + 2 * m + 48, &a3, 64);
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

work_return_code_t fir_filter_ccf::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const int L = (int)_taps.size();
    const int n_out = out[0].n_items; // decim_block::do_work: in[0].n_items == D * n_out
    const size_t n_in = (size_t)n_out * _decim;
    const gr_complex* x = static_cast<const gr_complex*>(in[0].buffer->read_ptr());
    _ext.resize((size_t)(L - 1) + n_in);
    std::memcpy(_ext.data() + (L - 1), x, n_in * sizeof(gr_complex));
    fir_rows(reinterpret_cast<const float*>(_ext.data()), _taps.data(), L, _decim,
             static_cast<float*>(out[0].buffer->write_ptr()), (size_t)n_out);
    // keep the last L-1 inputs as history
    std::memmove(_ext.data(), _ext.data() + n_in, (size_t)(L - 1) * sizeof(gr_complex));
    _ext.resize((size_t)(L - 1));
    out[0].n_produced = n_out;
    return work_return_code_t::WORK_OK;
}

} // namespace blocks
} // namespace gr
