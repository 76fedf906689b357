// In-test CPU references shared by the GPU and cross-process flowgraph tests: the
// counter-based synthetic stream, the complex product with the per-product
// rounding of the kernels, a float64-accumulated FIR with zero initial history (the a19
// semantics of SURVEY.md §8a), a norm-wise comparison and a Hamming-window lowpass.
#pragma once
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <gnuradio/types.hpp>
#include <vector>

inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
inline std::vector<gr_complex> synth(size_t n, uint64_t first = 0, uint64_t seed = 0x6E736368)
{
    std::vector<gr_complex> v(n);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t g = 2 * (first + i);
        v[i] = gr_complex((float)(int)(splitmix64(seed ^ g) >> 40) * (1.0f / 8388608.0f) - 1.0f,
                          (float)(int)(splitmix64(seed ^ (g + 1)) >> 40) * (1.0f / 8388608.0f) - 1.0f);
    }
    return v;
}
inline gr_complex cmul(gr_complex a, gr_complex k)
{
    volatile float p0 = a.real() * k.real(), p1 = a.imag() * k.imag(), p2 = a.real() * k.imag(), p3 = a.imag() * k.real();
    return gr_complex(p0 - p1, p2 + p3);
}
inline std::vector<gr_complex> fir_ref(const std::vector<gr_complex>& x, const std::vector<float>& h, int D)
{
    std::vector<gr_complex> y(x.size() / D);
    for (size_t m = 0; m < y.size(); ++m) {
        std::complex<double> acc = 0;
        for (size_t k = 0; k < h.size(); ++k) {
            const long g = (long)(m * D) - (long)k;
            if (g >= 0) acc += (double)h[k] * std::complex<double>(x[g]);
        }
        y[m] = gr_complex(acc);
    }
    return y;
}
inline bool close_normwise(const std::vector<gr_complex>& y, const std::vector<gr_complex>& r, double rel = 1e-5)
{
    if (y.size() != r.size()) {
        std::fprintf(stderr, "  size %zu != %zu\n", y.size(), r.size());
        return false;
    }
    double maxerr = 0, scale = 0;
    for (size_t i = 0; i < y.size(); ++i) {
        maxerr = std::max(maxerr, (double)std::abs(y[i] - r[i]));
        scale = std::max(scale, (double)std::abs(r[i]));
    }
    if (maxerr > rel * scale) std::fprintf(stderr, "  maxerr %g scale %g\n", maxerr, scale);
    return maxerr <= rel * scale;
}
inline std::vector<float> lowpass(int L, double fc)
{
    std::vector<float> h(L);
    double s = 0;
    for (int k = 0; k < L; ++k) {
        const double t = k - (L - 1) / 2.0;
        const double sinc = t == 0 ? 2 * fc : std::sin(2 * M_PI * fc * t) / (M_PI * t);
        h[k] = (float)(sinc * (0.54 - 0.46 * std::cos(2 * M_PI * k / (L - 1))));
        s += h[k];
    }
    for (auto& v : h) v = (float)(v / s);
    return h;
}

