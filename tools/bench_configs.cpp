// Secondary BASELINE configs (BASELINE.json configs[0,1,3,4]; configs[2] = C3 is bench.py),
// measured through the same runtime as the headline: flowgraphs in one scheduler_hip domain
// with an HBM-resident input ring (nop_source -> nop_head(n) -> [2n-item hip_buffer,
// preloaded with the counter-based stream] -> blocks -> null_sink), wall time of whole
// fg->run() calls (median of K after one warm-up) and, as bench.py times the headline since round 4,
// one run streaming K batches through the same flowgraph (nop_head passes K n items over the
// resident ring: every batch is read from HBM; the run's start and drain paid once), tail parity
// against an in-tool CPU reference, and the CPU scheduler_mt path of the same config where the
// CPU blocks exist.
//   build/tools/bench_configs [log2n=28] [steps=5]     -> one JSON line per config
#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <gnuradio/blocklib/blocks/copy.hpp>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/multiply_const.hpp>
#include <gnuradio/blocklib/blocks/nop.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/fir_filter_cascade_ccf.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_context.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>
#include <gnuradio/vmcircbuf.hpp>
#include <string>
#include <vector>

#include "nsh_hip.h"

using namespace gr;
using clk = std::chrono::steady_clock;

static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static std::vector<gr_complex> synth(size_t n, uint64_t first = 0, uint64_t seed = 0x6E736368)
{
    std::vector<gr_complex> v(n);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t g = 2 * (first + i);
        v[i] = gr_complex((float)(int)(splitmix64(seed ^ g) >> 40) * (1.0f / 8388608.0f) - 1.0f,
                          (float)(int)(splitmix64(seed ^ (g + 1)) >> 40) * (1.0f / 8388608.0f) - 1.0f);
    }
    return v;
}
static gr_complex cmul(gr_complex a, gr_complex k)
{
    volatile float p0 = a.real() * k.real(), p1 = a.imag() * k.imag(), p2 = a.real() * k.imag(), p3 = a.imag() * k.real();
    return gr_complex(p0 - p1, p2 + p3);
}
static std::vector<float> lowpass(int L, double fc) // firwin(L, 2 fc) with a Hamming window, unit DC gain
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
static std::vector<gr_complex> fir_ref(const std::vector<gr_complex>& x, const std::vector<float>& h, int D)
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
static double rel_err(const std::vector<gr_complex>& y, const std::vector<gr_complex>& r, size_t skip = 0)
{
    double e = 0, s = 0;
    for (size_t i = skip; i < y.size(); ++i) {
        e = std::max(e, (double)std::abs(y[i] - r[i]));
        s = std::max(s, (double)std::abs(r[i]));
    }
    return s > 0 ? e / s : e;
}
static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// GPU flowgraph with a resident input ring in front of `first` and a hip_buffer in front of
// the null_sink after `last`.
struct gpu_fg {
    flowgraph::sptr fg;
    schedulers::scheduler_hip::sptr sched;
    std::shared_ptr<blocks::nop_head> head;
    block_sptr snk;
    int64_t n_items;
    size_t isz;
    int dev = 0;

    gpu_fg(std::vector<block_sptr> chain, int64_t n_items_, size_t isz_, size_t out_buf_bytes, bool fusion = true,
           bool fir_fusion = true)
        : n_items(n_items_), isz(isz_)
    {
        auto src = blocks::nop_source::make(isz);
        head = blocks::nop_head::make(isz, (size_t)n_items);
        snk = blocks::null_sink::make(isz);
        fg = flowgraph::make();
        fg->connect(src, 0, head, 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
        const int64_t cap = 2 * n_items;
        const int d = dev;
        fg->connect(head, 0, chain[0], 0)
            ->set_custom_buffer(
                [cap, d](size_t, size_t item, std::shared_ptr<buffer_properties>) -> buffer_sptr {
                    return std::make_shared<hip_buffer>((size_t)cap, item, hip_buffer_type::D2D, d);
                },
                hip_buffer_properties::make(hip_buffer_type::D2D, d));
        for (size_t i = 1; i < chain.size(); ++i) fg->connect(chain[i - 1], 0, chain[i], 0);
        fg->connect(chain.back(), 0, snk, 0);
        sched = schedulers::scheduler_hip::make("hip", dev, out_buf_bytes);
        sched->set_fusion(fusion);
        sched->set_fir_fusion(fir_fusion);
        fg->set_scheduler(sched);
        fg->set_wait_spin_us(5000); // a run is ~1 ms: poll for its end instead of sleeping (as bench.py's flowgraph)
        // and the partition stream's drain, likewise (as bench.py's flowgraph): without it each
        // streamed batch waited ~22 us in a blocking stream sync between launches (r04zp trace)
        sched->set_flush_spin_us(5000);
        fg->validate();
        // the head's output edge (its consumer may be a fused block replacing chain[0])
        auto ring = std::dynamic_pointer_cast<hip_buffer>(sched->buffers()->get_output_buffers(head->output_stream_ports()[0])[0]);
        void* s = nullptr;
        hip::check(nsh_stream_create(dev, &s), "stream");
        const int64_t n_samples = n_items * (int64_t)(isz / sizeof(gr_complex));
        char* base = (char*)ring->device_base();
        hip::check(nsh_synth_cf32((float*)base, n_samples, 0, 0x6E736368, s), "preload");
        hip::check(nsh_synth_cf32((float*)(base + n_items * isz), n_samples, 0, 0x6E736368, s), "preload");
        hip::check(nsh_stream_sync(s), "preload");
        nsh_stream_destroy(s);
    }
    double run(int steps)
    {
        // warm-up to the sustained clock: at least 20 back-to-back runs (tools/probe/run_series.py)
        // and at least 1 s of them, as bench.py's warm-up -- 20 runs of a ~0.7 ms config last
        // ~15 ms, and the first GPU config then measured 4-6 % below its own streamed rate on a
        // cold chip (C2's hand-fused block in r04zc / r04zm)
        const auto tw = clk::now();
        for (int i = 0; i < 20 || std::chrono::duration<double>(clk::now() - tw).count() < 1.0; ++i) fg->run();
        std::vector<double> t;
        for (int i = 0; i < steps; ++i) {
            const auto t0 = clk::now();
            fg->run();
            t.push_back(std::chrono::duration<double>(clk::now() - t0).count());
        }
        return median(t);
    }
    // one run streaming `batches` batches (after run()'s warm-up): seconds per batch
    double run_streamed(int batches)
    {
        head->set_length((size_t)(batches * n_items));
        const auto t0 = clk::now();
        fg->run();
        const double s = std::chrono::duration<double>(clk::now() - t0).count() / batches;
        head->set_length((size_t)n_items);
        return s;
    }
    // last `count` samples written into the sink's input ring
    std::vector<gr_complex> tail(int64_t count)
    {
        auto r = std::dynamic_pointer_cast<hip_buffer>(sched->buffers()->get_input_buffer(snk->input_stream_ports()[0]));
        const size_t per = isz / sizeof(gr_complex);
        const uint64_t end = r->total_written() * per;
        const uint64_t cap = r->capacity() * per;
        std::vector<gr_complex> out((size_t)count);
        const uint64_t start = end - (uint64_t)count;
        const char* src = (const char*)r->device_base() + (start % cap) * sizeof(gr_complex);
        void* s = nullptr;
        hip::check(nsh_stream_create(dev, &s), "stream");
        hip::check(nsh_memcpy_async(out.data(), src, (size_t)count * sizeof(gr_complex), NSH_D2H, s), "tail");
        hip::check(nsh_stream_sync(s), "tail");
        nsh_stream_destroy(s);
        return out;
    }
};

// CPU scheduler_mt path: vector_source(repeat) -> head(n) -> chain -> null_sink
static double cpu_run(std::vector<block_sptr> chain, int64_t n, size_t fixed = 32768)
{
    auto src = blocks::vector_source_c::make(synth(1 << 16), true);
    auto head = blocks::head::make(sizeof(gr_complex), (size_t)n);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, chain[0], 0);
    for (size_t i = 1; i < chain.size(); ++i) fg->connect(chain[i - 1], 0, chain[i], 0);
    fg->connect(chain.back(), 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", (unsigned)fixed));
    fg->validate();
    const auto t0 = clk::now();
    fg->run();
    return std::chrono::duration<double>(clk::now() - t0).count();
}

static void emit(const std::string& s) { std::printf("%s\n", s.c_str()), std::fflush(stdout); }
static std::string num(double v, int prec = 1);
// the measured device copy (nsh_copy = k_copy_v4, 16 B per sample), GB/s: the second peak
// BASELINE.md asks every config to be quoted against -- measured last, on a warm chip, best of 3
static double measure_copy(int64_t n)
{
    void *x = nullptr, *y = nullptr, *s = nullptr, *e0 = nullptr, *e1 = nullptr;
    hip::check(nsh_malloc(0, (size_t)n * 8, &x), "copy");
    hip::check(nsh_malloc(0, (size_t)n * 8, &y), "copy");
    hip::check(nsh_stream_create(0, &s), "copy");
    hip::check(nsh_event_create(&e0), "copy");
    hip::check(nsh_event_create(&e1), "copy");
    hip::check(nsh_synth_cf32((float*)x, n, 0, 0x6E736368, s), "copy");
    const auto t0 = clk::now();
    while (std::chrono::duration<double>(clk::now() - t0).count() < 1.5) { // clocks settle (first GPU work of the run)
        hip::check(nsh_copy(x, y, (size_t)n * 8, s), "copy");
        hip::check(nsh_stream_sync(s), "copy");
    }
    const int reps = 10;
    float ms = 0;
    for (int k = 0; k < 3; ++k) {
        hip::check(nsh_event_record(e0, s), "copy");
        for (int i = 0; i < reps; ++i) hip::check(nsh_copy(x, y, (size_t)n * 8, s), "copy");
        hip::check(nsh_event_record(e1, s), "copy");
        hip::check(nsh_event_sync(e1), "copy");
        float m = 0;
        hip::check(nsh_event_elapsed_ms(e0, e1, &m), "copy");
        ms = k == 0 ? m : std::min(ms, m);
    }
    nsh_event_destroy(e0);
    nsh_event_destroy(e1);
    nsh_stream_destroy(s);
    nsh_free(x);
    nsh_free(y);
    return 16.0 * n / (ms / reps * 1e-3) / 1e9;
}
// the streamed figure (K batches in one run) beside the per-run one
static std::string streamed(double n_per_batch, double s, int batches, double bytes_per_sample, double hbm)
{
    const double gbs = bytes_per_sample * n_per_batch / s / 1e9;
    return ", \"streamed\": {\"batches_per_run\": " + std::to_string(batches) + ", \"value\": " + num(n_per_batch / s / 1e6, 1) +
           ", \"ms_per_batch\": " + num(s * 1e3, 3) + ", \"achieved_GBs\": " + num(gbs, 1) + ", \"hbm_frac\": " + num(gbs / hbm, 4) + "}";
}
static std::string num(double v, int prec)
{
    char b[64];
    std::snprintf(b, sizeof b, "%.*f", prec, v);
    return b;
}

int main(int argc, char** argv)
{
    const int log2n = argc > 1 ? std::atoi(argv[1]) : 28;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int64_t n = 1ll << log2n;
    const double hbm = 8000.0; // GB/s spec
    const std::vector<gr_complex> ks = { std::polar(1.0f, 0.1f), std::polar(1.0f, 0.2f), std::polar(1.0f, 0.3f),
                                         std::polar(1.0f, 0.4f) };

    // ---- C1: null_source -> head(2^20) -> copy -> null_sink, CPU only ----------------------
    {
        std::vector<double> t;
        for (int r = 0; r < 7; ++r) {
            auto src = blocks::null_source::make(sizeof(gr_complex));
            auto head = blocks::head::make(sizeof(gr_complex), 1u << 20);
            auto cp = blocks::copy::make(sizeof(gr_complex));
            auto snk = blocks::null_sink::make(sizeof(gr_complex));
            auto fg = flowgraph::make();
            fg->connect(src, 0, head, 0);
            fg->connect(head, 0, cp, 0);
            fg->connect(cp, 0, snk, 0);
            fg->set_scheduler(schedulers::scheduler_mt::make("mt", 32768));
            fg->validate();
            const auto t0 = clk::now();
            fg->run();
            t.push_back(std::chrono::duration<double>(clk::now() - t0).count());
        }
        const double s = median(t);
        emit("{\"config\": \"C1\", \"workload\": \"null_source->head(2^20)->copy->null_sink, scheduler_mt 4 threads, 32 KiB buffers\", "
             "\"value\": " + num((1 << 20) / s / 1e6, 2) + ", \"unit\": \"MSamples/s\", \"median_of\": 7, "
             "\"note\": \"drain-based termination; the reference adds a fixed 100 ms sleep per run (flowgraph_monitor.cpp:27)\"}");
    }

    // ---- C2: 4 x multiply_const_cc ----------------------------------------------------------
    // variant 0: hand-built multiply_const_chain_cc; 1: four multiply_const_cc blocks fused by
    // scheduler_hip (its default); 2: the four blocks with fusion off (every edge in HBM).
    for (int variant = 0; variant < 3; ++variant) {
        std::vector<block_sptr> chain;
        if (variant == 0)
            chain.push_back(hip::multiply_const_chain_cc::make(ks));
        else
            for (auto k : ks) chain.push_back(hip::multiply_const_cc::make(k));
        gpu_fg g(chain, n, sizeof(gr_complex), (size_t)n * sizeof(gr_complex), variant != 2);
        const bool one_pass = variant != 2;
        const double s = g.run(steps);
        const double ss = g.run_streamed(steps);
        auto y = g.tail(4096);
        auto x = synth(4096, n - 4096);
        for (auto& v : x)
            for (auto k : ks) v = cmul(v, k);
        const bool exact = y == x;
        const double gbs = (one_pass ? 16.0 : 64.0) * n / s / 1e9;
        const char* name[] = { "hand-fused multiply_const_chain_cc block",
                               "4 multiply_const_cc blocks, fused by scheduler_hip (default)",
                               "4 multiply_const_cc blocks, fusion off (every edge in HBM)" };
        std::string line = "{\"config\": \"C2\", \"variant\": \"" + std::string(name[variant]) +
                           "\", \"value\": " + num(n / s / 1e6) + ", \"unit\": \"MSamples/s\", \"ms_per_run\": " + num(s * 1e3, 3) +
                           ", \"hbm_bytes_per_sample\": " + (one_pass ? "16" : "64") + ", \"achieved_GBs\": " + num(gbs) +
                           ", \"hbm_frac\": " + num(gbs / hbm, 4) + streamed((double)n, ss, steps, one_pass ? 16.0 : 64.0, hbm) +
                           ", \"parity_tail_bitexact\": " + (exact ? "true" : "false");
        if (variant == 1) {
            const int64_t nc = 1 << 25;
            std::vector<block_sptr> cc;
            for (auto k : ks) cc.push_back(blocks::multiply_const_cc::make(k));
            const double cs = cpu_run(cc, nc);
            line += ", \"cpu_baseline\": {\"value\": " + num(nc / cs / 1e6, 2) +
                    ", \"unit\": \"MSamples/s\", \"sample\": \"2^25 samples, vector_source->head->4x blocks::multiply_const_cc->null_sink, scheduler_mt thread per block\"}";
        }
        emit(line + "}");
    }

    // ---- C4: fft1024 -> x W -> ifft1024: the channelizer block, and the three blocks fused or not --
    {
        std::vector<gr_complex> w(1024);
        for (int b = 0; b < 1024; ++b) w[b] = gr_complex((float)((1.0 + 0.5 * std::cos(2 * M_PI * b / 1024.0)) / 1024.0), 0.f);
        const int64_t frames = n / 1024;
        // parity reference: the last frame, direct DFT in double
        auto x = synth(1024, n - 1024);
        std::vector<std::complex<double>> X(1024);
        for (int k = 0; k < 1024; ++k) {
            std::complex<double> acc = 0;
            for (int t = 0; t < 1024; ++t) acc += std::complex<double>(x[t]) * std::polar(1.0, -2 * M_PI * k * t / 1024.0);
            X[k] = acc * std::complex<double>(w[k]);
        }
        std::vector<gr_complex> r(1024);
        for (int t = 0; t < 1024; ++t) {
            std::complex<double> acc = 0;
            for (int k = 0; k < 1024; ++k) acc += X[k] * std::polar(1.0, 2 * M_PI * k * t / 1024.0);
            r[t] = gr_complex(acc);
        }
        const char* names[3] = { "channelizer_vcc block (fft1024 * W ifft1024 in registers)",
                                 "fft_vcc -> multiply_const_vcc(W) -> ifft_vcc blocks, fused by scheduler_hip (default)",
                                 "fft_vcc -> multiply_const_vcc(W) -> ifft_vcc blocks, fusion off (3 launches, 48 B/sample)" };
        for (int variant = 0; variant < 3; ++variant) {
            std::vector<block_sptr> chain;
            if (variant == 0)
                chain = { hip::channelizer_vcc::make(w) };
            else
                chain = { hip::fft_vcc::make(1024, true), hip::multiply_const_vcc::make(w), hip::fft_vcc::make(1024, false) };
            gpu_fg g(chain, frames, 1024 * sizeof(gr_complex), (size_t)n * sizeof(gr_complex), variant != 2);
            const double s = g.run(steps);
            const double ss = g.run_streamed(steps);
            auto y = g.tail(1024);
            const int bytes = variant == 2 ? 48 : 16;
            const double gbs = (double)bytes * n / s / 1e9;
            emit(std::string("{\"config\": \"C4\", \"variant\": \"") + names[variant] + "\", \"value\": " + num(n / s / 1e6) +
                 ", \"unit\": \"MSamples/s\", \"ms_per_run\": " + num(s * 1e3, 3) + ", \"hbm_bytes_per_sample\": " +
                 std::to_string(bytes) + ", \"achieved_GBs\": " + num(gbs) + ", \"hbm_frac\": " + num(gbs / hbm, 4) +
                 streamed((double)n, ss, steps, bytes, hbm) + ", \"parity_last_frame_rel_err\": " + num(rel_err(y, r), 9) + "}");
        }
    }

    // ---- C5 at G = 1: 4 x (127-tap, D = 2) ----------------------------------------------------
    {
        const auto h = lowpass(127, 0.225); // firwin(127, 0.45)
        // parity: last 4096 outputs from the last 4096*16 + 4 stage halos of input
        const int64_t m = 4096, win = m * 16 + 2048;
        auto xr = synth(win, n - win);
        for (int i = 0; i < 4; ++i) xr = fir_ref(xr, h, 2);
        std::vector<gr_complex> r(xr.end() - m, xr.end());
        const int64_t nc = 1 << 24;
        std::vector<block_sptr> cc;
        for (int i = 0; i < 4; ++i) cc.push_back(blocks::fir_filter_ccf::make(h, 2));
        const double cs = cpu_run(cc, nc);
        for (int fused = 1; fused >= 0; --fused) {
            std::vector<block_sptr> chain;
            for (int i = 0; i < 4; ++i) chain.push_back(hip::fir_filter_ccf::make(h, 2));
            gpu_fg g(chain, n, sizeof(gr_complex), (size_t)n * sizeof(gr_complex), true, fused == 1);
            const double s = g.run(steps);
            std::string launches;
            for (auto& b : g.sched->fusion_plan().fused)
                if (auto c = std::dynamic_pointer_cast<hip::fir_filter_cascade_ccf>(b))
                    launches = ", \"cascade_launches_per_run\": " + num((double)c->launches() / (steps + 20), 2) +
                               ", \"cascade_kernel\": \"" + c->kernel() + "\"";
            const double ss = g.run_streamed(steps);
            auto y = g.tail(m);
            const double gbs = 8.5 * n / s / 1e9;
            const char* var = fused ? "G=1: 4 x fir_filter_ccf(127 taps, decim 2), fused by scheduler_hip into one "
                                      "fir_filter_cascade_ccf (k_fir_pfft2<16>, default)"
                                    : "G=1: 4 x fir_filter_ccf(127 taps, decim 2), FIR fusion off (4 launches, every "
                                      "stage streams its own input)";
            emit(std::string("{\"config\": \"C5\", \"variant\": \"") + var + "\", \"value\": " + num(n / s / 1e6) +
                 ", \"unit\": \"MSamples/s (input)\", \"ms_per_run\": " + num(s * 1e3, 3) +
                 ", \"hbm_bytes_per_input_sample\": 8.5, \"achieved_GBs\": " + num(gbs) + ", \"hbm_frac\": " +
                 num(gbs / hbm, 4) + streamed((double)n, ss, steps, 8.5, hbm) + ", \"parity_tail_rel_err\": " +
                 num(rel_err(y, r), 9) + launches +
                 (fused ? ", \"cpu_baseline\": {\"value\": " + num(nc / cs / 1e6, 2) +
                              ", \"unit\": \"MSamples/s (input)\", \"sample\": \"2^24 samples, vector_source->head->4x "
                              "blocks::fir_filter_ccf(decim 2)->null_sink, scheduler_mt thread per block\"}}"
                        : std::string("}")));
        }
    }
    // ---- the measured copy ceiling (after the GPU configs: the chip is warm) -------------------
    {
        const double gbs = measure_copy(n);
        emit("{\"config\": \"copy\", \"variant\": \"nsh_copy (k_copy_v4) of 2^" + std::to_string(log2n) +
             " complex samples on fresh buffers, 16 B per sample, best of 3 x 10 launches (HIP events)\", \"achieved_GBs\": " +
             num(gbs) + ", \"hbm_frac\": " + num(gbs / hbm, 4) + "}");
    }
    // ---- C3 with host endpoints: the PCIe-inclusive rate (not the metric: bench.py's input is
    // resident). vector_source(repeat) -> head -[H2D]-> hip::fir_filter_ccf -[D2H]-> null_sink,
    // host blocks in a scheduler_mt domain (thread per block), the FIR in scheduler_hip.
    {
        const int64_t nh = (int64_t)1 << 26;
        const auto h = lowpass(127, 0.1); // firwin(127, 0.2)
        auto run = [&](size_t buf) {
            auto src = blocks::vector_source_c::make(synth(1 << 20), true);
            auto head = blocks::head::make(sizeof(gr_complex), (size_t)nh);
            auto fir = hip::fir_filter_ccf::make(h, 1);
            auto snk = blocks::null_sink::make(sizeof(gr_complex));
            auto fg = flowgraph::make();
            fg->connect(src, 0, head, 0);
            fg->connect(head, 0, fir, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
            fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
            auto cpu = schedulers::scheduler_mt::make("cpu", (unsigned)buf);
            auto gpu = schedulers::scheduler_hip::make("gpu", 0, buf);
            fg->add_scheduler(cpu);
            fg->add_scheduler(gpu);
            auto da = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
            domain_conf_vec dc{ domain_conf(cpu, { src, head, snk }, da), domain_conf(gpu, { fir }, da) };
            fg->partition(dc);
            fg->run(); // warm-up
            std::vector<double> t;
            for (int i = 0; i < 5; ++i) {
                const auto t0 = clk::now();
                fg->run();
                t.push_back(std::chrono::duration<double>(clk::now() - t0).count());
            }
            return median(t);
        };
        for (size_t buf : { (size_t)16 << 20, (size_t)64 << 20 }) {
            const double s = run(buf);
            emit("{\"config\": \"C3-host\", \"variant\": \"vector_source -> head -[H2D]-> hip::fir_filter_ccf -[D2H]-> null_sink, " +
                 std::to_string(buf >> 20) + " MiB buffers (PCIe-inclusive; not the metric)\", \"value\": " + num(nh / s / 1e6) +
                 ", \"unit\": \"MSamples/s\", \"ms_per_run\": " + num(s * 1e3, 3) + ", \"pcie_GBs_each_way\": " +
                 num(8.0 * nh / s / 1e9, 2) + "}");
        }
    }
    return 0;
}
