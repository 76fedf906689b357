// libnewsched.so flowgraph runners (include/nsr_flowgraph.h).
#include <gnuradio/run_trace.hpp>
#include "nsr_flowgraph.h"

#include <chrono>
#include <cstring>
#include <gnuradio/blocklib/blocks/copy.hpp>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/blocklib/blocks/nop.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/synth_source.hpp>
#include <gnuradio/domain_adapter_remote.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_context.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>
#include <gnuradio/vmcircbuf.hpp>
#include <string>

#include "nsh_hip.h"

using namespace gr;

namespace {
thread_local std::string t_err;

template <class F>
int guarded(F&& f)
{
    try {
        f();
        t_err.clear();
        return 0;
    } catch (const std::exception& e) {
        t_err = e.what();
    } catch (...) {
        t_err = "unknown exception";
    }
    return -1;
}

uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
gr_complex synth_at(uint64_t i, uint64_t seed)
{
    const uint64_t g = 2 * i;
    return gr_complex((float)(int)(splitmix64(seed ^ g) >> 40) * (1.0f / 8388608.0f) - 1.0f,
                      (float)(int)(splitmix64(seed ^ (g + 1)) >> 40) * (1.0f / 8388608.0f) - 1.0f);
}

// The ntaps - 1 stream samples before first_index (a FIR's initial history); indices before the
// stream's start are zeros, as the filter's own start-up history.
std::vector<gr_complex> history_before(uint64_t first_index, int ntaps, uint64_t seed)
{
    std::vector<gr_complex> h((size_t)(ntaps > 1 ? ntaps - 1 : 0));
    for (size_t j = 0; j < h.size(); ++j) {
        const uint64_t back = h.size() - j; // first_index - back
        h[j] = back <= first_index ? synth_at(first_index - back, seed) : gr_complex(0.f, 0.f);
    }
    return h;
}

// A resident input ring holds the batch x (n samples from first_index) twice, the second copy
// `half` bytes after the first, so every run starts on a copy of x.
void preload_twice(char* base, size_t half, int64_t n, uint64_t first_index, uint64_t seed, int dev)
{
    void* s = nullptr;
    hip::check(nsh_stream_create(dev, &s), "nsr: stream");
    int rc = nsh_synth_cf32((float*)base, n, first_index, seed, s);
    if (rc == 0) rc = nsh_synth_cf32((float*)(base + half), n, first_index, seed, s);
    const int rc2 = nsh_stream_sync(s); // also after a failed launch: nothing of ours left queued
    nsh_stream_destroy(s);
    hip::check(rc != 0 ? rc : rc2, "nsr: preload");
}

// Tail of a device ring's last `count` written items -> host.
void ring_tail(const std::shared_ptr<hip_buffer>& r, int dev, int64_t count, float* out_host)
{
    if (count <= 0 || (size_t)count > r->capacity() / 2 || (uint64_t)count > r->total_written())
        throw std::invalid_argument("tail: bad count");
    const uint64_t start = r->total_written() - (uint64_t)count;
    const char* src = (const char*)r->device_base() + (start % r->capacity()) * r->item_size();
    void* s = nullptr;
    hip::check(nsh_stream_create(dev, &s), "nsr: stream");
    const int rc = nsh_memcpy_async(out_host, src, (size_t)count * r->item_size(), NSH_D2H, s);
    const int rc2 = rc == 0 ? nsh_stream_sync(s) : rc;
    nsh_stream_destroy(s);
    hip::check(rc2, "nsr: tail copy");
}

struct c5_pipeline {
    flowgraph::sptr fg;
    std::shared_ptr<domain_adapter_remote_conf> da;
    std::vector<hip::fir_filter_ccf::sptr> stages;
    std::shared_ptr<hip_buffer> out_ring; // last group only
    int dev = 0;
};

struct chain_bench {
    flowgraph::sptr fg;
    schedulers::scheduler_hip::sptr sched;
    blocks::nop_head::sptr head;
    std::shared_ptr<hip_buffer> out_ring;
    int64_t n_items = 0; // per batch, in the input ring's items
    size_t spi = 1;      // samples per item (1024 for the channelizer's vectors)
    int dev = 0;
};

struct fir_bench {
    flowgraph::sptr fg;
    schedulers::scheduler_hip::sptr sched;
    blocks::nop_head::sptr head;
    int64_t n = 0;
    bool timing = false;
    hip::fir_filter_ccf::sptr fir;
    std::shared_ptr<hip_buffer> out_ring;
    int dev = 0;
};
} // namespace

extern "C" {

const char* nsr_last_error(void) { return t_err.c_str(); }

int nsr_fir_bench_create(int dev, const float* taps, int ntaps, int algo, int64_t n, uint64_t first_index,
                         uint64_t seed, size_t out_buf_bytes, int timing, void** handle)
{
    return guarded([&] {
        if (n <= 0 || n % 256) throw std::invalid_argument("nsr_fir_bench_create: n must be a positive multiple of 256");
        if (!taps || ntaps <= 0) throw std::invalid_argument("nsr_fir_bench_create: no taps");
        auto b = std::make_unique<fir_bench>();
        b->dev = dev;
        const size_t isz = sizeof(gr_complex);
        auto src = blocks::nop_source::make(isz);
        auto head = blocks::nop_head::make(isz, (size_t)n);
        b->head = head;
        b->n = n;
        b->fir = hip::fir_filter_ccf::make(std::vector<float>(taps, taps + ntaps), 1, algo);
        b->timing = timing != 0;
        b->fir->enable_timing(b->timing);
        if (first_index > 0) b->fir->set_initial_history(history_before(first_index, ntaps, seed));
        auto snk = blocks::null_sink::make(isz);
        b->fg = flowgraph::make();
        // the nop edge is never touched: a host ring costs no memory traffic
        b->fg->connect(src, 0, head, 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
        // the resident input ring: exactly 2n items so every run starts on a copy of x
        const int64_t cap = 2 * n;
        b->fg->connect(head, 0, b->fir, 0)
            ->set_custom_buffer(
                [cap, dev](size_t, size_t item, std::shared_ptr<buffer_properties>) -> buffer_sptr {
                    return std::make_shared<hip_buffer>((size_t)cap, item, hip_buffer_type::D2D, dev);
                },
                hip_buffer_properties::make(hip_buffer_type::D2D, dev));
        b->fg->connect(b->fir, 0, snk, 0); // scheduler default: hip_buffer D2D
        b->sched = schedulers::scheduler_hip::make("hip" + std::to_string(dev), dev, out_buf_bytes);
        b->fg->set_scheduler(b->sched);
        b->fg->set_wait_spin_us(5000); // one run is ~1 ms: poll for its end instead of sleeping
        b->sched->set_flush_spin_us(5000); // and the partition stream's drain, likewise
        b->fg->validate();

        auto in_ring = std::dynamic_pointer_cast<hip_buffer>(b->sched->buffers()->get_input_buffer(b->fir->input_stream_ports()[0]));
        b->out_ring = std::dynamic_pointer_cast<hip_buffer>(b->sched->buffers()->get_input_buffer(snk->input_stream_ports()[0]));
        if (!in_ring || !b->out_ring) throw std::runtime_error("nsr_fir_bench_create: unexpected buffer types");
        if ((int64_t)in_ring->capacity() != cap) throw std::runtime_error("nsr_fir_bench_create: ring capacity mismatch");
        preload_twice((char*)in_ring->device_base(), n * isz, n, first_index, seed, dev);
        *handle = b.release();
    });
}

#if NSR_RUN_TRACE
int nsr_run_trace(int64_t* out16) // probe builds only: the last run's stamps (ns)
{
    for (int k = 0; k < 16; ++k) out16[k] = gr::g_run_trace[k].load();
    return 0;
}
#endif

int nsr_fir_bench_run(void* handle)
{
    return guarded([&] { static_cast<fir_bench*>(handle)->fg->run(); });
}

int nsr_fir_bench_set_batches(void* handle, int64_t batches)
{
    return guarded([&] {
        auto b = static_cast<fir_bench*>(handle);
        if (batches < 1) throw std::invalid_argument("nsr_fir_bench_set_batches: batches must be >= 1");
        b->head->set_length((size_t)(batches * b->n));
    });
}

int nsr_fir_bench_runs(void* handle, int64_t count)
{
    return guarded([&] {
        auto fg = static_cast<fir_bench*>(handle)->fg;
        for (int64_t i = 0; i < count; ++i) fg->run();
    });
}

int nsr_fir_bench_set_timing_stride(void* handle, int stride)
{
    return guarded([&] {
        auto b = static_cast<fir_bench*>(handle);
        b->fir->enable_timing(b->timing, stride);
    });
}

int nsr_fir_bench_stats(void* handle, double* kernel_ms, uint64_t* launches, uint64_t* samples, int* algo)
{
    return guarded([&] {
        auto b = static_cast<fir_bench*>(handle);
        if (kernel_ms) *kernel_ms = b->fir->kernel_ms();
        if (launches) *launches = b->fir->timed_launches();
        if (samples) *samples = b->fir->timed_samples();
        if (algo) *algo = b->fir->algo();
    });
}

const char* nsr_fir_bench_kernel(void* handle)
{
    static thread_local std::string name;
    name.clear();
    (void)guarded([&] { name = static_cast<fir_bench*>(handle)->fir->kernel(); });
    return name.c_str();
}

int nsr_fir_bench_tail(void* handle, int64_t count, float* out_host)
{
    return guarded([&] {
        auto b = static_cast<fir_bench*>(handle);
        ring_tail(b->out_ring, b->dev, count, out_host);
    });
}

int nsr_fir_bench_destroy(void* handle)
{
    return guarded([&] { delete static_cast<fir_bench*>(handle); });
}

int nsr_chain_bench_create(int dev, int kind, const float* params, int nparams, int decim, int64_t n,
                           uint64_t first_index, uint64_t seed, size_t out_buf_bytes, void** handle)
{
    return guarded([&] {
        if (!params || nparams <= 0) throw std::invalid_argument("nsr_chain_bench_create: no parameters");
        auto b = std::make_unique<chain_bench>();
        b->dev = dev;
        std::vector<block_sptr> chain;
        switch (kind) {
        case NSR_CHAIN_MUL_CONST_CC:
            if (nparams % 2) throw std::invalid_argument("nsr_chain_bench_create: constants come as (re, im) pairs");
            for (int i = 0; i < nparams; i += 2) chain.push_back(hip::multiply_const_cc::make(gr_complex(params[i], params[i + 1])));
            break;
        case NSR_CHAIN_CHANNELIZER: {
            if (nparams != 2048) throw std::invalid_argument("nsr_chain_bench_create: the channelizer needs 1024 (re, im) weights");
            std::vector<gr_complex> w(1024);
            for (int k = 0; k < 1024; ++k) w[k] = gr_complex(params[2 * k], params[2 * k + 1]);
            chain = { hip::fft_vcc::make(1024, true), hip::multiply_const_vcc::make(w), hip::fft_vcc::make(1024, false) };
            b->spi = 1024;
            break;
        }
        case NSR_CHAIN_FIR: {
            if (decim < 1) throw std::invalid_argument("nsr_chain_bench_create: decim must be >= 1");
            auto f = hip::fir_filter_ccf::make(std::vector<float>(params, params + nparams), decim);
            if (first_index > 0) f->set_initial_history(history_before(first_index, nparams, seed));
            chain.push_back(f);
            break;
        }
        default:
            throw std::invalid_argument("nsr_chain_bench_create: unknown kind");
        }
        if (n <= 0 || n % (int64_t)(256 * b->spi) || (kind == NSR_CHAIN_FIR && n % decim))
            throw std::invalid_argument("nsr_chain_bench_create: n must be a positive multiple of 256 items (and of decim)");
        b->n_items = n / (int64_t)b->spi;
        const size_t isz = sizeof(gr_complex) * b->spi;
        auto src = blocks::nop_source::make(isz);
        b->head = blocks::nop_head::make(isz, (size_t)b->n_items);
        auto snk = blocks::null_sink::make(isz);
        b->fg = flowgraph::make();
        b->fg->connect(src, 0, b->head, 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
        const int64_t cap = 2 * b->n_items; // the resident input ring holds x twice
        b->fg->connect(b->head, 0, chain[0], 0)
            ->set_custom_buffer(
                [cap, dev](size_t, size_t item, std::shared_ptr<buffer_properties>) -> buffer_sptr {
                    return std::make_shared<hip_buffer>((size_t)cap, item, hip_buffer_type::D2D, dev);
                },
                hip_buffer_properties::make(hip_buffer_type::D2D, dev));
        for (size_t i = 1; i < chain.size(); ++i) b->fg->connect(chain[i - 1], 0, chain[i], 0);
        b->fg->connect(chain.back(), 0, snk, 0);
        b->sched = schedulers::scheduler_hip::make("hipc" + std::to_string(dev), dev, out_buf_bytes);
        b->fg->set_scheduler(b->sched);
        b->fg->set_wait_spin_us(5000);
        b->sched->set_flush_spin_us(5000);
        b->fg->validate();
        // the head's output edge (its consumer may be a fused block that replaced chain[0])
        auto in_ring = std::dynamic_pointer_cast<hip_buffer>(b->sched->buffers()->get_output_buffers(b->head->output_stream_ports()[0])[0]);
        b->out_ring = std::dynamic_pointer_cast<hip_buffer>(b->sched->buffers()->get_input_buffer(snk->input_stream_ports()[0]));
        if (!in_ring || !b->out_ring) throw std::runtime_error("nsr_chain_bench_create: unexpected buffer types");
        if ((int64_t)in_ring->capacity() != cap) throw std::runtime_error("nsr_chain_bench_create: ring capacity mismatch");
        preload_twice((char*)in_ring->device_base(), b->n_items * isz, n, first_index, seed, dev);
        b->sched->set_kernel_timing(true);
        *handle = b.release();
    });
}

int nsr_chain_bench_run(void* handle)
{
    return guarded([&] { static_cast<chain_bench*>(handle)->fg->run(); });
}

int nsr_chain_bench_set_batches(void* handle, int64_t batches)
{
    return guarded([&] {
        auto b = static_cast<chain_bench*>(handle);
        if (batches < 1) throw std::invalid_argument("nsr_chain_bench_set_batches: batches must be >= 1");
        b->head->set_length((size_t)(batches * b->n_items));
    });
}

int nsr_chain_bench_stats(void* handle, double* kernel_ms, uint64_t* launches, uint64_t* samples, char* block,
                          int len, int* n_launching_blocks)
{
    return guarded([&] {
        auto b = static_cast<chain_bench*>(handle);
        const auto st = b->sched->kernel_stats();
        schedulers::scheduler_hip::kernel_stat best;
        for (auto& k : st)
            if (k.kernel_ms >= best.kernel_ms) best = k;
        if (kernel_ms) *kernel_ms = best.kernel_ms;
        if (launches) *launches = best.launches;
        if (samples) *samples = best.items * b->spi; // output samples (decimators: n / D per batch)
        if (n_launching_blocks) *n_launching_blocks = (int)st.size();
        if (block && len > 0) {
            std::strncpy(block, best.block.c_str(), (size_t)len - 1);
            block[len - 1] = 0;
        }
    });
}

int nsr_chain_bench_tail(void* handle, int64_t count, float* out_host)
{
    return guarded([&] {
        auto b = static_cast<chain_bench*>(handle);
        if (count <= 0 || count % (int64_t)b->spi) throw std::invalid_argument("nsr_chain_bench_tail: whole items only");
        ring_tail(b->out_ring, b->dev, count / (int64_t)b->spi, out_host);
    });
}

int nsr_chain_bench_destroy(void* handle)
{
    return guarded([&] { delete static_cast<chain_bench*>(handle); });
}

int nsr_c1_run(int64_t n, size_t fixed_buf_size, double* seconds, int* threads)
{
    return guarded([&] {
        auto src = blocks::null_source::make(sizeof(gr_complex));
        auto head = blocks::head::make(sizeof(gr_complex), (size_t)n);
        auto cp = blocks::copy::make(sizeof(gr_complex));
        auto snk = blocks::null_sink::make(sizeof(gr_complex));
        auto fg = flowgraph::make();
        fg->connect(src, 0, head, 0);
        fg->connect(head, 0, cp, 0);
        fg->connect(cp, 0, snk, 0);
        auto sched = schedulers::scheduler_mt::make("mt", (unsigned)fixed_buf_size);
        fg->set_scheduler(sched);
        fg->validate();
        if (threads) *threads = (int)sched->num_threads();
        const auto t0 = std::chrono::steady_clock::now();
        fg->run();
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (snk->consumed() != (uint64_t)n) throw std::runtime_error("nsr_c1_run: short run");
    });
}

int nsr_c5_create(int group, int n_groups, int dev, const float* taps, int ntaps, int decim, int64_t n,
                  uint64_t first_index, uint64_t seed, const char* rendezvous_dir, uint64_t nonce,
                  const char* transport, size_t buf_bytes, void** handle)
{
    return guarded([&] {
        const int n_stages = 4;
        if (n_groups < 1 || n_stages % n_groups || group < 0 || group >= n_groups)
            throw std::invalid_argument("nsr_c5_create: n_groups must divide 4 and 0 <= group < n_groups");
        int64_t total_decim = 1;
        for (int i = 0; i < n_stages; ++i) total_decim *= decim;
        if (n <= 0 || n % total_decim) throw std::invalid_argument("nsr_c5_create: n must be a multiple of decim^4");
        auto b = std::make_unique<c5_pipeline>();
        b->dev = dev;
        const size_t isz = sizeof(gr_complex);
        const std::vector<float> h(taps, taps + ntaps);
        auto src = hip::synth_source::make(first_index, (uint64_t)n, seed);
        for (int i = 0; i < n_stages; ++i) b->stages.push_back(hip::fir_filter_ccf::make(h, decim));
        auto snk = blocks::null_sink::make(isz);
        b->fg = flowgraph::make();
        b->fg->connect(src, 0, b->stages[0], 0);
        for (int i = 1; i < n_stages; ++i) b->fg->connect(b->stages[i - 1], 0, b->stages[i], 0);
        b->fg->connect(b->stages[n_stages - 1], 0, snk, 0);

        // SPMD: every process builds the same graph and domain list; the domains of the
        // other groups are remote_domain placeholders (domain_adapter_remote.hpp)
        const int per = n_stages / n_groups;
        std::vector<scheduler_sptr> scheds;
        domain_conf_vec dc;
        remote_edge_options o;
        if (n_groups > 1 && (!rendezvous_dir || !*rendezvous_dir))
            throw std::invalid_argument("nsr_c5_create: n_groups > 1 needs a rendezvous directory");
        o.rendezvous_dir = rendezvous_dir ? rendezvous_dir : "";
        o.nonce = nonce;
        o.transport = transport && *transport ? transport : "auto";
        o.device = dev;
        o.timeout_s = 120;
        o.stall_timeout_s = 600; // a receiver wedged with its socket open: an error, not a hang
        b->da = domain_adapter_remote_conf::make(o);
        for (int g = 0; g < n_groups; ++g) {
            scheduler_sptr sc;
            if (g == group)
                sc = schedulers::scheduler_hip::make("c5g" + std::to_string(g), dev, buf_bytes);
            else
                sc = remote_domain::make(g, "c5g" + std::to_string(g));
            scheds.push_back(sc);
            std::vector<node_sptr> blks;
            if (g == 0) blks.push_back(src);
            for (int i = g * per; i < (g + 1) * per; ++i) blks.push_back(b->stages[i]);
            if (g == n_groups - 1) blks.push_back(snk);
            dc.emplace_back(sc, blks, b->da);
        }
        b->fg->set_wait_spin_us(5000);
        if (n_groups == 1) {
            b->fg->set_scheduler(scheds[0]);
            b->fg->validate();
        } else {
            b->fg->set_schedulers(scheds);
            b->fg->partition(dc);
        }
        if (group == n_groups - 1) {
            auto sh = std::dynamic_pointer_cast<schedulers::scheduler_hip>(scheds[group]);
            b->out_ring = std::dynamic_pointer_cast<hip_buffer>(sh->buffers()->get_input_buffer(snk->input_stream_ports()[0]));
            if (!b->out_ring) throw std::runtime_error("nsr_c5_create: the sink edge is not a hip_buffer");
        }
        *handle = b.release();
    });
}

int nsr_c5_run(void* handle)
{
    return guarded([&] { static_cast<c5_pipeline*>(handle)->fg->run(); });
}

int nsr_c5_transport(void* handle, char* buf, int len)
{
    return guarded([&] {
        auto b = static_cast<c5_pipeline*>(handle);
        std::string t;
        for (auto& a : b->da->adapters()) {
            if (!t.empty()) t += ",";
            t += (a->role() == remote_role::SEND ? "send" : "recv") + std::to_string(a->crossing()) + ":" +
                 a->transport_kind();
        }
        if (len <= 0) throw std::invalid_argument("nsr_c5_transport: len");
        std::strncpy(buf, t.c_str(), (size_t)len - 1);
        buf[len - 1] = 0;
    });
}

int nsr_rccl_library(char* buf, int len)
{
    return guarded([&] {
        if (len <= 0 || !buf) throw std::invalid_argument("nsr_rccl_library: len");
        const std::string p = domain_adapter_remote::rccl_library();
        std::strncpy(buf, p.c_str(), (size_t)len - 1);
        buf[len - 1] = 0;
    });
}

int nsr_rccl_self_test(int dev, const void* src, void* dst, size_t bytes, void* stream, int peer)
{
    return guarded([&] { domain_adapter_remote::rccl_self_test(dev, src, dst, bytes, stream, peer); });
}

int nsr_c5_tail(void* handle, int64_t count, float* out_host)
{
    return guarded([&] {
        auto b = static_cast<c5_pipeline*>(handle);
        if (!b->out_ring) throw std::invalid_argument("nsr_c5_tail: this process does not own the sink");
        ring_tail(b->out_ring, b->dev, count, out_host);
    });
}

int nsr_c5_destroy(void* handle)
{
    return guarded([&] { delete static_cast<c5_pipeline*>(handle); });
}

int nsr_cpu_fir_work_only(const float* taps, int ntaps, const float* x, int64_t nx, int64_t n, int chunk, double* seconds,
                          char* isa, int len)
{
    return guarded([&] {
        if (chunk <= 0 || nx < chunk || nx % chunk) throw std::invalid_argument("nsr_cpu_fir_work_only: nx must be a multiple of chunk");
        auto fir = blocks::fir_filter_ccf::make(std::vector<float>(taps, taps + ntaps), 1);
        fir->start();
        std::vector<gr_complex> y((size_t)chunk);
        const gr_complex* xc = (const gr_complex*)x;
        const auto t0 = std::chrono::steady_clock::now();
        int64_t off = 0;
        for (int64_t done = 0; done < n; done += chunk) {
            const int m = (int)std::min<int64_t>(chunk, n - done);
            fir->filter(xc + off, y.data(), m);
            off = (off + chunk) % nx;
        }
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (isa && len > 0) {
            std::strncpy(isa, blocks::cpu_isa(), (size_t)len - 1);
            isa[len - 1] = 0;
        }
    });
}

int nsr_cpu_fir_run(const float* taps, int ntaps, const float* x, int64_t nx, int64_t n, size_t fixed_buf_size,
                    double* seconds, int* threads)
{
    return guarded([&] {
        std::vector<gr_complex> xv((const gr_complex*)x, (const gr_complex*)x + nx);
        auto src = blocks::vector_source_c::make(xv, true);
        auto head = blocks::head::make(sizeof(gr_complex), (size_t)n);
        auto fir = blocks::fir_filter_ccf::make(std::vector<float>(taps, taps + ntaps), 1);
        auto snk = blocks::null_sink::make(sizeof(gr_complex));
        auto fg = flowgraph::make();
        fg->connect(src, 0, head, 0);
        fg->connect(head, 0, fir, 0);
        fg->connect(fir, 0, snk, 0);
        auto sched = schedulers::scheduler_mt::make("mt", (unsigned)fixed_buf_size);
        fg->set_scheduler(sched);
        fg->validate();
        if (threads) *threads = (int)sched->num_threads(); // thread per block (reference scheduler_mt)
        const auto t0 = std::chrono::steady_clock::now();
        fg->run();
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (snk->consumed() != (uint64_t)n) throw std::runtime_error("nsr_cpu_fir_run: short run");
    });
}

} // extern "C"
