// Stress the host-endpoint C3 flowgraph (vector_source -> head -[H2D]-> hip::fir_filter_ccf
// -[D2H]-> null_sink; host blocks in scheduler_mt, the FIR in scheduler_hip) to reproduce an
// intermittent hang at run end. Builds a fresh flowgraph per iteration, runs it twice, prints a
// line per iteration (so a hang shows as the last line). Usage: c3host_stress [iters] [log2n]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>
#include <vector>

using namespace gr;

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 100;
    const int64_t nh = (int64_t)1 << (argc > 2 ? std::atoi(argv[2]) : 22);
    std::vector<float> h(127, 1.f / 127);
    std::vector<gr_complex> x(1 << 20, gr_complex(0.5f, -0.25f));
    const size_t buf = (size_t)16 << 20;
    auto mark = [](int it, const char* what) {
        std::printf("iter %d %s\n", it, what);
        std::fflush(stdout);
    };
    for (int it = 0; it < iters; ++it) {
      {
        const auto t0 = std::chrono::steady_clock::now();
        auto src = blocks::vector_source_c::make(x, true);
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
        mark(it, "built");
        for (int r = 0; r < 2; ++r) {
            fg->run();
            mark(it, r == 0 ? "run0 done" : "run1 done");
            if (snk->consumed() != (uint64_t)nh * (r + 1) && snk->consumed() != (uint64_t)nh)
                std::printf("iter %d run %d: sink consumed %llu\n", it, r, (unsigned long long)snk->consumed());
        }
        std::printf("iter %d ok %.1f ms\n", it,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3);
        std::fflush(stdout);
      }
        mark(it, "destroyed");
    }
    return 0;
}
