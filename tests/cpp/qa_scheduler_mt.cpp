// Behaviour tests of the CPU runtime restatement. The first three restate the reference's
// gtests verbatim in intent (schedulers/mt/test/qa_scheduler_mt.cpp:17-39 TwoSinks,
// :79-135 BlockFanout; qa_block_grouping.cpp:15-66 BasicBlockGrouping); DomainAdapterBasic
// enables the reference's disabled test (:40-78). The rest cover what this runtime adds:
// drain-based termination, restart, decimating FIR history, error propagation.
#include "qa.hpp"
#include "qa_ref.hpp"

#include <cmath>
#include <gnuradio/blocklib/blocks/arith.hpp>
#include <gnuradio/blocklib/blocks/copy.hpp>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/multiply_const.hpp>
#include <gnuradio/blocklib/blocks/nop.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/blocks/vector_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

using namespace gr;

static std::vector<gr_complex> ramp(int n)
{
    std::vector<gr_complex> v(n);
    for (int i = 0; i < n; ++i) v[i] = gr_complex(2 * i, 2 * i + 1);
    return v;
}

TEST(SchedulerMTTest, TwoSinks)
{
    std::vector<float> input_data{ 1.0, 2.0, 3.0, 4.0, 5.0 };
    auto src = blocks::vector_source_f::make(input_data, false);
    auto snk1 = blocks::vector_sink_f::make();
    auto snk2 = blocks::vector_sink_f::make();
    auto fg = flowgraph::make();
    fg->connect(src, 0, snk1, 0);
    fg->connect(src, 0, snk2, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make());
    fg->validate();
    fg->start();
    fg->wait();
    EXPECT_EQ(snk1->data(), input_data);
    EXPECT_EQ(snk2->data(), input_data);
}

TEST(SchedulerMTTest, BlockFanout)
{
    const int nsamples = 1000000;
    const auto input_data = ramp(nsamples);
    for (int nblocks : { 2, 8, 16 }) {
        auto src = blocks::vector_source_c::make(input_data);
        std::vector<blocks::vector_sink_c::sptr> snk(nblocks);
        std::vector<blocks::multiply_const_cc::sptr> mul(nblocks);
        auto fg = flowgraph::make();
        for (int i = 0; i < nblocks; ++i) {
            mul[i] = blocks::multiply_const_cc::make(1.0f, 1);
            snk[i] = blocks::vector_sink_c::make();
            fg->connect(src, 0, mul[i], 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
            fg->connect(mul[i], 0, snk[i], 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
        }
        fg->add_scheduler(schedulers::scheduler_mt::make("mtsched", 8192));
        fg->validate();
        fg->start();
        fg->wait();
        for (int i = 0; i < nblocks; ++i) {
            EXPECT_EQ(snk[i]->data().size(), input_data.size());
            EXPECT_TRUE(snk[i]->data() == input_data);
        }
    }
}

TEST(SchedulerBlockGrouping, BasicBlockGrouping)
{
    const int nsamples = 1000000;
    const auto input_data = ramp(nsamples);
    for (int ngroups : { 2, 4, 8 }) {
        for (int nblocks : { 2, 8, 16 }) {
            auto src = blocks::vector_source_c::make(input_data);
            auto snk = blocks::vector_sink_c::make();
            std::vector<blocks::multiply_const_cc::sptr> mul(nblocks * ngroups);
            for (auto& m : mul) m = blocks::multiply_const_cc::make(1.0f, 1);
            auto fg = flowgraph::make();
            auto sch = schedulers::scheduler_mt::make("mtsched");
            fg->connect(src, 0, mul[0], 0);
            for (int n = 0; n < ngroups; ++n) {
                std::vector<block_sptr> bg;
                for (int i = 0; i < nblocks; ++i) {
                    const int idx = n * nblocks + i;
                    if (idx > 0) fg->connect(mul[idx - 1], 0, mul[idx], 0);
                    bg.push_back(mul[idx]);
                }
                sch->add_block_group(bg);
            }
            fg->connect(mul[nblocks * ngroups - 1], 0, snk, 0);
            fg->add_scheduler(sch);
            fg->validate();
            fg->start();
            fg->wait();
            EXPECT_TRUE(snk->data() == input_data);
        }
    }
}

TEST(SchedulerMTTest, DomainAdapterBasic)
{
    std::vector<float> input_data{ 1.0, 2.0, 3.0, 4.0, 5.0 };
    std::vector<float> expected;
    for (auto d : input_data) expected.push_back(100.0f * 200.0f * d);
    auto src = blocks::vector_source_f::make(input_data, false);
    auto m1 = blocks::multiply_const_ff::make(100.0f);
    auto m2 = blocks::multiply_const_ff::make(200.0f);
    auto snk = blocks::vector_sink_f::make();
    auto fg = flowgraph::make();
    fg->connect(src, 0, m1, 0);
    fg->connect(m1, 0, m2, 0);
    fg->connect(m2, 0, snk, 0);
    auto s1 = schedulers::scheduler_mt::make("sched1");
    auto s2 = schedulers::scheduler_mt::make("sched2");
    fg->add_scheduler(s1);
    fg->add_scheduler(s2);
    for (auto pref : { buffer_preference_t::UPSTREAM, buffer_preference_t::DOWNSTREAM }) {
        auto da = domain_adapter_direct_conf::make(pref);
        domain_conf_vec dconf{ domain_conf(s1, { src, m1 }, da), domain_conf(s2, { m2, snk }, da) };
        fg->partition(dconf);
        fg->start();
        fg->wait();
        EXPECT_EQ(snk->data(), expected);
    }
}

TEST(SchedulerMTTest, RestartAcrossDomainsNeverHangs)
{
    // The restart path of the race fixed in flowgraph::start(): fresh
    // two-domain flowgraphs, each run twice, both buffer preferences. Each scheduler used to
    // reset its own edges' done flags inside start(), after the other domain's threads had begun
    // the run; the host -> GPU -> host variant hung within tens of iterations
    // (tests/test_restart_stress.py). This all-host variant did not reproduce it on its own
    // timing; it guards the restart sequence on the CPU suite.
    const auto data = ramp(20000);
    for (int it = 0; it < 150; ++it) {
        auto src = blocks::vector_source_c::make(data);
        auto m1 = blocks::multiply_const_cc::make(gr_complex(0.5f, 0.f));
        auto m2 = blocks::multiply_const_cc::make(gr_complex(2.f, 0.f));
        auto snk = blocks::vector_sink_c::make();
        auto fg = flowgraph::make();
        fg->connect(src, 0, m1, 0);
        fg->connect(m1, 0, m2, 0);
        fg->connect(m2, 0, snk, 0);
        auto s1 = schedulers::scheduler_mt::make("a", 4096);
        auto s2 = schedulers::scheduler_mt::make("b", 4096);
        fg->add_scheduler(s1);
        fg->add_scheduler(s2);
        auto da = domain_adapter_direct_conf::make(it % 2 ? buffer_preference_t::UPSTREAM : buffer_preference_t::DOWNSTREAM);
        domain_conf_vec dconf{ domain_conf(s1, { src, m1 }, da), domain_conf(s2, { m2, snk }, da) };
        fg->partition(dconf);
        for (int r = 0; r < 2; ++r) {
            fg->run();
            EXPECT_EQ(snk->data().size(), data.size());
        }
    }
}

TEST(SchedulerMTTest, NullSourceHeadCopyNullSink)
{
    // BASELINE config C1 (reference schedulers/mt/bench/bm_copy.cpp:77-101 shape)
    const size_t n = 1u << 20;
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), n);
    auto cp = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, cp, 0);
    fg->connect(cp, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 32768));
    fg->validate();
    const auto t0 = std::chrono::steady_clock::now();
    fg->run();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    EXPECT_EQ(snk->consumed(), (uint64_t)n);
    EXPECT_TRUE(s < 5.0); // drains, no fixed 100 ms sleep per termination stage
}

TEST(SchedulerMTTest, RestartRunsAgain)
{
    const auto data = ramp(50000);
    auto src = blocks::vector_source_c::make(data);
    auto mul = blocks::multiply_const_cc::make(gr_complex(0.5f, -0.25f));
    auto snk = blocks::vector_sink_c::make();
    auto fg = flowgraph::make();
    fg->connect(src, 0, mul, 0);
    fg->connect(mul, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 4096));
    fg->validate();
    std::vector<gr_complex> first;
    for (int run = 0; run < 3; ++run) {
        fg->run();
        auto d = snk->data();
        EXPECT_EQ(d.size(), data.size());
        if (run == 0)
            first = d;
        else
            EXPECT_TRUE(d == first);
    }
    // same per-product rounding as the formula
    bool ok = true;
    for (size_t i = 0; i < data.size(); ++i) {
        const float ar = data[i].real(), ai = data[i].imag();
        volatile float p0 = ar * 0.5f, p1 = ai * -0.25f, p2 = ar * -0.25f, p3 = ai * 0.5f;
        if (first[i] != gr_complex(p0 - p1, p2 + p3)) ok = false;
    }
    EXPECT_TRUE(ok);
}

TEST(SchedulerMTTest, CpuFirAcrossChunks)
{
    std::vector<gr_complex> x(100003);
    for (size_t i = 0; i < x.size(); ++i) x[i] = gr_complex(std::sin(0.001f * i * i), std::cos(0.37f * i));
    // every tap-residue shape of the rolling-window kernel (blocks_cpu.cpp): fewer taps than one
    // 8-tap stride, exact multiples, one over, and the C3 / C5 length
    for (int L : { 1, 2, 7, 8, 9, 16, 17, 63, 127, 128, 161 }) {
        std::vector<float> h(L);
        for (int k = 0; k < L; ++k) h[k] = 0.02f * std::cos(0.1f * k) * (k % 7 == 3 ? -1.0f : 1.0f);
        for (int D : { 1, 2, 4 }) {
            auto src = blocks::vector_source_c::make(x);
            auto fir = blocks::fir_filter_ccf::make(h, D);
            auto snk = blocks::vector_sink_c::make();
            auto fg = flowgraph::make();
            fg->connect(src, 0, fir, 0);
            fg->connect(fir, 0, snk, 0);
            fg->set_scheduler(schedulers::scheduler_mt::make("mt", 4096)); // many small work() calls
            fg->validate();
            fg->run();
            const auto y = snk->data();
            const auto r = fir_ref(x, h, D);
            EXPECT_EQ(y.size(), r.size());
            double maxerr = 0, scale = 0;
            for (size_t i = 0; i < std::min(y.size(), r.size()); ++i) {
                maxerr = std::max(maxerr, (double)std::abs(y[i] - r[i]));
                scale = std::max(scale, (double)std::abs(r[i]));
            }
            if (!(maxerr <= 1e-5 * scale)) std::printf("  L=%d D=%d maxerr %.3g scale %.3g\n", L, D, maxerr, scale);
            EXPECT_TRUE(maxerr <= 1e-5 * scale);
        }
    }
}

// A decimator leaves its input's remainder below one output unread at the end of a run; a
// restarted run must not read it as the start of its stream (buffer::discard_unread()). The
// source ran 100003 items into a decimate-by-4 chain of two stages: 3 and then 0 or 1 items stay.
TEST(SchedulerMTTest, RestartDropsUnreadItems)
{
    std::vector<float> h(31);
    for (int k = 0; k < 31; ++k) h[k] = 0.03f * std::cos(0.2f * k);
    std::vector<gr_complex> x(100003);
    for (size_t i = 0; i < x.size(); ++i) x[i] = gr_complex(std::sin(0.01f * i), std::cos(0.37f * i));
    auto src = blocks::vector_source_c::make(x);
    auto f1 = blocks::fir_filter_ccf::make(h, 4);
    auto f2 = blocks::fir_filter_ccf::make(h, 2);
    auto snk = blocks::vector_sink_c::make();
    auto fg = flowgraph::make();
    fg->connect(src, 0, f1, 0);
    fg->connect(f1, 0, f2, 0);
    fg->connect(f2, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 4096));
    fg->validate();
    std::vector<gr_complex> first;
    for (int run = 0; run < 3; ++run) {
        fg->run();
        const auto y = snk->data();
        EXPECT_EQ(y.size(), x.size() / 8);
        if (run == 0)
            first = y;
        else
            EXPECT_TRUE(y == first);
    }
}

struct failing_block : sync_block {
    failing_block() : sync_block("failing") {}
    static std::shared_ptr<failing_block> make()
    {
        auto p = std::make_shared<failing_block>();
        p->add_port(port<float>::make("in", port_direction_t::INPUT));
        p->add_port(port<float>::make("out", port_direction_t::OUTPUT));
        return p;
    }
    work_return_code_t work(std::vector<block_work_input>&, std::vector<block_work_output>&) override
    {
        return work_return_code_t::WORK_ERROR; // the reference executor would spin forever
    }
};

TEST(SchedulerMTTest, WorkErrorThrowsInsteadOfSpinning)
{
    auto src = blocks::vector_source_f::make(std::vector<float>(1000, 1.0f));
    auto bad = failing_block::make();
    auto snk = blocks::vector_sink_f::make();
    auto fg = flowgraph::make();
    fg->connect(src, 0, bad, 0);
    fg->connect(bad, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make());
    fg->validate();
    bool threw = false;
    try {
        fg->run();
    } catch (const std::runtime_error&) {
        threw = true;
    }
    EXPECT_TRUE(threw);
}

TEST(SchedulerMTTest, AddMultiplyTwoInputs)
{
    const auto a = ramp(20000);
    std::vector<gr_complex> b(20000);
    for (int i = 0; i < 20000; ++i) b[i] = gr_complex(0.5f * i, -1.0f);
    auto sa = blocks::vector_source_c::make(a);
    auto sb = blocks::vector_source_c::make(b);
    auto add = blocks::add_cc::make(2);
    auto snk = blocks::vector_sink_c::make();
    auto fg = flowgraph::make();
    fg->connect(sa, 0, add, 0);
    fg->connect(sb, 0, add, 1);
    fg->connect(add, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 2048));
    fg->validate();
    fg->run();
    auto y = snk->data();
    EXPECT_EQ(y.size(), a.size());
    bool ok = y.size() == a.size();
    for (size_t i = 0; ok && i < y.size(); ++i) ok = y[i] == a[i] + b[i];
    EXPECT_TRUE(ok);
}

// decim_block (reference block.hpp:86-99 names it; buffer_management.cpp:125-145 has the
// sizing rule commented out): with a 32-byte fixed_buf_size the rule gives the edge into a
// decimate-by-8 FIR 2 * D = 16 items instead of 8 (vmcircbuf's page rounding would hide the
// difference at run time, so the size is checked directly), and decim_block::do_work clamps
// and consumes D items per output.
TEST(DecimBlock, TinyBuffersStillFlow)
{
    const size_t n = 4096;
    auto x = synth(n, 77);
    const auto h = lowpass(31, 0.05);
    auto src = blocks::vector_source_c::make(x);
    auto fir = blocks::fir_filter_ccf::make(h, 8);
    auto snk = blocks::vector_sink_c::make(1, n / 8);
    auto fg = flowgraph::make();
    fg->connect(src, 0, fir, 0);
    fg->connect(fir, 0, snk, 0);
    auto sched = schedulers::scheduler_mt::make("mt", 32);
    fg->set_scheduler(sched);
    fg->validate();
    fg->run();
    EXPECT_EQ(fir->relative_rate(), 1.0 / 8);
    schedulers::buffer_manager bm(32);
    auto ffg = flat_graph::make_flat(fg);
    for (auto& e : ffg->edges()) {
        if (e->dst().node() == fir) EXPECT_EQ(bm.get_buffer_num_items(e, ffg), (size_t)16);
        if (e->dst().node() == snk) EXPECT_EQ(bm.get_buffer_num_items(e, ffg), (size_t)8);
    }
    EXPECT_TRUE(close_normwise(snk->data(), fir_ref(x, h, 8)));
}
