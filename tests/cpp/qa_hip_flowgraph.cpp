// GPU behaviour/parity tests of the MI355X block-execution path through the runtime:
// blocks -> graph_executor -> work() -> libnsh_hip.so, with hip_buffer edges.
//   CudaCopy{Basic,MultiThreaded}  restate schedulers/mt/test/cuda/qa_scheduler_mt_cuda_copy.cpp:20-86
//                                  (H2D -> copy -> D2D -> copy -> D2H, exact equality)
//   Fusion*                        scheduler_hip's elementwise fusion (bit-identical on/off;
//                                  BasicBlockGrouping's 128-block identity chain restated)
//   the others cover BASELINE configs C2-C5 in the GPU scheduler domain against in-test
//   CPU references (bit-exact where the arithmetic is the same formula; 1e-5 norm-wise
//   for FIR/FFT), restart, and cross-thread device edges (event ordering).
#include "qa.hpp"

#include <cmath>
#include <complex>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/multiply_const.hpp>
#include <gnuradio/blocklib/blocks/nop.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/blocks/vector_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/arith.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/fir_filter_cascade_ccf.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/blocklib/hip/synth_source.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>
#include <gnuradio/vmcircbuf.hpp>

using namespace gr;

#include "qa_ref.hpp"

// ---- reference CudaCopy tests restated --------------------------------------------------
static void cuda_copy_case(bool one_group)
{
    const int veclen = 1024, num_samples = veclen * 100;
    std::vector<gr_complex> input(num_samples);
    for (int i = 0; i < num_samples; ++i) input[i] = gr_complex((float)i, (float)-i);
    auto src = blocks::vector_source_c::make(input, false, veclen);
    auto snk = blocks::vector_sink_c::make(veclen);
    auto c1 = hip::copy::make(veclen);
    auto c2 = hip::copy::make(veclen);
    auto fg = flowgraph::make();
    fg->connect(src, 0, c1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(c1, 0, c2, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(c2, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto sched = schedulers::scheduler_mt::make("sched", 32768);
    fg->set_scheduler(sched);
    if (one_group) sched->add_block_group({ c1, c2 });
    fg->validate();
    fg->start();
    fg->wait();
    EXPECT_TRUE(snk->data() == input);
}
TEST(SchedulerMTTest, CudaCopyBasic) { cuda_copy_case(true); }
TEST(SchedulerMTTest, CudaCopyMultiThreaded) { cuda_copy_case(false); }

// The reference's CUDA copy benchmark flowgraph (schedulers/mt/bench/cuda/bm_copy.cpp:55-100),
// mem_model 0, with hip::copy::make(batch_size, load) and the HIP_BUFFER_ARGS_* edges:
// null_source -> head -[H2D]-> copy x nblocks -[D2D]...-[D2H]-> null_sink, one scheduler_mt
// with vmcirc default buffers of 2 items. Every sample must arrive; with load > 1 each copy
// block repeats its pass (and is not fused).
static void bm_copy_case(int nblocks, int load, int batch_size, uint64_t samples)
{
    std::vector<hip::copy::sptr> copy_blks(nblocks);
    for (int i = 0; i < nblocks; i++) copy_blks[i] = hip::copy::make(batch_size, load);
    auto src = blocks::null_source::make(sizeof(gr_complex) * batch_size);
    auto snk = blocks::null_sink::make(sizeof(gr_complex) * batch_size);
    auto head = blocks::head::make(sizeof(gr_complex) * batch_size, samples / batch_size);
    auto fg = flowgraph::make();
    fg->connect(src, 0, head, 0)->set_custom_buffer(VMCIRC_BUFFER_ARGS);
    auto sched = schedulers::scheduler_mt::make("sched", sizeof(gr_complex) * batch_size * 2);
    sched->set_default_buffer_factory(VMCIRC_BUFFER_ARGS);
    fg->set_scheduler(sched);
    fg->connect(head, 0, copy_blks[0], 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    for (int i = 0; i < nblocks - 1; i++)
        fg->connect(copy_blks[i], 0, copy_blks[i + 1], 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(copy_blks[nblocks - 1], 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->validate();
    fg->start();
    fg->wait();
    EXPECT_EQ(snk->consumed(), samples / batch_size);
    EXPECT_EQ(copy_blks[0]->load(), (size_t)load);
}
TEST(SchedulerMTTest, BmCopyFlowgraph) { bm_copy_case(4, 1, 1024, 1500000); }
TEST(SchedulerMTTest, BmCopyFlowgraphLoad) { bm_copy_case(4, 3, 1024, 500000); }

// ---- GPU scheduler domain ---------------------------------------------------------------
TEST(HipDomain, FirMatchesCpuAndReruns)
{
    const size_t n = 3 * 1000003; // not a multiple of any chunk
    const auto h = lowpass(127, 0.1);
    auto src = hip::synth_source::make(0, n);
    auto fir = hip::fir_filter_ccf::make(h);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, fir, 0);
    fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->set_scheduler(schedulers::scheduler_hip::make("hip", 0, 1u << 20)); // small rings: many work() calls
    fg->validate();
    fg->run();
    const auto y = snk->data();
    const auto ref = fir_ref(synth(n), h, 1);
    EXPECT_TRUE(close_normwise(y, ref));
    fg->run(); // restart: history and counters re-armed
    EXPECT_TRUE(snk->data() == y || close_normwise(snk->data(), ref));
}

TEST(HipDomain, DirectFirBitExactAcrossRuns)
{
    const size_t n = 777777;
    const auto h = lowpass(127, 0.2);
    auto src = hip::synth_source::make(0, n);
    auto fir = hip::fir_filter_ccf::make(h, 1, 1 /*DIRECT*/);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, fir, 0);
    fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->set_scheduler(schedulers::scheduler_hip::make("hip", 0, 1u << 18));
    fg->validate();
    fg->run();
    const auto y1 = snk->data();
    EXPECT_TRUE(close_normwise(y1, fir_ref(synth(n), h, 1)));
    fg->run();
    EXPECT_TRUE(snk->data() == y1);
}

TEST(HipDomain, MultiplyChainC2)
{
    // variant 0: one hand-built multiply_const_chain_cc; 1: four multiply_const_cc blocks,
    // fused by scheduler_hip; 2: the same four blocks with fusion off (every edge in HBM).
    // All bit-identical to the per-stage product.
    const size_t n = 1u << 22;
    const std::vector<gr_complex> ks = { std::polar(1.0f, 0.1f), std::polar(1.0f, 0.2f), std::polar(1.0f, 0.3f),
                                         std::polar(1.0f, 0.4f) };
    auto x = synth(n);
    std::vector<gr_complex> ref(x);
    for (auto k : ks)
        for (auto& v : ref) v = cmul(v, k);
    for (int variant = 0; variant < 3; ++variant) {
        auto src = hip::synth_source::make(0, n);
        auto snk = blocks::vector_sink_c::make(1, n);
        auto fg = flowgraph::make();
        if (variant == 0) {
            auto ch = hip::multiply_const_chain_cc::make(ks);
            fg->connect(src, 0, ch, 0);
            fg->connect(ch, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        } else {
            std::vector<hip::multiply_const_cc::sptr> m;
            for (auto k : ks) m.push_back(hip::multiply_const_cc::make(k));
            fg->connect(src, 0, m[0], 0);
            for (size_t i = 1; i < m.size(); ++i) fg->connect(m[i - 1], 0, m[i], 0);
            fg->connect(m.back(), 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        }
        auto sched = schedulers::scheduler_hip::make("hip", 0, 4u << 20);
        sched->set_fusion(variant != 2);
        fg->set_scheduler(sched);
        fg->validate();
        EXPECT_EQ(sched->fusion_plan().fused.size(), variant == 1 ? 1u : 0u);
        fg->run();
        EXPECT_TRUE(snk->data() == ref);
        if (variant == 1) { // restart through the fused graph
            fg->run();
            EXPECT_TRUE(snk->data() == ref);
        }
    }
}

// scheduler_hip's kernel timing (set_kernel_timing / kernel_stats, bench.py's legs): every work()
// call that launches records its own event pair; calls that launch nothing (the synthetic source
// here launches k_synth -- the sink does not) are not counted. Fusion on: the four multiply blocks
// are one block with one launch per work() call; off: four blocks, each with the same count. Off
// by default; reset clears; the outputs stay bit-exact with timing on.
TEST(HipDomain, KernelTimingPerBlock)
{
    const size_t n = 1u << 20;
    const std::vector<gr_complex> ks = { std::polar(1.0f, 0.1f), std::polar(1.0f, 0.2f), std::polar(1.0f, 0.3f),
                                         std::polar(1.0f, 0.4f) };
    auto x = synth(n);
    std::vector<gr_complex> ref(x);
    for (auto k : ks)
        for (auto& v : ref) v = cmul(v, k);
    for (int fused = 1; fused >= 0; --fused) {
        auto src = hip::synth_source::make(0, n);
        std::vector<hip::multiply_const_cc::sptr> m;
        for (auto k : ks) m.push_back(hip::multiply_const_cc::make(k));
        auto snk = blocks::vector_sink_c::make(1, n);
        auto fg = flowgraph::make();
        fg->connect(src, 0, m[0], 0);
        for (size_t i = 1; i < m.size(); ++i) fg->connect(m[i - 1], 0, m[i], 0);
        fg->connect(m.back(), 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 20); // 128 Ki samples per call: 8 calls
        sched->set_fusion(fused == 1);
        fg->set_scheduler(sched);
        fg->validate();
        fg->run();
        EXPECT_TRUE(sched->kernel_stats().empty()); // off by default
        sched->set_kernel_timing(true);
        fg->run();
        EXPECT_TRUE(snk->data() == ref);
        auto st = sched->kernel_stats();
        // the source (k_synth) and the multiply blocks launch; the D2H sink's edge copy is not a work() launch
        size_t mul_blocks = 0;
        uint64_t src_calls = 0;
        for (auto& k : st) {
            EXPECT_TRUE(k.launches > 0 && k.kernel_ms > 0);
            if (k.block.find("multiply_const") != std::string::npos) {
                ++mul_blocks;
                EXPECT_EQ(k.items, (uint64_t)n); // every sample once per block
            } else if (k.block.find("synth") != std::string::npos) {
                src_calls = k.launches;
            } else {
                std::printf("  unexpected launching block: %s\n", k.block.c_str());
                EXPECT_TRUE(false);
            }
        }
        EXPECT_EQ(mul_blocks, fused ? 1u : 4u);
        for (auto& k : st)
            if (k.block.find("multiply_const") != std::string::npos) EXPECT_EQ(k.launches, src_calls);
        std::printf("  fused=%d: %zu launching blocks, %llu calls each\n", fused, st.size(), (unsigned long long)src_calls);
        sched->reset_kernel_stats();
        EXPECT_TRUE(sched->kernel_stats().empty());
        sched->set_kernel_timing(false);
        fg->run();
        EXPECT_TRUE(sched->kernel_stats().empty());
        EXPECT_TRUE(snk->data() == ref);
    }
}

// Both timings on at once (documented as unsupported: the block's own pair displaces the
// scheduler's): nothing throws, the block's own times are intact, and the scheduler does not count
// the displaced pairs as launches of the FIR.
TEST(HipDomain, KernelTimingDisplacedByBlockTiming)
{
    const size_t n = 1u << 18;
    std::vector<float> h(127);
    for (int k = 0; k < 127; ++k) h[k] = 0.01f * std::cos(0.05f * k);
    auto src = hip::synth_source::make(0, n);
    auto fir = hip::fir_filter_ccf::make(h, 1);
    fir->enable_timing(true);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, fir, 0);
    fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto sched = schedulers::scheduler_hip::make("hip", 0, 256u << 10);
    fg->set_scheduler(sched);
    fg->validate();
    sched->set_kernel_timing(true);
    fg->run();
    bool threw = false;
    std::vector<schedulers::scheduler_hip::kernel_stat> st;
    try {
        st = sched->kernel_stats();
    } catch (const std::exception& e) {
        threw = true;
        std::printf("  kernel_stats threw: %s\n", e.what());
    }
    EXPECT_TRUE(!threw);
    for (auto& k : st) EXPECT_TRUE(k.block.find("fir_filter_ccf") == std::string::npos);
    EXPECT_TRUE(fir->timed_launches() > 0 && fir->kernel_ms() > 0);
    EXPECT_EQ(snk->data().size(), n);
}

// Reference BasicBlockGrouping (schedulers/mt/test/qa_block_grouping.cpp:15-66) in the GPU
// domain: 128 chained multiply_const(1) blocks are the identity. scheduler_hip fuses them
// into 8 blocks of 16 stages (the fused kernel's limit).
TEST(HipDomain, Fusion128BlockIdentityChain)
{
    const size_t n = 1000003;
    auto src = hip::synth_source::make(0, n);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    block_sptr prev = src;
    for (int i = 0; i < 128; ++i) {
        auto m = hip::multiply_const_cc::make(gr_complex(1.0f, 0.0f));
        fg->connect(prev, 0, m, 0);
        prev = m;
    }
    fg->connect(prev, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 20);
    fg->set_scheduler(sched);
    fg->validate();
    EXPECT_EQ(sched->fusion_plan().fused.size(), 8u);
    fg->run();
    EXPECT_TRUE(snk->data() == synth(n));
}

// A fused chain whose ends are domain crossings (CPU -[H2D]-> m1 -> copy -> m2 -[D2H]-> CPU)
// and a fan-out inside the GPU domain: results identical with fusion on and off.
TEST(HipDomain, FusionAcrossDomainsAndFanOut)
{
    const size_t n = 400000;
    auto x = synth(n, 4242);
    const gr_complex k1(0.5f, -0.25f), k2(-1.5f, 0.75f), k3(0.0f, 1.0f);
    std::vector<gr_complex> r1(x), r2(x);
    for (auto& v : r1) v = cmul(cmul(v, k1), k2);
    for (auto& v : r2) v = cmul(cmul(v, k1), k3);
    for (int fuse = 1; fuse >= 0; --fuse) {
        auto src = blocks::vector_source_c::make(x);
        auto m1 = hip::multiply_const_cc::make(k1);
        auto cp = hip::copy::make(1);
        auto m2 = hip::multiply_const_cc::make(k2);
        auto m3 = hip::multiply_const_cc::make(k3);
        auto cp3 = hip::copy::make(1);
        auto s1 = blocks::vector_sink_c::make(1, n);
        auto s2 = blocks::vector_sink_c::make(1, n);
        auto fg = flowgraph::make();
        fg->connect(src, 0, m1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
        fg->connect(m1, 0, cp, 0);  // m1 fans out: a chain boundary
        fg->connect(m1, 0, m3, 0);
        fg->connect(cp, 0, m2, 0);  // cp -> m2 fused
        fg->connect(m3, 0, cp3, 0); // m3 -> cp3 fused
        fg->connect(m2, 0, s1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        fg->connect(cp3, 0, s2, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto cpu = schedulers::scheduler_mt::make("cpu", 1u << 16);
        auto gpu = schedulers::scheduler_hip::make("gpu", 0, 1u << 18);
        gpu->set_fusion(fuse);
        fg->add_scheduler(cpu);
        fg->add_scheduler(gpu);
        auto da = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
        domain_conf_vec dc{ domain_conf(cpu, { src, s1, s2 }, da), domain_conf(gpu, { m1, cp, m2, m3, cp3 }, da) };
        fg->partition(dc);
        EXPECT_EQ(gpu->fusion_plan().fused.size(), fuse ? 2u : 0u);
        for (int run = 0; run < 2; ++run) {
            fg->run();
            EXPECT_TRUE(s1->data() == r1);
            EXPECT_TRUE(s2->data() == r2);
        }
    }
}

// A fused, domain-partitioned flowgraph initialized twice (partition() again after a run):
// the second fusion pass must start from the user's original port links (ADVICE r1:
// release_fused() restores them), and the crossing notifications must reach the new fused
// block -- the run completes with the same, bit-exact output.
TEST(HipDomain, FusedPartitionInitializedTwice)
{
    const size_t n = 1u << 20;
    auto src = hip::synth_source::make(0, n);
    auto m0 = hip::multiply_const_cc::make(gr_complex(0.5f, 0.25f));
    auto m1 = hip::multiply_const_cc::make(gr_complex(-1.0f, 2.0f));
    auto cp = hip::copy::make(1);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, m0, 0);
    fg->connect(m0, 0, m1, 0);
    fg->connect(m1, 0, cp, 0);
    fg->connect(cp, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = schedulers::scheduler_hip::make("hip0", 0, 1u << 20);
    auto s1 = schedulers::scheduler_mt::make("mt", 32768);
    fg->set_schedulers({ s0, s1 });
    auto da = domain_adapter_direct_conf::make(buffer_preference_t::UPSTREAM);
    std::vector<gr_complex> first;
    for (int round = 0; round < 2; ++round) {
        domain_conf_vec dc{ domain_conf(s0, { src, m0, m1, cp }, da), domain_conf(s1, { snk }, da) };
        fg->partition(dc);
        fg->run();
        EXPECT_EQ(s0->fusion_plan().fused.size(), 1u);
        if (round == 0)
            first = snk->data();
        else
            EXPECT_TRUE(snk->data() == first);
    }
    auto x = synth(n);
    for (auto& v : x) v = (v * gr_complex(0.5f, 0.25f)) * gr_complex(-1.0f, 2.0f);
    EXPECT_TRUE(first == x);
}

TEST(HipDomain, ChannelizerC4)
{
    const size_t frames = 512, n = frames * 1024;
    std::vector<gr_complex> w(1024);
    for (int b = 0; b < 1024; ++b) w[b] = gr_complex((1.0f + 0.5f * std::cos(2 * (float)M_PI * b / 1024)) / 1024.0f, 0);
    auto x = synth(n);
    // reference: direct DFT per frame in double (spot-check 8 frames), plus round trip
    auto src = hip::synth_source::make(0, n, 0x6E736368, 1024);
    auto ch = hip::channelizer_vcc::make(w);
    auto snk = blocks::vector_sink_c::make(1024, frames);
    auto fg = flowgraph::make();
    fg->connect(src, 0, ch, 0);
    fg->connect(ch, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->set_scheduler(schedulers::scheduler_hip::make("hip", 0, 1u << 20));
    fg->validate();
    fg->run();
    const auto y = snk->data();
    ASSERT_TRUE(y.size() == n);
    std::vector<gr_complex> yr, got;
    for (size_t f : { (size_t)0, (size_t)1, (size_t)77, (size_t)511 }) {
        std::vector<std::complex<double>> X(1024), t(1024);
        for (int k = 0; k < 1024; ++k) {
            std::complex<double> s = 0;
            for (int m = 0; m < 1024; ++m) s += std::complex<double>(x[f * 1024 + m]) * std::polar(1.0, -2 * M_PI * k * m / 1024);
            X[k] = s * std::complex<double>(w[k]);
        }
        for (int m = 0; m < 1024; ++m) {
            std::complex<double> s = 0;
            for (int k = 0; k < 1024; ++k) s += X[k] * std::polar(1.0, 2 * M_PI * k * m / 1024);
            yr.push_back(gr_complex(s));
            got.push_back(y[f * 1024 + m]);
        }
    }
    EXPECT_TRUE(close_normwise(got, yr));
}

// C4 as separate blocks: fft_vcc -> multiply_const_vcc(w) -> fft_vcc(inverse). scheduler_hip
// fuses the three into one channelizer launch; fused, unfused (three kernels, two interior
// HBM edges) and the channelizer_vcc block must agree bit for bit.
TEST(HipDomain, ChannelizerFromBlocksFused)
{
    const size_t frames = 300, n = frames * 1024;
    std::vector<gr_complex> w(1024);
    for (int b = 0; b < 1024; ++b) w[b] = gr_complex((1.0f + 0.5f * std::cos(2 * (float)M_PI * b / 1024)) / 1024.0f, 0.25f / (1 + b));
    auto run = [&](int how) { // 0: blocks fused, 1: blocks unfused, 2: channelizer_vcc
        auto src = hip::synth_source::make(0, n, 0x6E736368, 1024);
        auto snk = blocks::vector_sink_c::make(1024, frames);
        auto fg = flowgraph::make();
        if (how == 2) {
            auto ch = hip::channelizer_vcc::make(w);
            fg->connect(src, 0, ch, 0);
            fg->connect(ch, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        } else {
            auto f1 = hip::fft_vcc::make(1024, true);
            auto m = hip::multiply_const_vcc::make(w);
            auto f2 = hip::fft_vcc::make(1024, false);
            fg->connect(src, 0, f1, 0);
            fg->connect(f1, 0, m, 0);
            fg->connect(m, 0, f2, 0);
            fg->connect(f2, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        }
        auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 20);
        sched->set_fusion(how != 1);
        fg->set_scheduler(sched);
        fg->validate();
        const size_t nfused = sched->fusion_plan().fused.size();
        EXPECT_TRUE(nfused == (how == 0 ? 1u : 0u));
        fg->run();
        return snk->data();
    };
    const auto yf = run(0), yu = run(1), yc = run(2);
    ASSERT_TRUE(yf.size() == n && yu.size() == n && yc.size() == n);
    EXPECT_TRUE(yf == yu);
    EXPECT_TRUE(yf == yc);
}

TEST(HipDomain, DecimatingChainC5)
{
    // 4 x fir(127, 2): staged (FIR fusion off) and fused by scheduler_hip into one
    // fir_filter_cascade_ccf (default), both against the in-test chain; 512 KiB buffers make
    // many work() calls (history hand-off), the fused graph runs twice (restart), and a ragged
    // length leaves a partial last output group unconsumed in both forms.
    const auto h = lowpass(127, 0.225);
    for (size_t n : { size_t(1) << 20, (size_t(1) << 20) + 37 }) {
        auto ref = synth(n - n % 16);
        for (int i = 0; i < 4; ++i) ref = fir_ref(ref, h, 2);
        for (int fused = 0; fused < 2; ++fused) {
            auto src = hip::synth_source::make(0, n);
            std::vector<hip::fir_filter_ccf::sptr> st;
            for (int i = 0; i < 4; ++i) st.push_back(hip::fir_filter_ccf::make(h, 2));
            auto snk = blocks::vector_sink_c::make(1, n / 16);
            auto fg = flowgraph::make();
            fg->connect(src, 0, st[0], 0);
            for (int i = 1; i < 4; ++i) fg->connect(st[i - 1], 0, st[i], 0);
            fg->connect(st[3], 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
            auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 19);
            sched->set_fir_fusion(fused == 1);
            fg->set_scheduler(sched);
            fg->validate();
            EXPECT_TRUE(sched->fusion_plan().fused.size() == (fused ? 1u : 0u));
            for (int run = 0; run < 1 + fused; ++run) {
                fg->run();
                ASSERT_TRUE(snk->data().size() == ref.size());
                const bool ok = close_normwise(snk->data(), ref);
                if (!ok) {
                    const auto y = snk->data();
                    size_t first = 0;
                    while (first < y.size() && std::abs(y[first] - ref[first]) <= 1e-5f * 0.6f) ++first;
                    std::fprintf(stderr, "  n=%zu fused=%d run=%d first bad output %zu of %zu\n", n, fused, run, first, y.size());
                }
                EXPECT_TRUE(ok);
            }
            if (fused) {
                auto c = std::dynamic_pointer_cast<hip::fir_filter_cascade_ccf>(sched->fusion_plan().fused[0]);
                ASSERT_TRUE(c != nullptr);
                EXPECT_TRUE(c->kernel() == "k_fir_pfft2<16>");
                EXPECT_TRUE(c->launches() > 4u);
                EXPECT_TRUE(st[0]->launches() == 0u); // the staged blocks were replaced
            }
        }
    }
}

// Kernel timing through the polyphase-FFT kernel: its launch must record the event
// pair the block arms (nsh::launch), so kernel_ms() reads recorded events -- for the fused C5
// cascade and for a single decim-16 fir_filter_ccf, which AUTO resolves to k_fir_pfft. Both are
// parity-checked on the same run.
TEST(HipDomain, TimedPfftLaunches)
{
    const size_t n = size_t(1) << 20;
    const auto h = lowpass(127, 0.225);
    {
        auto ref = synth(n);
        for (int i = 0; i < 4; ++i) ref = fir_ref(ref, h, 2);
        auto src = hip::synth_source::make(0, n);
        std::vector<hip::fir_filter_ccf::sptr> st;
        for (int i = 0; i < 4; ++i) st.push_back(hip::fir_filter_ccf::make(h, 2));
        auto snk = blocks::vector_sink_c::make(1, n / 16);
        auto fg = flowgraph::make();
        fg->connect(src, 0, st[0], 0);
        for (int i = 1; i < 4; ++i) fg->connect(st[i - 1], 0, st[i], 0);
        fg->connect(st[3], 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 19);
        fg->set_scheduler(sched);
        fg->validate();
        ASSERT_TRUE(sched->fusion_plan().fused.size() == 1u);
        auto c = std::dynamic_pointer_cast<hip::fir_filter_cascade_ccf>(sched->fusion_plan().fused[0]);
        ASSERT_TRUE(c != nullptr);
        c->enable_timing(true);
        fg->run();
        EXPECT_TRUE(close_normwise(snk->data(), ref));
        const double ms = c->kernel_ms(); // throws if any armed pair went unrecorded
        std::printf("  cascade: %llu launches, %.3f ms\n", (unsigned long long)c->launches(), ms);
        EXPECT_TRUE(ms > 0.0);
    }
    {
        const auto h16 = lowpass(127, 0.03);
        const auto ref = fir_ref(synth(n), h16, 16);
        auto src = hip::synth_source::make(0, n);
        auto fir = hip::fir_filter_ccf::make(h16, 16);
        auto snk = blocks::vector_sink_c::make(1, n / 16);
        auto fg = flowgraph::make();
        fg->connect(src, 0, fir, 0);
        fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto sched = schedulers::scheduler_hip::make("hip", 0, 1u << 19);
        fg->set_scheduler(sched);
        fg->validate();
        fir->enable_timing(true);
        fg->run();
        EXPECT_TRUE(fir->kernel() == "k_fir_pfft2<16>");
        EXPECT_TRUE(close_normwise(snk->data(), ref));
        const double ms = fir->kernel_ms();
        std::printf("  decim-16 fir: %llu timed launches, %.3f ms\n", (unsigned long long)fir->timed_launches(), ms);
        EXPECT_TRUE(fir->timed_launches() > 0 && ms > 0.0);
    }
}

TEST(HipDomain, CrossThreadDeviceEdges)
{
    // hip blocks on separate scheduler_mt threads: each thread has its own stream, so
    // every D2D edge is ordered by events (post_write record / read_info wait).
    const size_t n = 5000001;
    const auto h = lowpass(61, 0.3);
    auto src = hip::synth_source::make(0, n);
    auto m1 = hip::multiply_const_cc::make(gr_complex(0.75f, 0.5f));
    auto fir = hip::fir_filter_ccf::make(h);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, m1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(m1, 0, fir, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 1u << 20));
    fg->validate();
    fg->run();
    auto x = synth(n);
    for (auto& v : x) v = cmul(v, gr_complex(0.75f, 0.5f));
    EXPECT_TRUE(close_normwise(snk->data(), fir_ref(x, h, 1)));
}

TEST(HipDomain, HostToDeviceToHostAcrossDomains)
{
    // CPU domain (sources/sinks) + GPU domain (kernels), joined by adapters whose edge
    // buffers are H2D / D2H hip_buffers.
    const size_t n = 300000;
    auto x = synth(n, 12345);
    auto src = blocks::vector_source_c::make(x);
    auto m = hip::multiply_const_cc::make(gr_complex(-0.5f, 2.0f));
    auto a = hip::add_cc::make(1);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, m, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(m, 0, a, 0);
    fg->connect(a, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto cpu = schedulers::scheduler_mt::make("cpu", 1u << 16);
    auto gpu = schedulers::scheduler_hip::make("gpu", 0, 1u << 16);
    fg->add_scheduler(cpu);
    fg->add_scheduler(gpu);
    auto da = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
    domain_conf_vec dc{ domain_conf(cpu, { src, snk }, da), domain_conf(gpu, { m, a }, da) };
    fg->partition(dc);
    fg->run();
    for (auto& v : x) v = cmul(v, gr_complex(-0.5f, 2.0f));
    EXPECT_TRUE(snk->data() == x);
}
