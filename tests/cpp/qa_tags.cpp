// Stream tags through the scheduler (reference schedulers/mt/test/qa_tags.cpp:21-220,
// restated with the same flowgraphs and expected tag counts; its t5 is disabled there), plus
// the same propagation across device edges: H2D / D2D / D2H hip_buffers and gr::hip blocks
// keep _total_read/_total_written exact, so tag offsets survive the GPU domain.
#include "qa.hpp"

#include <gnuradio/blocklib/blocks/annotator.hpp>
#include <gnuradio/blocklib/blocks/copy.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

using namespace gr;
using A = blocks::annotator;
constexpr auto ONE = tag_propagation_policy_t::TPP_ONE_TO_ONE;
constexpr auto ALL = tag_propagation_policy_t::TPP_ALL_TO_ALL;

TEST(SchedulerMTTags, OneToOne)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(int));
    auto head = blocks::head::make(sizeof(int), N);
    auto ann0 = A::make(10000, sizeof(int), 1, 2, ONE);
    auto ann1 = A::make(10000, sizeof(int), 1, 1, ONE);
    auto ann2 = A::make(10000, sizeof(int), 1, 1, ONE);
    auto snk0 = blocks::null_sink::make(sizeof(int));
    auto snk1 = blocks::null_sink::make(sizeof(int));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, ann1, 0);
    fg->connect(ann0, 1, ann2, 0);
    fg->connect(ann1, 0, snk0, 0);
    fg->connect(ann2, 0, snk1, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make());
    fg->validate();
    fg->start();
    fg->wait();
    EXPECT_EQ(ann0->data().size(), 0u);
    EXPECT_EQ(ann1->data().size(), 4u);
    EXPECT_EQ(ann2->data().size(), 4u);
}

TEST(SchedulerMTTags, t1)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(int));
    auto head = blocks::head::make(sizeof(int), N);
    auto ann0 = A::make(10000, sizeof(int), 1, 2, ALL);
    auto ann1 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann2 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann3 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann4 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto snk0 = blocks::null_sink::make(sizeof(int));
    auto snk1 = blocks::null_sink::make(sizeof(int));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, ann1, 0);
    fg->connect(ann0, 1, ann2, 0);
    fg->connect(ann1, 0, ann3, 0);
    fg->connect(ann2, 0, ann4, 0);
    fg->connect(ann3, 0, snk0, 0);
    fg->connect(ann4, 0, snk1, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make());
    fg->validate();
    fg->run();
    EXPECT_EQ(ann0->data().size(), 0u);
    EXPECT_EQ(ann3->data().size(), 8u);
    EXPECT_EQ(ann4->data().size(), 8u);
}

TEST(SchedulerMTTags, t2)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(int));
    auto head = blocks::head::make(sizeof(int), N);
    auto ann0 = A::make(10000, sizeof(int), 1, 2, ALL);
    auto ann1 = A::make(10000, sizeof(int), 2, 3, ALL);
    auto ann2 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann3 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann4 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto snk0 = blocks::null_sink::make(sizeof(int));
    auto snk1 = blocks::null_sink::make(sizeof(int));
    auto snk2 = blocks::null_sink::make(sizeof(int));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, ann1, 0);
    fg->connect(ann0, 1, ann1, 1);
    fg->connect(ann1, 0, ann2, 0);
    fg->connect(ann1, 1, ann3, 0);
    fg->connect(ann1, 2, ann4, 0);
    fg->connect(ann2, 0, snk0, 0);
    fg->connect(ann3, 0, snk1, 0);
    fg->connect(ann4, 0, snk2, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make());
    fg->validate();
    fg->run();
    EXPECT_EQ(ann0->data().size(), 0u);
    EXPECT_EQ(ann1->data().size(), 8u);
    EXPECT_EQ(ann2->data().size(), 12u);
    EXPECT_EQ(ann3->data().size(), 12u);
    EXPECT_EQ(ann4->data().size(), 12u);
}

TEST(SchedulerMTTags, t3)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(int));
    auto head = blocks::head::make(sizeof(int), N);
    auto ann0 = A::make(10000, sizeof(int), 2, 2, ONE);
    auto ann1 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann2 = A::make(10000, sizeof(int), 1, 1, ALL);
    auto ann3 = A::make(10000, sizeof(int), 1, 1, ONE);
    auto ann4 = A::make(10000, sizeof(int), 1, 1, ONE);
    auto snk0 = blocks::null_sink::make(sizeof(int));
    auto snk1 = blocks::null_sink::make(sizeof(int));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(head, 0, ann0, 1);
    fg->connect(ann0, 0, ann1, 0);
    fg->connect(ann0, 1, ann2, 0);
    fg->connect(ann1, 0, ann3, 0);
    fg->connect(ann2, 0, ann4, 0);
    fg->connect(ann3, 0, snk0, 0);
    fg->connect(ann4, 0, snk1, 0);
    auto sched = schedulers::scheduler_mt::make();
    sched->add_block_group({ src, head, ann0, ann1, ann2, ann3, ann4, snk0, snk1 });
    fg->set_scheduler(sched);
    fg->validate();
    fg->start();
    fg->wait();
    EXPECT_EQ(ann0->data().size(), 0u);
    EXPECT_EQ(ann3->data().size(), 8u);
    EXPECT_EQ(ann4->data().size(), 8u);
}

// Not in the reference (its domain adapters carry no tags): tags crossing in-process domain
// boundaries. src -> head -> ann0 | copy | ann1 -> sink in three scheduler_mt domains;
// the adapter pair's tag calls resolve to the shared edge buffer, so ann1 sees ann0's 4 tags
// at their absolute offsets.
TEST(SchedulerMTTags, AcrossDomains)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), N);
    auto ann0 = A::make(10000, sizeof(gr_complex), 1, 1, ALL);
    auto cp = blocks::copy::make(sizeof(gr_complex));
    auto ann1 = A::make(1u << 30, sizeof(gr_complex), 1, 1, ALL);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, cp, 0);
    fg->connect(cp, 0, ann1, 0);
    fg->connect(ann1, 0, snk, 0);
    auto a = schedulers::scheduler_mt::make("a", 32768);
    auto b = schedulers::scheduler_mt::make("b", 32768);
    auto a2 = schedulers::scheduler_mt::make("c", 32768);
    fg->add_scheduler(a);
    fg->add_scheduler(b);
    fg->add_scheduler(a2);
    auto da = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
    // crossings ann0 -> cp (the annotator writes into an adapter: offsets come from the
    // edge buffer's counters) and cp -> ann1
    domain_conf_vec dc{ domain_conf(a, { src, head, ann0 }, da), domain_conf(b, { cp }, da),
                        domain_conf(a2, { ann1, snk }, da) };
    fg->partition(dc);
    fg->run();
    auto seen = ann1->data();
    ASSERT_TRUE(seen.size() == 4u);
    for (size_t i = 0; i < 4; ++i) {
        EXPECT_EQ(seen[i].offset, (uint64_t)(10000 * i));
        EXPECT_TRUE(std::get<int64_t>(seen[i].value->value()) == (int64_t)i);
    }
}

// Device edges: annotator -[H2D]-> hip::copy -[D2D]-> hip::copy -[D2H]-> annotator. The
// second annotator must see the first one's 4 tags at their original absolute offsets.
TEST(DeviceTags, ThroughHipBlocks)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), N);
    auto ann0 = A::make(10000, sizeof(gr_complex), 1, 1, ALL);
    auto c1 = hip::copy::make(1);
    auto c2 = hip::copy::make(1);
    auto ann1 = A::make(1u << 30, sizeof(gr_complex), 1, 1, ALL);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, c1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(c1, 0, c2, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(c2, 0, ann1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->connect(ann1, 0, snk, 0);
    fg->set_scheduler(schedulers::scheduler_mt::make("mt", 32768));
    fg->validate();
    fg->run();
    auto seen = ann1->data();
    // ann1 tags offset 0 itself (when = 2^30), which it does not see on its input
    ASSERT_TRUE(seen.size() == 4u);
    for (size_t i = 0; i < seen.size(); ++i) {
        EXPECT_EQ(seen[i].offset, (uint64_t)(10000 * i));
        EXPECT_TRUE(std::get<int64_t>(seen[i].value->value()) == (int64_t)i);
    }
}

// The same through scheduler_hip with elementwise fusion: CPU domain (annotators) and a GPU
// domain where copy -> multiply_const(1) -> copy is fused into one block. Tags must keep
// their absolute offsets through the fused block.
TEST(DeviceTags, ThroughFusedChain)
{
    const int N = 40000;
    auto fg = flowgraph::make();
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), N);
    auto ann0 = A::make(10000, sizeof(gr_complex), 1, 1, ALL);
    auto c1 = hip::copy::make(1);
    auto m = hip::multiply_const_cc::make(gr_complex(1.0f, 0.0f));
    auto c2 = hip::copy::make(1);
    auto ann1 = A::make(1u << 30, sizeof(gr_complex), 1, 1, ALL);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, c1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(c1, 0, m, 0);
    fg->connect(m, 0, c2, 0);
    fg->connect(c2, 0, ann1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->connect(ann1, 0, snk, 0);
    auto cpu = schedulers::scheduler_mt::make("cpu", 32768);
    auto gpu = schedulers::scheduler_hip::make("gpu", 0, 1u << 16);
    fg->add_scheduler(cpu);
    fg->add_scheduler(gpu);
    auto da = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
    domain_conf_vec dc{ domain_conf(cpu, { src, head, ann0, ann1, snk }, da), domain_conf(gpu, { c1, m, c2 }, da) };
    fg->partition(dc);
    ASSERT_TRUE(gpu->fusion_plan().fused.size() == 1u);
    fg->run();
    auto seen = ann1->data();
    ASSERT_TRUE(seen.size() == 4u);
    for (size_t i = 0; i < seen.size(); ++i) {
        EXPECT_EQ(seen[i].offset, (uint64_t)(10000 * i));
        EXPECT_TRUE(std::get<int64_t>(seen[i].value->value()) == (int64_t)i);
    }
}
