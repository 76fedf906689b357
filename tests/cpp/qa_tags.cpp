// Stream tags through the scheduler (reference schedulers/mt/test/qa_tags.cpp:21-220,
// restated with the same flowgraphs and expected tag counts; its t5 is disabled there), plus
// the same propagation across device edges: H2D / D2D / D2H hip_buffers and gr::hip blocks
// keep _total_read/_total_written exact, so tag offsets survive the GPU domain.
#include "qa.hpp"

#include <gnuradio/blocklib/blocks/annotator.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
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
