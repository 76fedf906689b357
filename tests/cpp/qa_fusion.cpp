// The scheduler_hip elementwise-fusion pass (gnuradio/hip_fusion.hpp) as host logic: which
// chains it finds, how it splits them, and how it rewires the graph and ports. No device is
// touched (block constructors and the pass are host-only), so this runs in the CPU suite;
// the fused flowgraphs' results are checked on the GPU in qa_hip_flowgraph.cpp.
#include "qa.hpp"

#include <algorithm>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/arith.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/fir_filter_cascade_ccf.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_fusion.hpp>

using namespace gr;
using hip::multiply_const_cc;

static gr_complex K(int i) { return gr_complex(1.0f + 0.25f * (float)i, -0.5f * (float)i); }

static flat_graph_sptr flat(const flowgraph::sptr& fg) { return flat_graph::make_flat(fg); }

static bool connected(const port_sptr& a, const port_sptr& b)
{
    auto v = a->connected_ports();
    return std::find(v.begin(), v.end(), b) != v.end();
}

static std::vector<gr_complex> fused_ks(const block_sptr& b)
{
    return std::dynamic_pointer_cast<hip::multiply_const_chain_cc>(b)->ks();
}

// src -> m0 -> m1 -> copy -> m2 -[D2H]-> sink: one chain of four blocks, three stages
TEST(Fusion, LinearChainRewired)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(16));
    auto m0 = multiply_const_cc::make(K(0));
    auto m1 = multiply_const_cc::make(K(1));
    auto cp = hip::copy::make(1);
    auto m2 = multiply_const_cc::make(K(2));
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, m0, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(m0, 0, m1, 0);
    fg->connect(m1, 0, cp, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(cp, 0, m2, 0);
    fg->connect(m2, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    // an in-process domain crossing keeps the original port pair linked outside the
    // partition graph: that link must move to the fused block too
    auto remote = blocks::null_sink::make(sizeof(gr_complex));
    auto xin = remote->input_stream_ports()[0];
    m2->output_stream_ports()[0]->connect(xin);
    xin->connect(m2->output_stream_ports()[0]);
    auto r = hip::fuse_elementwise_cc(flat(fg));
    ASSERT_TRUE(r.fused.size() == 1u);
    EXPECT_TRUE(r.chains[0].size() == 4u);
    EXPECT_TRUE(connected(xin, r.fused[0]->output_stream_ports()[0]));
    EXPECT_TRUE(connected(r.fused[0]->output_stream_ports()[0], xin));
    EXPECT_FALSE(connected(xin, m2->output_stream_ports()[0]));
    EXPECT_TRUE((fused_ks(r.fused[0]) == std::vector<gr_complex>{ K(0), K(1), K(2) }));
    auto& e = r.graph->edges();
    ASSERT_TRUE(e.size() == 2u);
    auto f = r.fused[0];
    auto fin = f->input_stream_ports()[0], fout = f->output_stream_ports()[0];
    auto sout = src->output_stream_ports()[0], kin = snk->input_stream_ports()[0];
    EXPECT_TRUE(e[0]->src().node() == src && e[0]->dst().port() == fin);
    EXPECT_TRUE(e[1]->src().port() == fout && e[1]->dst().node() == snk);
    // custom buffers of the boundary edges carried over
    auto p0 = std::dynamic_pointer_cast<hip_buffer_properties>(e[0]->buf_properties());
    auto p1 = std::dynamic_pointer_cast<hip_buffer_properties>(e[1]->buf_properties());
    EXPECT_TRUE(p0 && p0->buffer_type() == hip_buffer_type::H2D);
    EXPECT_TRUE(p1 && p1->buffer_type() == hip_buffer_type::D2H);
    // port notifications now go to the fused block, and the chain is detached
    EXPECT_TRUE(connected(sout, fin) && connected(fin, sout));
    EXPECT_TRUE(connected(kin, fout) && connected(fout, kin));
    EXPECT_FALSE(connected(sout, m0->input_stream_ports()[0]));
    EXPECT_TRUE(m1->output_stream_ports()[0]->connected_ports().empty());
    auto blocks = r.graph->calc_used_blocks();
    EXPECT_TRUE(blocks.size() == 3u);
}

// Fan-out ends a chain: m0 -> {m1, m2}; m1 -> m3 -> sink0; m2 -> sink1
TEST(Fusion, FanOutIsABoundary)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(16));
    std::vector<multiply_const_cc::sptr> m;
    for (int i = 0; i < 4; ++i) m.push_back(multiply_const_cc::make(K(i)));
    auto s0 = blocks::null_sink::make(sizeof(gr_complex));
    auto s1 = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, m[0], 0);
    fg->connect(m[0], 0, m[1], 0);
    fg->connect(m[0], 0, m[2], 0);
    fg->connect(m[1], 0, m[3], 0);
    fg->connect(m[3], 0, s0, 0);
    fg->connect(m[2], 0, s1, 0);
    auto r = hip::fuse_elementwise_cc(flat(fg));
    ASSERT_TRUE(r.fused.size() == 1u);
    EXPECT_TRUE(r.chains[0].size() == 2u && r.chains[0][0] == m[1] && r.chains[0][1] == m[3]);
    EXPECT_TRUE((fused_ks(r.fused[0]) == std::vector<gr_complex>{ K(1), K(3) }));
    EXPECT_TRUE(r.graph->edges().size() == 5u); // src->m0, m0->F, m0->m2, F->s0, m2->s1
    EXPECT_TRUE(connected(m[0]->output_stream_ports()[0], r.fused[0]->input_stream_ports()[0]));
    EXPECT_TRUE(connected(m[0]->output_stream_ports()[0], m[2]->input_stream_ports()[0]));
}

// Host-visible interior edges, float blocks, non-elementwise blocks and mixed tag policies
// are boundaries.
TEST(Fusion, Boundaries)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(16));
    auto a = multiply_const_cc::make(K(0));
    auto b = multiply_const_cc::make(K(1)); // a -[D2H]-> b: not fused
    auto c = multiply_const_cc::make(K(2));
    auto add = hip::add_cc::make(1);       // not elementwise_cc
    auto d = multiply_const_cc::make(K(3));
    auto e = multiply_const_cc::make(K(4)); // other tag policy
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    e->set_tag_propagation_policy(tag_propagation_policy_t::TPP_DONT);
    auto fg = flowgraph::make();
    fg->connect(src, 0, a, 0);
    fg->connect(a, 0, b, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->connect(b, 0, c, 0); // b, c fuse
    fg->connect(c, 0, add, 0);
    fg->connect(add, 0, d, 0);
    fg->connect(d, 0, e, 0);
    fg->connect(e, 0, snk, 0);
    auto r = hip::fuse_elementwise_cc(flat(fg));
    ASSERT_TRUE(r.fused.size() == 1u);
    EXPECT_TRUE(r.chains[0].size() == 2u && r.chains[0][0] == b && r.chains[0][1] == c);

    auto fsrc = blocks::vector_source_f::make(std::vector<float>(16));
    auto f1 = hip::multiply_const_ff::make(2.0f);
    auto f2 = hip::multiply_const_ff::make(3.0f);
    auto fsnk = blocks::null_sink::make(sizeof(float));
    auto fg2 = flowgraph::make();
    fg2->connect(fsrc, 0, f1, 0);
    fg2->connect(f1, 0, f2, 0);
    fg2->connect(f2, 0, fsnk, 0);
    auto r2 = hip::fuse_elementwise_cc(flat(fg2));
    EXPECT_TRUE(r2.fused.empty());
    EXPECT_TRUE(r2.graph->edges().size() == 3u);
}

// Long chains are cut at the fused kernel's 16-stage limit (the reference's
// BasicBlockGrouping builds chains of up to 128 multiply_const blocks).
TEST(Fusion, LongChainsSplitAtStageLimit)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(16));
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    // a 10-stage hand-fused block, then 30 single stages with a copy in the middle
    std::vector<gr_complex> ten;
    for (int i = 0; i < 10; ++i) ten.push_back(K(i));
    block_sptr prev = hip::multiply_const_chain_cc::make(ten);
    fg->connect(src, 0, prev, 0);
    for (int i = 0; i < 31; ++i) {
        block_sptr nb = i == 15 ? block_sptr(hip::copy::make(1)) : block_sptr(multiply_const_cc::make(K(i)));
        fg->connect(prev, 0, nb, 0);
        prev = nb;
    }
    fg->connect(prev, 0, snk, 0);
    auto r = hip::fuse_elementwise_cc(flat(fg));
    // stages: 10 + 30 = 40 -> 16 (chain10 + 6), 16 (9 singles, the copy, 6 singles... ), rest
    size_t total = 0, blocks_total = 0;
    for (size_t i = 0; i < r.fused.size(); ++i) {
        EXPECT_TRUE(fused_ks(r.fused[i]).size() <= hip::max_fused_stages);
        total += fused_ks(r.fused[i]).size();
        blocks_total += r.chains[i].size();
    }
    EXPECT_TRUE(total == 40u);
    EXPECT_TRUE(blocks_total == 32u);
    EXPECT_TRUE(r.fused.size() == 3u);
    EXPECT_TRUE(fused_ks(r.fused[0]).size() == 16u && r.chains[0].size() == 7u);
    // the fused blocks form one path src -> F0 -> F1 -> F2 -> snk
    EXPECT_TRUE(r.graph->edges().size() == 4u);
    EXPECT_TRUE(r.graph->calc_used_blocks().size() == 5u);
}

static std::vector<gr_complex> W1024()
{
    std::vector<gr_complex> w(1024);
    for (int b = 0; b < 1024; ++b) w[b] = gr_complex(1.0f / (1 + b), 0.5f);
    return w;
}

// src -[H2D]-> fft -> w -> ifft -[D2H]-> sink becomes src -> channelizer(w) -> sink
TEST(Fusion, ChannelizerFromBlocks)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(2048), false, 1024);
    auto f1 = hip::fft_vcc::make(1024, true);
    auto m = hip::multiply_const_vcc::make(W1024());
    auto f2 = hip::fft_vcc::make(1024, false);
    auto snk = blocks::null_sink::make(1024 * sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, f1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(f1, 0, m, 0);
    fg->connect(m, 0, f2, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2D);
    fg->connect(f2, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto r = hip::fuse_channelizer(flat(fg));
    ASSERT_TRUE(r.fused.size() == 1u);
    auto c = std::dynamic_pointer_cast<hip::channelizer_vcc>(r.fused[0]);
    ASSERT_TRUE(c != nullptr);
    EXPECT_TRUE(c->w() == W1024());
    EXPECT_TRUE(r.chains[0].size() == 3u && r.chains[0][0] == f1 && r.chains[0][2] == f2);
    auto& e = r.graph->edges();
    ASSERT_TRUE(e.size() == 2u);
    EXPECT_TRUE(e[0]->src().node() == src && e[0]->dst().port() == c->input_stream_ports()[0]);
    EXPECT_TRUE(e[1]->src().port() == c->output_stream_ports()[0] && e[1]->dst().node() == snk);
    auto p0 = std::dynamic_pointer_cast<hip_buffer_properties>(e[0]->buf_properties());
    auto p1 = std::dynamic_pointer_cast<hip_buffer_properties>(e[1]->buf_properties());
    EXPECT_TRUE(p0 && p0->buffer_type() == hip_buffer_type::H2D);
    EXPECT_TRUE(p1 && p1->buffer_type() == hip_buffer_type::D2H);
    EXPECT_TRUE(connected(src->output_stream_ports()[0], c->input_stream_ports()[0]));
    EXPECT_TRUE(connected(snk->input_stream_ports()[0], c->output_stream_ports()[0]));
    EXPECT_TRUE(r.graph->calc_used_blocks().size() == 3u);
}

// Not the pattern: two forward transforms, a host-visible interior edge, a fan-out of the
// spectrum, an ifft first.
TEST(Fusion, ChannelizerBoundaries)
{
    auto run = [](int variant) {
        auto src = blocks::vector_source_c::make(std::vector<gr_complex>(2048), false, 1024);
        auto f1 = hip::fft_vcc::make(1024, variant != 3);
        auto m = hip::multiply_const_vcc::make(W1024());
        auto f2 = hip::fft_vcc::make(1024, variant == 0);
        auto snk = blocks::null_sink::make(1024 * sizeof(gr_complex));
        auto fg = flowgraph::make();
        fg->connect(src, 0, f1, 0);
        auto e1 = fg->connect(f1, 0, m, 0);
        if (variant == 1) e1->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        fg->connect(m, 0, f2, 0);
        fg->connect(f2, 0, snk, 0);
        if (variant == 2) fg->connect(f1, 0, blocks::null_sink::make(1024 * sizeof(gr_complex)), 0);
        return hip::fuse_channelizer(flat(fg)).fused.size();
    };
    EXPECT_TRUE(run(0) == 0u); // fft -> w -> fft (both forward)
    EXPECT_TRUE(run(1) == 0u); // spectrum crosses to the host
    EXPECT_TRUE(run(2) == 0u); // spectrum fans out
    EXPECT_TRUE(run(3) == 0u); // ifft -> w -> fft
}

// fusion_result::undo() (scheduler_hip::release_fused) gives the user's blocks their original
// port links back, so the same flowgraph can be initialized (and fused) again.
TEST(Fusion, UndoRestoresPortLinks)
{
    auto src = blocks::vector_source_c::make(std::vector<gr_complex>(16));
    auto m0 = multiply_const_cc::make(K(0));
    auto m1 = multiply_const_cc::make(K(1));
    auto m2 = multiply_const_cc::make(K(2));
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, m0, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(m0, 0, m1, 0);
    fg->connect(m1, 0, m2, 0);
    fg->connect(m2, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto remote = blocks::null_sink::make(sizeof(gr_complex)); // a crossing's extra link
    auto xin = remote->input_stream_ports()[0];
    m2->output_stream_ports()[0]->connect(xin);
    xin->connect(m2->output_stream_ports()[0]);
    const std::vector<block_sptr> blks{ src, m0, m1, m2, snk, remote };
    auto snapshot = [&] {
        std::vector<std::vector<port_sptr>> v;
        for (auto& b : blks)
            for (auto& p : b->all_ports()) {
                auto c = p->connected_ports(); // as a set: restored links may come back in another order
                std::sort(c.begin(), c.end());
                v.push_back(c);
            }
        return v;
    };
    const auto before = snapshot();
    for (int round = 0; round < 2; ++round) {
        auto r = hip::fuse_elementwise_cc(flat(fg));
        ASSERT_TRUE(r.fused.size() == 1u);
        EXPECT_TRUE(connected(xin, r.fused[0]->output_stream_ports()[0]));
        EXPECT_FALSE(connected(m0->output_stream_ports()[0], m1->input_stream_ports()[0]));
        r.undo();
        EXPECT_TRUE(snapshot() == before);
        EXPECT_FALSE(connected(xin, r.fused[0]->output_stream_ports()[0]));
    }
}

// ---- FIR-chain pass (hip::fuse_fir_cascade) ------------------------------------------------
static std::vector<float> lp(int n)
{
    std::vector<float> h((size_t)n);
    for (int i = 0; i < n; ++i) h[(size_t)i] = 1.0f / (float)(n + i); // any finite taps
    return h;
}
static std::shared_ptr<hip::fir_filter_cascade_ccf> as_casc(const block_sptr& b)
{
    return std::dynamic_pointer_cast<hip::fir_filter_cascade_ccf>(b);
}

// BASELINE C5: src -> 4 x fir(127, 2) -> sink becomes one cascade (D = 16); a fifth stage is left
TEST(Fusion, FirChainC5)
{
    for (int nst : { 4, 5 }) {
        auto src = blocks::vector_source_c::make(std::vector<gr_complex>(64));
        auto snk = blocks::null_sink::make(sizeof(gr_complex));
        auto fg = flowgraph::make();
        std::vector<block_sptr> firs;
        for (int i = 0; i < nst; ++i) firs.push_back(hip::fir_filter_ccf::make(lp(127), 2));
        fg->connect(src, 0, firs[0], 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
        for (int i = 0; i + 1 < nst; ++i) fg->connect(firs[(size_t)i], 0, firs[(size_t)i + 1], 0);
        fg->connect(firs.back(), 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto r = hip::fuse_fir_cascade(flat(fg));
        ASSERT_TRUE(r.fused.size() == 1u);
        ASSERT_TRUE(r.chains[0].size() == 4u);
        auto c = as_casc(r.fused[0]);
        ASSERT_TRUE(c != nullptr);
        EXPECT_TRUE(c->decimation() == 16u);
        EXPECT_TRUE(c->stages().size() == 4u);
        EXPECT_TRUE(connected(src->output_stream_ports()[0], c->input_stream_ports()[0]));
        if (nst == 4)
            EXPECT_TRUE(connected(c->output_stream_ports()[0], snk->input_stream_ports()[0]));
        else // the fifth stage stays, fed by the cascade
            EXPECT_TRUE(connected(c->output_stream_ports()[0], firs[4]->input_stream_ports()[0]));
        EXPECT_TRUE(r.graph->calc_used_blocks().size() == (nst == 4 ? 3u : 4u));
        r.undo();
        EXPECT_TRUE(connected(firs[0]->output_stream_ports()[0], firs[1]->input_stream_ports()[0]));
    }
}

// runs with total decimation 8 or 16 only; a run that would exceed 16 ends where it still fits
TEST(Fusion, FirChainSegments)
{
    auto count = [](std::vector<int> decims, std::vector<int> ntaps) {
        auto src = blocks::vector_source_c::make(std::vector<gr_complex>(64));
        auto snk = blocks::null_sink::make(sizeof(gr_complex));
        auto fg = flowgraph::make();
        std::vector<block_sptr> firs;
        for (size_t i = 0; i < decims.size(); ++i) firs.push_back(hip::fir_filter_ccf::make(lp(ntaps[i]), decims[i]));
        fg->connect(src, 0, firs[0], 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
        for (size_t i = 0; i + 1 < firs.size(); ++i) fg->connect(firs[i], 0, firs[i + 1], 0);
        fg->connect(firs.back(), 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        auto r = hip::fuse_fir_cascade(flat(fg));
        std::vector<size_t> lens;
        for (auto& c : r.chains) lens.push_back(c.size());
        return lens;
    };
    EXPECT_TRUE(count({ 2, 2 }, { 31, 31 }) == std::vector<size_t>{});              // D = 4: no gain kept
    EXPECT_TRUE(count({ 2, 2, 2 }, { 31, 31, 31 }) == std::vector<size_t>{ 3 });    // D = 8
    EXPECT_TRUE(count({ 4, 4 }, { 63, 63 }) == std::vector<size_t>{ 2 });           // D = 16
    EXPECT_TRUE(count({ 2, 8, 2, 2, 2 }, { 31, 31, 31, 31, 31 }) == (std::vector<size_t>{ 2, 3 }));
    EXPECT_TRUE(count({ 1, 2, 2, 2 }, { 15, 31, 31, 31 }) == std::vector<size_t>{ 4 }); // decim-1 stage joins
    EXPECT_TRUE(count({ 2, 2, 2, 2 }, { 1200, 127, 127, 127 }).empty() == false);  // D = 8 prefix fits
    EXPECT_TRUE(count({ 8, 2 }, { 4200, 3 }).empty());                             // too long for 256 rows
}

TEST(Fusion, FirChainBoundaries)
{
    // 0: forced algorithm, 1: preloaded history, 2: fan-out after stage 2, 3: host edge in the middle
    auto run = [](int variant) {
        auto src = blocks::vector_source_c::make(std::vector<gr_complex>(64));
        auto snk = blocks::null_sink::make(sizeof(gr_complex));
        auto fg = flowgraph::make();
        std::vector<std::shared_ptr<hip::fir_filter_ccf>> firs;
        for (int i = 0; i < 4; ++i) firs.push_back(hip::fir_filter_ccf::make(lp(127), 2, variant == 0 && i == 2 ? 1 : 0));
        if (variant == 1) firs[1]->set_initial_history(std::vector<gr_complex>(126));
        fg->connect(src, 0, firs[0], 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
        for (int i = 0; i < 3; ++i) {
            auto e = fg->connect(firs[(size_t)i], 0, firs[(size_t)i + 1], 0);
            if (variant == 3 && i == 1) e->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        }
        if (variant == 2) fg->connect(firs[1], 0, blocks::null_sink::make(sizeof(gr_complex)), 0);
        fg->connect(firs.back(), 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
        return hip::fuse_fir_cascade(flat(fg)).fused.size();
    };
    for (int v = 0; v < 4; ++v) EXPECT_TRUE(run(v) == 0u);
}
