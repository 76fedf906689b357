// Elementwise-chain fusion pass for scheduler_hip (see gnuradio/hip_fusion.hpp).
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/fir_filter_cascade_ccf.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_fusion.hpp>

#include <map>
#include <set>

namespace gr {
namespace hip {

namespace {

struct link_info {
    edge_sptr in;                 // the single upstream edge of the block's input port
    std::vector<edge_sptr> outs;  // every edge leaving its output port
};

bool device_to_device(const edge_sptr& e)
{
    if (!e->has_custom_buffer()) return true; // scheduler_hip's default edge is a D2D hip_buffer
    auto p = std::dynamic_pointer_cast<hip_buffer_properties>(e->buf_properties());
    return p && p->buffer_type() == hip_buffer_type::D2D;
}

} // namespace

namespace {
// Replace each chain (a path of blocks joined by single edges) by one block with the head's
// input port and the tail's output port; shared by the passes.
flat_graph_sptr rewrite_chains(flat_graph_sptr fg, const std::vector<std::vector<block_sptr>>& chains,
                               const std::vector<block_sptr>& fused, fusion_result& r)
{
    auto cut = [&r](const port_sptr& a, const port_sptr& b) {
        a->disconnect(b);
        r.cut.emplace_back(a, b);
    };
    auto link = [&r](const port_sptr& a, const port_sptr& b) {
        a->connect(b);
        r.added.emplace_back(a, b);
    };
    auto as_block = [](const node_sptr& n) { return std::dynamic_pointer_cast<block>(n); };
    std::map<block*, std::pair<size_t, block_sptr>> owner;
    for (size_t i = 0; i < chains.size(); ++i)
        for (auto& b : chains[i]) owner[b.get()] = { i, fused[i] };
    auto g = std::make_shared<flat_graph>();
    for (auto& e : fg->edges()) {
        auto s = as_block(e->src().node());
        auto d = as_block(e->dst().node());
        auto so = s ? owner.find(s.get()) : owner.end();
        auto dn = d ? owner.find(d.get()) : owner.end();
        if (so == owner.end() && dn == owner.end()) {
            g->edges().push_back(e);
            continue;
        }
        cut(e->src().port(), e->dst().port());
        cut(e->dst().port(), e->src().port());
        if (so != owner.end() && dn != owner.end() && so->second.first == dn->second.first) continue; // interior
        auto src = so == owner.end() ? e->src()
                                     : node_endpoint(so->second.second, so->second.second->output_stream_ports()[0]);
        auto dst = dn == owner.end() ? e->dst()
                                     : node_endpoint(dn->second.second, dn->second.second->input_stream_ports()[0]);
        auto ne = g->connect(src, dst); // links src.port <-> dst.port
        r.added.emplace_back(src.port(), dst.port());
        r.added.emplace_back(dst.port(), src.port());
        if (e->has_custom_buffer()) ne->set_custom_buffer(e->buffer_factory(), e->buf_properties());
    }
    auto move_links = [&](const port_sptr& from, const port_sptr& to) {
        for (auto& peer : from->connected_ports()) {
            cut(peer, from);
            cut(from, peer);
            link(peer, to);
            link(to, peer);
        }
    };
    for (size_t i = 0; i < chains.size(); ++i) {
        move_links(chains[i].front()->input_stream_ports()[0], fused[i]->input_stream_ports()[0]);
        move_links(chains[i].back()->output_stream_ports()[0], fused[i]->output_stream_ports()[0]);
    }
    for (auto& o : fg->orphan_nodes()) g->add_orphan_node(o);
    for (auto& f : fused) {
        bool linked = false;
        for (auto& e : g->edges()) linked = linked || e->src().node() == f || e->dst().node() == f;
        if (!linked) g->add_orphan_node(f);
    }
    return g;
}
} // namespace

fusion_result fuse_elementwise_cc(flat_graph_sptr fg)
{
    fusion_result r;
    r.graph = fg;
    auto blocks = fg->calc_used_blocks();

    // Elementwise blocks with exactly one stream input and one stream output, and their stages.
    std::map<block*, std::vector<gr_complex>> stages;
    for (auto& b : blocks) {
        auto ew = std::dynamic_pointer_cast<elementwise_cc>(b);
        if (!ew || b->input_stream_ports().size() != 1 || b->output_stream_ports().size() != 1) continue;
        std::vector<gr_complex> ks;
        if (!ew->elementwise_stages(ks) || ks.size() > max_fused_stages) continue;
        stages[b.get()] = std::move(ks);
    }
    if (stages.size() < 2) return r;

    std::map<block*, link_info> links;
    for (auto& e : fg->edges()) {
        auto s = std::dynamic_pointer_cast<block>(e->src().node());
        auto d = std::dynamic_pointer_cast<block>(e->dst().node());
        if (s && stages.count(s.get())) links[s.get()].outs.push_back(e);
        if (d && stages.count(d.get())) links[d.get()].in = e;
    }
    auto as_block = [](const node_sptr& n) { return std::dynamic_pointer_cast<block>(n); };
    // the edge from b to the next chain member, if b's output may be fused forward
    auto next_link = [&](const block_sptr& b) -> edge_sptr {
        auto& l = links[b.get()];
        if (l.outs.size() != 1) return nullptr;
        auto e = l.outs[0];
        auto d = as_block(e->dst().node());
        if (!d || !stages.count(d.get()) || d == b || !device_to_device(e)) return nullptr;
        if (d->tag_propagation_policy() != b->tag_propagation_policy()) return nullptr;
        if (e->src().port()->itemsize() != e->dst().port()->itemsize()) return nullptr;
        return e;
    };

    // Chain heads: elementwise blocks whose input is not fused from an elementwise producer.
    std::set<block*> interior;
    for (auto& b : blocks) {
        if (!stages.count(b.get())) continue;
        if (auto e = next_link(b)) interior.insert(as_block(e->dst().node()).get());
    }
    std::vector<std::vector<block_sptr>> chains;
    for (auto& b : blocks) {
        if (!stages.count(b.get()) || interior.count(b.get())) continue;
        std::vector<block_sptr> chain{ b };
        std::set<block*> seen{ b.get() };
        for (auto e = next_link(b); e; e = next_link(chain.back())) {
            auto d = as_block(e->dst().node());
            if (!seen.insert(d.get()).second) break; // a cycle of elementwise blocks
            chain.push_back(d);
        }
        // split at the fused kernel's stage limit; a segment of one block gains nothing
        std::vector<block_sptr> seg;
        size_t m = 0;
        for (auto& c : chain) {
            const size_t k = stages[c.get()].size();
            if (m + k > max_fused_stages) {
                if (seg.size() >= 2) chains.push_back(seg);
                seg.clear();
                m = 0;
            }
            seg.push_back(c);
            m += k;
        }
        if (seg.size() >= 2) chains.push_back(seg);
    }
    if (chains.empty()) return r;

    for (size_t i = 0; i < chains.size(); ++i) {
        auto& c = chains[i];
        std::vector<gr_complex> ks;
        for (auto& b : c) ks.insert(ks.end(), stages[b.get()].begin(), stages[b.get()].end());
        const size_t vlen = c.front()->input_stream_ports()[0]->itemsize() / sizeof(gr_complex);
        auto f = multiply_const_chain_cc::make(ks, vlen);
        f->set_tag_propagation_policy(c.front()->tag_propagation_policy());
        f->set_alias("fused(" + c.front()->alias() + ".." + c.back()->alias() + ")");
        r.fused.push_back(f);
    }
    // Every edge touching a chain member is interior to its chain (dropped), into a chain
    // head, or out of a chain tail; the latter two are re-made on the fused block (both ends
    // when one segment of a split chain feeds the next). Links that are not edges of this
    // partition (an in-process domain crossing keeps the original cross-domain port pair
    // connected for notifications) move to the fused block.
    auto g = rewrite_chains(fg, chains, r.fused, r);
    r.chains = std::move(chains);
    r.graph = g;
    return r;
}


fusion_result fuse_channelizer(flat_graph_sptr fg)
{
    fusion_result r;
    r.graph = fg;
    auto as_block = [](const node_sptr& n) { return std::dynamic_pointer_cast<block>(n); };
    // the single out-edge of b's single output port, if it goes to a block, else null
    std::map<block*, std::vector<edge_sptr>> outs;
    std::map<block*, int> ins;
    for (auto& e : fg->edges()) {
        if (auto s = as_block(e->src().node())) outs[s.get()].push_back(e);
        if (auto d = as_block(e->dst().node())) ins[d.get()]++;
    }
    auto next = [&](const block_sptr& b) -> block_sptr {
        auto it = outs.find(b.get());
        if (it == outs.end() || it->second.size() != 1 || b->output_stream_ports().size() != 1) return nullptr;
        auto e = it->second[0];
        auto d = as_block(e->dst().node());
        if (!d || !device_to_device(e) || ins[d.get()] != 1 || d->input_stream_ports().size() != 1) return nullptr;
        if (d->tag_propagation_policy() != b->tag_propagation_policy()) return nullptr;
        return d;
    };
    std::set<block*> used;
    for (auto& b : fg->calc_used_blocks()) {
        auto f1 = std::dynamic_pointer_cast<fft_vcc>(b);
        if (!f1 || !f1->forward() || used.count(b.get())) continue;
        auto m = std::dynamic_pointer_cast<multiply_const_vcc>(next(b));
        if (!m || m->k().size() != 1024) continue;
        auto f2 = std::dynamic_pointer_cast<fft_vcc>(next(m));
        if (!f2 || f2->forward() || used.count(f2.get())) continue;
        auto c = channelizer_vcc::make(m->k());
        c->set_tag_propagation_policy(b->tag_propagation_policy());
        c->set_alias("fused(" + b->alias() + ".." + f2->alias() + ")");
        r.chains.push_back({ b, m, f2 });
        r.fused.push_back(c);
        used.insert(b.get());
        used.insert(m.get());
        used.insert(f2.get());
    }
    if (r.fused.empty()) return r;
    r.graph = rewrite_chains(fg, r.chains, r.fused, r);
    return r;
}

fusion_result fuse_fir_cascade(flat_graph_sptr fg)
{
    fusion_result r;
    r.graph = fg;
    auto as_block = [](const node_sptr& n) { return std::dynamic_pointer_cast<block>(n); };
    auto as_fir = [](const block_sptr& b) -> std::shared_ptr<fir_filter_ccf> {
        auto f = std::dynamic_pointer_cast<fir_filter_ccf>(b);
        // a forced algorithm or a preloaded history keeps the block as placed
        if (!f || f->requested_algo() != 0 || f->has_initial_history()) return nullptr;
        return f;
    };
    std::map<block*, std::vector<edge_sptr>> outs;
    std::map<block*, int> ins;
    for (auto& e : fg->edges()) {
        if (auto s = as_block(e->src().node())) outs[s.get()].push_back(e);
        if (auto d = as_block(e->dst().node())) ins[d.get()]++;
    }
    // the FIR that b's single output edge feeds, if that edge may be fused
    auto next = [&](const block_sptr& b) -> std::shared_ptr<fir_filter_ccf> {
        auto it = outs.find(b.get());
        if (it == outs.end() || it->second.size() != 1) return nullptr;
        auto e = it->second[0];
        auto d = as_fir(as_block(e->dst().node()));
        if (!d || d == b || !device_to_device(e) || ins[d.get()] != 1) return nullptr;
        if (d->tag_propagation_policy() != b->tag_propagation_policy()) return nullptr;
        return d;
    };
    std::set<block*> interior;
    for (auto& b : fg->calc_used_blocks())
        if (as_fir(b))
            if (auto d = next(b)) interior.insert(d.get());
    for (auto& b : fg->calc_used_blocks()) {
        auto head = as_fir(b);
        if (!head || interior.count(b.get())) continue;
        std::vector<std::shared_ptr<fir_filter_ccf>> chain{ head };
        std::set<block*> seen{ b.get() };
        for (auto d = next(head); d && seen.insert(d.get()).second; d = next(chain.back())) chain.push_back(d);
        // segments: from each position the longest run of >= 2 stages with total decimation 8 or
        // 16 that the cascade kernel supports
        for (size_t i = 0; i < chain.size();) {
            size_t best = 0;
            std::vector<fir_filter_cascade_ccf::stage> st, best_st;
            int64_t dec = 1;
            for (size_t k = i; k < chain.size(); ++k) {
                dec *= chain[k]->decimation();
                if (dec > 16) break;
                st.emplace_back(chain[k]->taps(), chain[k]->decimation());
                if (k > i && (dec == 8 || dec == 16) && fir_filter_cascade_ccf::supported(st)) {
                    best = k - i + 1;
                    best_st = st;
                }
            }
            if (!best) {
                ++i;
                continue;
            }
            auto f = fir_filter_cascade_ccf::make(best_st);
            f->set_tag_propagation_policy(chain[i]->tag_propagation_policy());
            f->set_alias("fused(" + chain[i]->alias() + ".." + chain[i + best - 1]->alias() + ")");
            r.chains.emplace_back(chain.begin() + i, chain.begin() + i + best);
            r.fused.push_back(f);
            i += best;
        }
    }
    if (r.fused.empty()) return r;
    r.graph = rewrite_chains(fg, r.chains, r.fused, r);
    return r;
}

} // namespace hip
} // namespace gr
