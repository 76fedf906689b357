// Elementwise-chain fusion pass for scheduler_hip (see gnuradio/hip_fusion.hpp).
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

    // Rewrite. Every edge touching a chain member is interior to its chain (dropped), into a
    // chain head, or out of a chain tail; the latter two are re-made on the fused block
    // (both ends when one segment of a split chain feeds the next).
    std::map<block*, std::pair<size_t, block_sptr>> owner; // member -> (chain index, fused block)
    for (size_t i = 0; i < chains.size(); ++i) {
        auto& c = chains[i];
        std::vector<gr_complex> ks;
        for (auto& b : c) ks.insert(ks.end(), stages[b.get()].begin(), stages[b.get()].end());
        const size_t vlen = c.front()->input_stream_ports()[0]->itemsize() / sizeof(gr_complex);
        auto f = multiply_const_chain_cc::make(ks, vlen);
        f->set_tag_propagation_policy(c.front()->tag_propagation_policy());
        f->set_alias("fused(" + c.front()->alias() + ".." + c.back()->alias() + ")");
        for (auto& b : c) owner[b.get()] = { i, f };
        r.fused.push_back(f);
    }
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
        e->src().port()->disconnect(e->dst().port());
        e->dst().port()->disconnect(e->src().port());
        if (so != owner.end() && dn != owner.end() && so->second.first == dn->second.first) continue; // interior
        auto src = so == owner.end() ? e->src()
                                     : node_endpoint(so->second.second, so->second.second->output_stream_ports()[0]);
        auto dst = dn == owner.end() ? e->dst()
                                     : node_endpoint(dn->second.second, dn->second.second->input_stream_ports()[0]);
        auto ne = g->connect(src, dst);
        if (e->has_custom_buffer()) ne->set_custom_buffer(e->buffer_factory(), e->buf_properties());
    }
    // Links that are not edges of this partition (an in-process domain crossing keeps the
    // original cross-domain port pair connected for notifications) move to the fused block.
    auto move_links = [](const port_sptr& from, const port_sptr& to) {
        for (auto& peer : from->connected_ports()) {
            peer->disconnect(from);
            from->disconnect(peer);
            peer->connect(to);
            to->connect(peer);
        }
    };
    for (size_t i = 0; i < chains.size(); ++i) {
        move_links(chains[i].front()->input_stream_ports()[0], r.fused[i]->input_stream_ports()[0]);
        move_links(chains[i].back()->output_stream_ports()[0], r.fused[i]->output_stream_ports()[0]);
    }
    for (auto& o : fg->orphan_nodes()) g->add_orphan_node(o);
    for (auto& f : r.fused) {
        bool linked = false;
        for (auto& e : g->edges()) linked = linked || e->src().node() == f || e->dst().node() == f;
        if (!linked) g->add_orphan_node(f);
    }
    r.chains = std::move(chains);
    r.graph = g;
    return r;
}

} // namespace hip
} // namespace gr
