// graph / flat_graph (reference runtime/lib/graph.cpp, runtime/lib/flat_graph.cpp).
#include <gnuradio/flat_graph.hpp>
#include <gnuradio/graph.hpp>

#include <algorithm>
#include <map>
#include <set>

namespace gr {

edge_sptr graph::connect(const node_endpoint& src, const node_endpoint& dst)
{
    if (!src.node() || !src.port() || !dst.node() || !dst.port()) throw std::invalid_argument("connect: null endpoint");
    if (src.port()->itemsize() != dst.port()->itemsize() && src.port()->type() == port_type_t::STREAM)
        throw std::invalid_argument("connect: item size mismatch " + std::to_string(src.port()->itemsize()) +
                                    " != " + std::to_string(dst.port()->itemsize()));
    auto e = edge::make(src, dst);
    _edges.push_back(e);
    _nodes = calc_used_nodes();
    for (auto& n : _nodes) // alias = name + unique id (reference graph.cpp:29-31)
        if (n->alias().empty()) n->set_alias(n->name() + std::to_string(n->id()));
    src.port()->connect(dst.port());
    dst.port()->connect(src.port());
    return e;
}

edge_sptr graph::connect(node_sptr src, unsigned int sp, node_sptr dst, unsigned int dp)
{
    auto s = src->get_port(sp, port_type_t::STREAM, port_direction_t::OUTPUT);
    if (!s) throw std::invalid_argument("Source Port not found");
    auto d = dst->get_port(dp, port_type_t::STREAM, port_direction_t::INPUT);
    if (!d) throw std::invalid_argument("Destination port not found");
    return connect(node_endpoint(src, s), node_endpoint(dst, d));
}

edge_sptr graph::connect(node_sptr src, const std::string& sp, node_sptr dst, const std::string& dp)
{
    auto s = src->get_port(sp);
    if (!s) throw std::invalid_argument("Source Port not found");
    auto d = dst->get_port(dp);
    if (!d) throw std::invalid_argument("Destination port not found");
    return connect(node_endpoint(src, s), node_endpoint(dst, d));
}

node_vector_t graph::calc_used_nodes()
{
    node_vector_t r;
    std::set<node*> seen;
    auto add = [&](const node_sptr& n) {
        if (n && seen.insert(n.get()).second) r.push_back(n);
    };
    for (auto& e : _edges) {
        add(e->src().node());
        add(e->dst().node());
    }
    for (auto& n : _orphan_nodes) add(n);
    return r;
}

edge_vector_t graph::find_edge(port_sptr port)
{
    edge_vector_t r;
    for (auto& e : _edges)
        if (e->src().port() == port || e->dst().port() == port) r.push_back(e);
    return r;
}

block_vector_t flat_graph::calc_used_blocks()
{
    block_vector_t r;
    std::set<block*> seen;
    auto add = [&](const node_sptr& n) {
        auto b = std::dynamic_pointer_cast<block>(n);
        if (b && seen.insert(b.get()).second) r.push_back(b);
    };
    for (auto& e : _edges) {
        add(e->src().node());
        add(e->dst().node());
    }
    for (auto& n : _orphan_nodes) add(n);
    return r;
}

std::shared_ptr<flat_graph> flat_graph::make_flat(graph_sptr g)
{
    // The reference assumes an already-flat graph and copies edges + buffer choices
    // (flat_graph.hpp:64-79); so does this runtime (no hierarchical blocks).
    auto fg = std::make_shared<flat_graph>();
    for (auto& e : g->edges()) fg->connect(e->src(), e->dst())->set_custom_buffer(e->buffer_factory(), e->buf_properties());
    for (auto& o : g->orphan_nodes()) fg->add_orphan_node(o);
    return fg;
}

block_vector_t flat_graph::calc_downstream_blocks(block_sptr b)
{
    block_vector_t r;
    for (auto& e : _edges)
        if (e->src().node() == b) {
            auto d = std::dynamic_pointer_cast<block>(e->dst().node());
            if (d && std::find(r.begin(), r.end(), d) == r.end()) r.push_back(d);
        }
    return r;
}

block_vector_t flat_graph::calc_upstream_blocks(block_sptr b)
{
    block_vector_t r;
    for (auto& e : _edges)
        if (e->dst().node() == b) {
            auto s = std::dynamic_pointer_cast<block>(e->src().node());
            if (s && std::find(r.begin(), r.end(), s) == r.end()) r.push_back(s);
        }
    return r;
}

block_vector_t flat_graph::topological_sort(const block_vector_t& blocks)
{
    std::map<block*, int> indeg;
    for (auto& b : blocks) indeg[b.get()] = 0;
    for (auto& e : _edges) {
        auto s = std::dynamic_pointer_cast<block>(e->src().node());
        auto d = std::dynamic_pointer_cast<block>(e->dst().node());
        if (s && d && indeg.count(s.get()) && indeg.count(d.get())) indeg[d.get()]++;
    }
    block_vector_t order, pending(blocks);
    bool progress = true;
    while (!pending.empty() && progress) {
        progress = false;
        for (auto it = pending.begin(); it != pending.end();) {
            if (indeg[it->get()] == 0) {
                for (auto& d : calc_downstream_blocks(*it))
                    if (indeg.count(d.get())) indeg[d.get()]--;
                order.push_back(*it);
                it = pending.erase(it);
                progress = true;
            } else {
                ++it;
            }
        }
    }
    order.insert(order.end(), pending.begin(), pending.end()); // cycles, if any
    return order;
}

} // namespace gr
