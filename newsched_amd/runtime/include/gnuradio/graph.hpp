// A set of nodes joined by edges (reference runtime/include/gnuradio/graph.hpp,
// runtime/lib/graph.cpp). connect() also tells both ports about each other so work()
// notifications reach the neighbour's thread.
#pragma once
#include <gnuradio/edge.hpp>
#include <stdexcept>

namespace gr {

class graph : public node, public std::enable_shared_from_this<graph>
{
public:
    using sptr = std::shared_ptr<graph>;
    static sptr make() { return std::make_shared<graph>(); }
    graph() : node() {}
    ~graph() override = default;
    std::shared_ptr<graph> base() { return shared_from_this(); }

    edge_vector_t& edges() { return _edges; }
    node_vector_t& orphan_nodes() { return _orphan_nodes; }

    edge_sptr connect(const node_endpoint& src, const node_endpoint& dst);
    edge_sptr connect(node_sptr src, unsigned int src_port, node_sptr dst, unsigned int dst_port);
    edge_sptr connect(node_sptr src, const std::string& src_port, node_sptr dst, const std::string& dst_port);
    void disconnect(const node_endpoint&, const node_endpoint&) {}
    virtual void validate() {}
    virtual void clear() {}
    void add_orphan_node(node_sptr n) { _orphan_nodes.push_back(std::move(n)); }

    // Nodes in order of first appearance in the edge list, then orphans (deterministic;
    // the reference sorts shared_ptrs by address, Appendix A).
    node_vector_t calc_used_nodes();
    edge_vector_t find_edge(port_sptr port);

protected:
    node_vector_t _nodes;
    edge_vector_t _edges;
    node_vector_t _orphan_nodes;
};

using graph_sptr = graph::sptr;

} // namespace gr
