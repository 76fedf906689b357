// Flattened graph of blocks (reference runtime/include/gnuradio/flat_graph.hpp:64-79,
// runtime/lib/flat_graph.cpp). topological_sort() is public and used: the GPU domain
// runs its blocks producer-first so one pass of its thread moves data end to end (the
// reference executor runs blocks in group order, graph_executor.cpp:17).
#pragma once
#include <gnuradio/block.hpp>
#include <gnuradio/graph.hpp>

namespace gr {

class block_endpoint : public node_endpoint
{
public:
    block_endpoint(block_sptr b, port_sptr p) : node_endpoint(b, p) {}
    block_endpoint(const node_endpoint& n) : node_endpoint(n) {}
    block_sptr block() const { return std::dynamic_pointer_cast<gr::block>(node()); }
};

class flat_graph : public graph
{
public:
    using sptr = std::shared_ptr<flat_graph>;
    flat_graph() = default;
    ~flat_graph() override = default;

    block_vector_t calc_used_blocks();
    static std::shared_ptr<flat_graph> make_flat(graph_sptr g);

    // Blocks ordered so that every edge goes from an earlier to a later block (Kahn);
    // blocks on cycles, if any, keep their relative order at the end.
    block_vector_t topological_sort(const block_vector_t& blocks);
    block_vector_t calc_downstream_blocks(block_sptr b);
    block_vector_t calc_upstream_blocks(block_sptr b);
};

using flat_graph_sptr = flat_graph::sptr;

} // namespace gr
