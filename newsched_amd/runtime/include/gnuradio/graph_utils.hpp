// Split a flowgraph into per-domain subgraphs joined by domain-adapter pairs (reference
// runtime/include/gnuradio/graph_utils.hpp, runtime/lib/graph_utils.cpp:11-205).
#pragma once
#include <gnuradio/domain.hpp>
#include <gnuradio/graph.hpp>
#include <gnuradio/neighbor_interface_info.hpp>
#include <gnuradio/scheduler.hpp>

namespace gr {
struct graph_partition_info {
    scheduler_sptr scheduler;
    graph_sptr subgraph;
    neighbor_interface_map neighbor_map;
};
using graph_partition_info_vec = std::vector<graph_partition_info>;

struct graph_utils {
    static graph_partition_info_vec partition(graph_sptr input_graph, std::vector<scheduler_sptr> scheds,
                                              std::vector<domain_conf>& confs,
                                              neighbor_interface_map neighbor_intf_map = neighbor_interface_map());
};
} // namespace gr
