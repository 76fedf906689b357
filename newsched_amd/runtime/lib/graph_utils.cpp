// Domain partitioning (reference runtime/lib/graph_utils.cpp:11-205): split the graph by
// domain_conf, replace every crossing edge with an adapter pair, and record the
// neighbouring schedulers of the blocks at each crossing.
#include <gnuradio/block.hpp>
#include <gnuradio/domain_adapter_remote.hpp>
#include <gnuradio/graph_utils.hpp>

#include <algorithm>
#include <map>

namespace gr {

graph_partition_info_vec graph_utils::partition(graph_sptr input_graph, std::vector<scheduler_sptr> scheds,
                                                std::vector<domain_conf>& confs, neighbor_interface_map nmap)
{
    graph_partition_info_vec ret;
    std::map<nodeid_t, scheduler_sptr> blk_sched;
    std::map<nodeid_t, size_t> blk_part;
    struct crossing {
        edge_sptr e;
        size_t conf;
    };
    std::vector<crossing> crossings;

    for (size_t ci = 0; ci < confs.size(); ++ci) {
        auto& conf = confs[ci];
        auto g = graph::make();
        graph_partition_info info;
        auto blocks = conf.blocks();
        for (auto& b : blocks) {
            blk_sched[b->id()] = conf.sched();
            blk_part[b->id()] = ci;
            for (auto& in : b->input_stream_ports()) {
                auto es = input_graph->find_edge(in);
                if (es.empty()) continue;
                auto e = es[0]; // an input port has exactly one upstream edge
                if (std::find(blocks.begin(), blocks.end(), e->src().node()) != blocks.end())
                    g->connect(e->src(), e->dst())->set_custom_buffer(e->buffer_factory(), e->buf_properties());
                else
                    crossings.push_back({ e, ci });
            }
            if (nmap.count(b->id())) info.neighbor_map = nmap;
        }
        info.subgraph = g;
        info.scheduler = conf.sched();
        ret.push_back(info);
    }

    // blocks with no edge inside their own partition still belong to it
    for (size_t ci = 0; ci < confs.size(); ++ci) {
        auto g = ret[ci].subgraph;
        for (auto& b : confs[ci].blocks()) {
            bool connected = false;
            for (auto& e : g->edges())
                if (e->src().node() == b || e->dst().node() == b) connected = true;
            if (!connected) g->add_orphan_node(b);
        }
    }

    // Crossings are numbered in the order found above: identical in every process that
    // builds the same flowgraph and domain_conf list, so crossing i names the same edge
    // (and TCP port) on both sides of a process boundary.
    int crossing_index = 0;
    for (auto& c : crossings) {
        const int xi = crossing_index++;
        auto src_node = c.e->src().node();
        auto dst_node = c.e->dst().node();
        if (!blk_part.count(src_node->id()) || !blk_part.count(dst_node->id()))
            throw std::runtime_error("Cannot find both sides of domain adapter");
        auto& conf = confs[c.conf]; // the downstream block's domain
        domain_adapter_conf_sptr da_conf = nullptr;
        for (auto& ec : conf.da_edge_confs())
            if (*std::get<0>(ec) == *c.e) da_conf = std::get<1>(ec);
        if (!da_conf) da_conf = conf.da_conf();
        if (!da_conf) throw std::runtime_error("domain crossing without a domain_adapter_conf");

        const bool src_remote = std::dynamic_pointer_cast<remote_domain>(blk_sched[src_node->id()]) != nullptr;
        const bool dst_remote = std::dynamic_pointer_cast<remote_domain>(blk_sched[dst_node->id()]) != nullptr;
        const std::string name = "da_" + src_node->alias() + "->" + dst_node->alias();
        if (src_remote && dst_remote) continue; // neither end runs here
        if (src_remote || dst_remote) {
            // the far block does not run in this process: notifications must stop at the
            // adapter instead of reaching its (scheduler-less) port
            c.e->src().port()->disconnect(c.e->dst().port());
            c.e->dst().port()->disconnect(c.e->src().port());
            // one half only; the other process builds the matching half for crossing xi
            if (!src_remote) {
                auto up = da_conf->make_remote_adapter(c.e->src().port(), true, xi, name);
                ret[blk_part[src_node->id()]]
                    .subgraph->connect(c.e->src(), node_endpoint(up, up->all_ports()[0]))
                    ->set_custom_buffer(c.e->buffer_factory(), c.e->buf_properties());
            } else {
                auto down = da_conf->make_remote_adapter(c.e->dst().port(), false, xi, name);
                ret[blk_part[dst_node->id()]]
                    .subgraph->connect(node_endpoint(down, down->all_ports()[0]), c.e->dst())
                    ->set_custom_buffer(c.e->buffer_factory(), c.e->buf_properties());
            }
            continue;
        }

        auto pair = da_conf->make_domain_adapter_pair(c.e->src().port(), c.e->dst().port(), name);
        auto up = pair.first;    // takes the upstream block's output
        auto down = pair.second; // feeds the downstream block's input
        ret[blk_part[src_node->id()]]
            .subgraph->connect(c.e->src(), node_endpoint(up, up->all_ports()[0]))
            ->set_custom_buffer(c.e->buffer_factory(), c.e->buf_properties());
        ret[blk_part[dst_node->id()]]
            .subgraph->connect(node_endpoint(down, down->all_ports()[0]), c.e->dst())
            ->set_custom_buffer(c.e->buffer_factory(), c.e->buf_properties());

        ret[blk_part[dst_node->id()]].neighbor_map[dst_node->id()].set_upstream(blk_sched[src_node->id()], src_node->id());
        ret[blk_part[src_node->id()]].neighbor_map[src_node->id()].add_downstream(blk_sched[dst_node->id()], dst_node->id());
    }
    (void)scheds;
    return ret;
}

} // namespace gr
