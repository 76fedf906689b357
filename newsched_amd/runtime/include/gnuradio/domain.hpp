// Domain configuration: one scheduler + its blocks + adapter policy (reference
// runtime/include/gnuradio/domain.hpp:23-47).
#pragma once
#include <gnuradio/block.hpp>
#include <gnuradio/domain_adapter.hpp>
#include <gnuradio/graph.hpp>
#include <gnuradio/scheduler.hpp>

namespace gr {
class domain_conf
{
public:
    domain_conf(scheduler_sptr sched, std::vector<node_sptr> blocks, domain_adapter_conf_sptr da_conf = nullptr,
                domain_adapter_conf_per_edge da_edge_confs = domain_adapter_conf_per_edge())
        : _sched(std::move(sched)), _blocks(std::move(blocks)), _da_conf(std::move(da_conf)),
          _da_edge_confs(std::move(da_edge_confs))
    {
    }
    scheduler_sptr sched() const { return _sched; }
    std::vector<node_sptr> blocks() const { return _blocks; }
    domain_adapter_conf_sptr da_conf() const { return _da_conf; }
    domain_adapter_conf_per_edge da_edge_confs() const { return _da_edge_confs; }

private:
    scheduler_sptr _sched;
    std::vector<node_sptr> _blocks;
    domain_adapter_conf_sptr _da_conf;
    domain_adapter_conf_per_edge _da_edge_confs;
};
using domain_conf_vec = std::vector<domain_conf>;
} // namespace gr
