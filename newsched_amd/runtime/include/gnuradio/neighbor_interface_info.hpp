// Per-block upstream/downstream scheduler neighbours across domain crossings (reference
// runtime/include/gnuradio/neighbor_interface_info.hpp).
#pragma once
#include <gnuradio/neighbor_interface.hpp>
#include <gnuradio/node.hpp>
#include <map>
#include <vector>

namespace gr {
struct neighbor_interface_info {
    std::shared_ptr<neighbor_interface> upstream_neighbor_intf = nullptr;
    nodeid_t upstream_neighbor_blkid = (nodeid_t)-1;
    std::vector<std::shared_ptr<neighbor_interface>> downstream_neighbor_intf;
    std::vector<nodeid_t> downstream_neighbor_blkids;
    void set_upstream(std::shared_ptr<neighbor_interface> intf, nodeid_t blkid)
    {
        upstream_neighbor_intf = std::move(intf);
        upstream_neighbor_blkid = blkid;
    }
    void add_downstream(std::shared_ptr<neighbor_interface> intf, nodeid_t blkid)
    {
        downstream_neighbor_intf.push_back(std::move(intf));
        downstream_neighbor_blkids.push_back(blkid);
    }
};
using neighbor_interface_map = std::map<nodeid_t, neighbor_interface_info>;
} // namespace gr
