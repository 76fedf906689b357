// Edge buffers (reference schedulers/mt/lib/buffer_management.cpp:8-148).
#include <cmath>
#include <gnuradio/block.hpp>
#include <gnuradio/domain_adapter.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/schedulers/mt/buffer_management.hpp>

namespace gr {
namespace schedulers {

void buffer_manager::initialize_buffers(flat_graph_sptr fg, buffer_factory_function buf_factory,
                                        std::shared_ptr<buffer_properties> buf_props)
{
    auto make_buf = [&](const edge_sptr& e) {
        const size_t n = get_buffer_num_items(e, fg);
        buffer_sptr b = e->has_custom_buffer() ? e->buffer_factory()(n, e->itemsize(), e->buf_properties())
                                               : buf_factory(n, e->itemsize(), buf_props);
        b->set_name(e->identifier());
        return b;
    };
    for (auto& e : fg->edges()) {
        // A domain adapter on either end IS the edge buffer on this side of the crossing:
        //   BLK1 -> [DA] ~~~ [DA] -> BLK2     (the LOCAL adapter owns the real buffer)
        auto da = std::dynamic_pointer_cast<domain_adapter>(e->src().node());
        if (!da) da = std::dynamic_pointer_cast<domain_adapter>(e->dst().node());
        if (da) {
            if (da->buffer_location() == buffer_location_t::LOCAL) {
                da->set_buffer(make_buf(e));
                da->buffer_ready(); // direct: publish to the peer; remote: connect + handshake
            }
            d_edge_buffers[e.get()] = std::dynamic_pointer_cast<buffer>(da);
        } else {
            d_edge_buffers[e.get()] = make_buf(e);
        }
    }
    for (auto& b : fg->calc_used_blocks()) {
        for (auto& p : b->input_stream_ports()) {
            auto& v = d_block_buffers[p];
            v.clear();
            for (auto& e : fg->find_edge(p)) v.push_back(d_edge_buffers[e.get()]);
        }
        for (auto& p : b->output_stream_ports()) {
            auto& v = d_block_buffers[p];
            v.clear();
            for (auto& e : fg->find_edge(p)) v.push_back(d_edge_buffers[e.get()]);
        }
    }
}

std::vector<buffer_sptr> buffer_manager::all_buffers() const
{
    std::vector<buffer_sptr> r;
    for (auto& kv : d_edge_buffers) r.push_back(kv.second);
    return r;
}

size_t buffer_manager::get_buffer_num_items(edge_sptr e, flat_graph_sptr) const
{
    // 2x: buffers are filled at most half way (reference buffer_management.cpp:110-148).
    const size_t isz = e->itemsize() ? e->itemsize() : 1;
    size_t nitems = std::max<size_t>((2 * s_fixed_buf_size) / isz, 2);
    // A decimator needs D * output_multiple readable items per call: size its input edge
    // for two such calls (the reference's commented-out rule, :125-145). The edge object
    // carries both endpoints, so domain adapters do not hide the downstream block here.
    if (auto b = std::dynamic_pointer_cast<block>(e->dst().node())) {
        const double rr = b->relative_rate();
        if (rr > 0 && rr < 1.0) {
            const size_t need = 2 * (size_t)std::ceil(1.0 / rr) * (size_t)b->output_multiple();
            nitems = std::max(nitems, need);
        }
    }
    return nitems;
}

} // namespace schedulers
} // namespace gr
