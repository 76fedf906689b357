// Edge -> buffer assignment and sizing (reference schedulers/mt/include/gnuradio/
// schedulers/mt/buffer_management.hpp, schedulers/mt/lib/buffer_management.cpp:8-148).
// Every edge gets a buffer from its custom factory or the scheduler default, sized
// 2 * fixed_buf_size / itemsize items (reference :117); domain adapters become the edge
// buffer on their side of a crossing (:31-73).
#pragma once
#include <gnuradio/flat_graph.hpp>
#include <map>

namespace gr {
namespace schedulers {

class buffer_manager
{
public:
    using sptr = std::shared_ptr<buffer_manager>;
    explicit buffer_manager(size_t default_buffer_size_in_bytes) : s_fixed_buf_size(default_buffer_size_in_bytes) {}

    void initialize_buffers(flat_graph_sptr fg, buffer_factory_function buf_factory,
                            std::shared_ptr<buffer_properties> buf_props);
    buffer_sptr get_input_buffer(port_sptr p) { return d_block_buffers.at(p)[0]; }
    std::vector<buffer_sptr>& get_output_buffers(port_sptr p) { return d_block_buffers.at(p); }
    std::vector<buffer_sptr> all_buffers() const;

    // Items for the edge buffer: 2 * fixed_buf_size / itemsize, at least 2 * D *
    // output_multiple when the downstream block decimates by D.
    size_t get_buffer_num_items(edge_sptr e, flat_graph_sptr fg) const;

private:
    const size_t s_fixed_buf_size;
    std::map<port_sptr, std::vector<buffer_sptr>> d_block_buffers;
    std::map<edge*, buffer_sptr> d_edge_buffers;
};

} // namespace schedulers
} // namespace gr
