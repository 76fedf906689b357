// gr::hip::copy -- device stream copy, one launch per work() (replaces cuda::copy,
// reference blocklib/cuda/include/gnuradio/blocklib/cuda/copy.hpp:11-42,
// blocklib/cuda/lib/copy.cpp:22-63, which launches per 1024-sample vector and syncs).
#pragma once
#include <gnuradio/hip_fusion.hpp>
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace hip {
class copy : public sync_block, public elementwise_cc
{
public:
    using sptr = std::shared_ptr<copy>;
    // Same make() shape as cuda::copy: items are batch_size complex samples.
    static sptr make(const size_t batch_size = 1)
    {
        auto p = std::make_shared<copy>(batch_size);
        p->add_port(port<gr_complex>::make("input", port_direction_t::INPUT, { batch_size }));
        p->add_port(port<gr_complex>::make("output", port_direction_t::OUTPUT, { batch_size }));
        return p;
    }
    explicit copy(size_t batch_size) : sync_block("copy (hip)"), d_batch_size(batch_size) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    bool elementwise_stages(std::vector<gr_complex>&) const override { return true; } // identity

private:
    size_t d_batch_size;
};
} // namespace hip
} // namespace gr
