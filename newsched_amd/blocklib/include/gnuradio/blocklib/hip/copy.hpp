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
    // Same make() as cuda::copy (copy.hpp:17-27): items are batch_size complex samples; `load`
    // repeats the copy (the reference's compute-load knob, copy.cu:7-16, here `load` passes
    // over the items per work()). A block with load > 1 is kept out of scheduler_hip's fusion
    // so that its load is really paid.
    static sptr make(const size_t batch_size = 1, const size_t load = 1)
    {
        auto p = std::make_shared<copy>(batch_size, load);
        p->add_port(port<gr_complex>::make("input", port_direction_t::INPUT, { batch_size }));
        p->add_port(port<gr_complex>::make("output", port_direction_t::OUTPUT, { batch_size }));
        return p;
    }
    copy(size_t batch_size, size_t load = 1)
        : sync_block("copy (hip)"), d_batch_size(batch_size), d_load(load < 1 ? 1 : load)
    {
    }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    bool elementwise_stages(std::vector<gr_complex>&) const override { return d_load == 1; } // identity
    size_t load() const { return d_load; }

private:
    size_t d_batch_size;
    size_t d_load;
};
} // namespace hip
} // namespace gr
