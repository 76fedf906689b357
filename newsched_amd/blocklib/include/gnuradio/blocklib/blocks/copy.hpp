// blocks::copy (reference blocklib/blocks/include/gnuradio/blocklib/blocks/copy.hpp:8-48).
#pragma once
#include <cstring>
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
class copy : public sync_block
{
public:
    using sptr = std::shared_ptr<copy>;
    static sptr make(size_t itemsize)
    {
        auto p = std::make_shared<copy>(itemsize);
        p->add_port(untyped_port::make("input", port_direction_t::INPUT, itemsize));
        p->add_port(untyped_port::make("out", port_direction_t::OUTPUT, itemsize));
        return p;
    }
    explicit copy(size_t itemsize) : sync_block("copy"), _itemsize(itemsize) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        std::memcpy(out[0].buffer->write_ptr(), in[0].buffer->read_ptr(), (size_t)out[0].n_items * _itemsize);
        out[0].n_produced = out[0].n_items;
        return work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize;
};
} // namespace blocks
} // namespace gr
