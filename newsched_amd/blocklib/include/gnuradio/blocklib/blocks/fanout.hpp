// blocks::fanout (reference blocklib/blocks/include/gnuradio/blocklib/blocks/fanout.hpp).
#pragma once
#include <cstring>
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
class fanout : public sync_block
{
public:
    using sptr = std::shared_ptr<fanout>;
    static sptr make(size_t itemsize, size_t nports = 2)
    {
        auto p = std::make_shared<fanout>(itemsize, nports);
        p->add_port(untyped_port::make("input", port_direction_t::INPUT, itemsize));
        for (size_t i = 0; i < nports; ++i)
            p->add_port(untyped_port::make("out" + std::to_string(i), port_direction_t::OUTPUT, itemsize));
        return p;
    }
    fanout(size_t itemsize, size_t nports) : sync_block("fanout"), _itemsize(itemsize), _nports(nports) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        for (auto& o : out) {
            std::memcpy(o.buffer->write_ptr(), in[0].buffer->read_ptr(), (size_t)o.n_items * _itemsize);
            o.n_produced = o.n_items;
        }
        return work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize, _nports;
};
} // namespace blocks
} // namespace gr
