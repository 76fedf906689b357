// blocks::null_source -- zeros (reference blocklib/blocks/include/gnuradio/blocklib/blocks/
// null_source.hpp:9-52).
#pragma once
#include <cstring>
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
class null_source : public sync_block
{
public:
    using sptr = std::shared_ptr<null_source>;
    static sptr make(size_t itemsize, size_t nports = 1)
    {
        auto p = std::make_shared<null_source>(itemsize, nports);
        for (size_t i = 0; i < nports; ++i)
            p->add_port(untyped_port::make("out" + std::to_string(i), port_direction_t::OUTPUT, itemsize));
        return p;
    }
    null_source(size_t itemsize, size_t nports) : sync_block("null_source"), _itemsize(itemsize), _nports(nports) {}
    work_return_code_t work(std::vector<block_work_input>&, std::vector<block_work_output>& out) override
    {
        for (auto& o : out) {
            std::memset(o.buffer->write_ptr(), 0, (size_t)o.n_items * _itemsize);
            o.n_produced = o.n_items;
        }
        return work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize, _nports;
};
} // namespace blocks
} // namespace gr
