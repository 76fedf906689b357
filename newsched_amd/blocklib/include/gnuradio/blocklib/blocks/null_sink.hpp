// blocks::null_sink -- consumes everything, touches nothing (reference
// blocklib/blocks/include/gnuradio/blocklib/blocks/null_sink.hpp:17-51). Works on any
// buffer type, device rings included.
#pragma once
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
class null_sink : public sync_block
{
public:
    using sptr = std::shared_ptr<null_sink>;
    static sptr make(size_t itemsize, size_t nports = 1)
    {
        auto p = std::make_shared<null_sink>(itemsize, nports);
        for (size_t i = 0; i < nports; ++i)
            p->add_port(untyped_port::make("input" + std::to_string(i), port_direction_t::INPUT, itemsize));
        return p;
    }
    null_sink(size_t itemsize, size_t nports) : sync_block("null_sink"), _itemsize(itemsize), _nports(nports) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>&) override
    {
        _consumed += in.empty() ? 0 : (uint64_t)in[0].n_items;
        return work_return_code_t::WORK_OK;
    }
    bool start() override
    {
        _consumed = 0;
        return sync_block::start();
    }
    uint64_t consumed() const { return _consumed; }

private:
    size_t _itemsize, _nports;
    uint64_t _consumed = 0;
};
} // namespace blocks
} // namespace gr
