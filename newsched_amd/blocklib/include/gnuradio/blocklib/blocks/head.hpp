// blocks::head / nop_head -- pass the first nitems then WORK_DONE (reference
// blocklib/blocks/include/gnuradio/blocklib/blocks/head.hpp:10-73, nop_head.hpp). The
// counter re-arms in start(), so a restarted flowgraph passes nitems again.
#pragma once
#include <algorithm>
#include <cstring>
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
template <bool COPY>
class head_t : public sync_block
{
public:
    using sptr = std::shared_ptr<head_t>;
    static sptr make(size_t itemsize, size_t nitems)
    {
        auto p = std::make_shared<head_t>(itemsize, nitems);
        p->add_port(untyped_port::make("input", port_direction_t::INPUT, itemsize));
        p->add_port(untyped_port::make("output", port_direction_t::OUTPUT, itemsize));
        return p;
    }
    head_t(size_t itemsize, size_t nitems)
        : sync_block(COPY ? "head" : "nop_head"), _itemsize(itemsize), _nitems(nitems)
    {
    }
    bool start() override
    {
        _ncopied_items = 0;
        return sync_block::start();
    }
    // items passed per run from the next start() on (GNU Radio head::set_length)
    void set_length(size_t nitems) { _nitems = nitems; }
    size_t length() const { return _nitems; }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        if (_ncopied_items >= _nitems) {
            out[0].n_produced = 0;
            return work_return_code_t::WORK_DONE;
        }
        const size_t n = std::min<size_t>(_nitems - _ncopied_items, (size_t)out[0].n_items);
        if (COPY && n) std::memcpy(out[0].buffer->write_ptr(), in[0].buffer->read_ptr(), n * _itemsize);
        _ncopied_items += n;
        out[0].n_produced = (int)n;
        return _ncopied_items >= _nitems ? work_return_code_t::WORK_DONE : work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize, _nitems, _ncopied_items = 0;
};
using head = head_t<true>;
using nop_head = head_t<false>;
} // namespace blocks
} // namespace gr
