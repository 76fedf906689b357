// blocks::nop / nop_source: pass/produce items without touching memory (reference
// blocklib/blocks/include/gnuradio/blocklib/blocks/nop.hpp, nop_source.hpp) -- scheduler
// overhead benches, and the "inputs already resident" bench configuration.
#pragma once
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
class nop : public sync_block
{
public:
    using sptr = std::shared_ptr<nop>;
    static sptr make(size_t itemsize)
    {
        auto p = std::make_shared<nop>(itemsize);
        p->add_port(untyped_port::make("input", port_direction_t::INPUT, itemsize));
        p->add_port(untyped_port::make("out", port_direction_t::OUTPUT, itemsize));
        return p;
    }
    explicit nop(size_t itemsize) : sync_block("nop"), _itemsize(itemsize) {}
    work_return_code_t work(std::vector<block_work_input>&, std::vector<block_work_output>& out) override
    {
        out[0].n_produced = out[0].n_items;
        return work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize;
};

class nop_source : public sync_block
{
public:
    using sptr = std::shared_ptr<nop_source>;
    static sptr make(size_t itemsize, size_t nports = 1)
    {
        auto p = std::make_shared<nop_source>(itemsize, nports);
        for (size_t i = 0; i < nports; ++i)
            p->add_port(untyped_port::make("out" + std::to_string(i), port_direction_t::OUTPUT, itemsize));
        return p;
    }
    nop_source(size_t itemsize, size_t nports) : sync_block("nop_source"), _itemsize(itemsize), _nports(nports) {}
    work_return_code_t work(std::vector<block_work_input>&, std::vector<block_work_output>& out) override
    {
        for (auto& o : out) o.n_produced = o.n_items;
        return work_return_code_t::WORK_OK;
    }

private:
    size_t _itemsize, _nports;
};
} // namespace blocks
} // namespace gr
