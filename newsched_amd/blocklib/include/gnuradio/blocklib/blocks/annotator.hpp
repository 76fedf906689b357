// blocks::annotator: tag test block (reference blocklib/blocks/include/gnuradio/blocklib/
// blocks/annotator.hpp:19-60, lib/annotator.cpp:26-105). Items pass untouched (the data is
// irrelevant); every `when` items written to each output it adds a tag ("seq", running
// counter, srcid = its alias) at that absolute offset, and it records every tag it sees in
// the window each work() call reads. The scheduler propagates tags by the block's policy.
#pragma once
#include <gnuradio/sync_block.hpp>
#include <string>

namespace gr {
namespace blocks {
class annotator : public sync_block
{
public:
    using sptr = std::shared_ptr<annotator>;
    static sptr make(uint64_t when, size_t itemsize, size_t num_inputs, size_t num_outputs,
                     tag_propagation_policy_t tpp)
    {
        auto p = std::make_shared<annotator>(when, num_inputs, num_outputs);
        for (size_t i = 0; i < num_inputs; ++i)
            p->add_port(untyped_port::make("in" + std::to_string(i), port_direction_t::INPUT, itemsize));
        for (size_t i = 0; i < num_outputs; ++i)
            p->add_port(untyped_port::make("out" + std::to_string(i), port_direction_t::OUTPUT, itemsize));
        p->set_tag_propagation_policy(tpp);
        return p;
    }
    annotator(uint64_t when, size_t num_inputs, size_t num_outputs)
        : sync_block("annotator"), _when(when), _nin(num_inputs), _nout(num_outputs)
    {
    }
    std::vector<tag_t> data() const { return _seen; }

    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        const int n = out[0].n_items;
        for (size_t i = 0; i < _nin; ++i) {
            auto t = in[i].buffer->tags_in_window(0, (uint64_t)n);
            _seen.insert(_seen.end(), t.begin(), t.end());
        }
        const auto key = pmtf::make("seq");
        const auto src = pmtf::make(alias());
        const uint64_t first = out[0].buffer->total_written();
        for (int j = 0; j < n; ++j)
            for (size_t o = 0; o < _nout; ++o)
                if ((first + (uint64_t)j) % _when == 0)
                    out[o].buffer->add_tag(first + (uint64_t)j, key, pmtf::make((int64_t)_counter++), src);
        for (auto& w : out) w.n_produced = n;
        return work_return_code_t::WORK_OK;
    }

private:
    uint64_t _when;
    size_t _nin, _nout;
    uint64_t _counter = 0;
    std::vector<tag_t> _seen;
};
} // namespace blocks
} // namespace gr
