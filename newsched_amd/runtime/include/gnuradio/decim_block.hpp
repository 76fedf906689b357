// D:1 block: the `decim_block` special case the reference's block::do_work documents
// (runtime/include/gnuradio/block.hpp:86-99) but never implements. Every output is clamped
// to the smallest count such that D items per output are readable on every input, work()
// sets n_produced (equal on all outputs), and every input consumes D * n_produced. Buffer
// managers size the edges into a decimator for at least 2 * D * output_multiple items
// (the reference's commented-out rule, schedulers/mt/lib/buffer_management.cpp:125-145).
#pragma once
#include <algorithm>
#include <gnuradio/block.hpp>
#include <limits>
#include <stdexcept>

namespace gr {

class decim_block : public block
{
public:
    decim_block(const std::string& name, unsigned decimation) : block(name), _decim(decimation ? decimation : 1) {}
    unsigned decimation() const { return _decim; }
    double relative_rate() const override { return 1.0 / (double)_decim; }

    work_return_code_t do_work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        int n = std::numeric_limits<int>::max();
        for (auto& w : in) n = std::min(n, w.n_items / (int)_decim);
        for (auto& w : out) n = std::min(n, w.n_items);
        if (n <= 0) return work_return_code_t::WORK_INSUFFICIENT_INPUT_ITEMS;
        for (auto& w : in) w.n_items = n * (int)_decim;
        for (auto& w : out) w.n_items = n;

        const work_return_code_t ret = work(in, out);

        int produced = -1;
        for (size_t i = 0; i < out.size(); ++i) {
            if (i == 0)
                produced = out[i].n_produced;
            else if (out[i].n_produced != produced)
                throw std::runtime_error("outputs for decim_block must produce same number of items");
        }
        for (auto& w : in) w.n_consumed = produced < 0 ? 0 : produced * (int)_decim;
        return ret;
    }

private:
    unsigned _decim;
};

} // namespace gr
