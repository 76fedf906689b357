// 1:1 block (reference runtime/include/gnuradio/sync_block.hpp:13-86): every port is
// clamped to the smallest item count before work(), all outputs must produce the same
// count, and every input consumes what was produced (all of n_items when there are no
// outputs). A mismatch throws std::runtime_error by value (the reference throws a
// pointer, sync_block.hpp:75, Appendix A quirk not replicated).
#pragma once
#include <algorithm>
#include <gnuradio/block.hpp>
#include <limits>

namespace gr {

class sync_block : public block
{
public:
    explicit sync_block(const std::string& name) : block(name) {}

    work_return_code_t do_work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        int n = std::numeric_limits<int>::max();
        for (auto& w : in) n = std::min(n, w.n_items);
        for (auto& w : out) n = std::min(n, w.n_items);
        for (auto& w : in) w.n_items = n;
        for (auto& w : out) w.n_items = n;

        const work_return_code_t ret = work(in, out);

        int produced = -1;
        for (size_t i = 0; i < out.size(); ++i) {
            if (i == 0)
                produced = out[i].n_produced;
            else if (out[i].n_produced != produced)
                throw std::runtime_error("outputs for sync_block must produce same number of items");
        }
        for (auto& w : in) w.n_consumed = produced < 0 ? w.n_items : produced;
        return ret;
    }
};

} // namespace gr
