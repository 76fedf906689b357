// gr::hip::synth_source -- device-side counter-based synthetic complex stream
// (nsh_synth_cf32). Regenerable anywhere from (seed, index), so shards
// and halos on other GPUs need no transfer. Optional item limit (then WORK_DONE).
#pragma once
#include <gnuradio/sync_block.hpp>
#include <stdexcept>

namespace gr {
namespace hip {
class synth_source : public sync_block
{
public:
    using sptr = std::shared_ptr<synth_source>;
    // first_index / nitems count samples; items are vlen samples each.
    static sptr make(uint64_t first_index = 0, uint64_t nitems = 0, uint64_t seed = 0x6E736368, size_t vlen = 1)
    {
        auto p = std::make_shared<synth_source>(first_index, nitems, seed, vlen);
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    synth_source(uint64_t first_index, uint64_t nitems, uint64_t seed, size_t vlen = 1)
        : sync_block("synth_source (hip)"), _first(first_index), _limit(nitems), _seed(seed), _vlen(vlen)
    {
        if (vlen == 0 || nitems % vlen) throw std::invalid_argument("synth_source: nitems must be a multiple of vlen");
    }
    bool start() override
    {
        _index = _first;
        return sync_block::start();
    }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;

private:
    uint64_t _first, _limit, _seed, _index = 0;
    size_t _vlen;
};
} // namespace hip
} // namespace gr
