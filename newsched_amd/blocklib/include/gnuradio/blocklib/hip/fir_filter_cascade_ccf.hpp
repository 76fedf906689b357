// gr::hip::fir_filter_cascade_ccf -- a chain of decimating FIRs as ONE decimating block (the
// fused form of fir_filter_ccf(h_1, D_1) -> ... -> fir_filter_ccf(h_S, D_S); BASELINE config C5).
// scheduler_hip's FIR-chain fusion pass builds it from such chains; it can also be placed
// directly. The chain composes into y[m] = sum_n heq[n] x[m D - n], D = prod D_s (8 or 16),
// computed in one pass over HBM by polyphase-FFT overlap-save (nsh_fir_cascade_ccf,
// k_fir_pfft<D>): outputs within fp32 transform rounding of the staged chain (north-star
// tolerance 1e-5), not bit-identical to it. The rounding is relative to each 512-row frame's
// input level, not to each output: |y - y_chain| <= 1e-5 |y_chain| + 1e-6 max|x in the frame|
// sum|heq|, so a quiet stretch sharing a frame with a far louder burst is accurate to the
// burst's level (nsh_hip.h). Frames holding inf/NaN run the staged chain itself: NaN and inf
// outputs exactly where the chain puts them. State: the (len(heq) - 1)-sample input history,
// ping-ponged between work() calls like fir_filter_ccf's; zeroed on every start() -- the same
// state as a chain whose stages all start from zero history.
// Tags: propagated as by one decimating block with D = prod D_s (the runtime's rule applied
// once, graph_executor.cpp), not once per stage.
#pragma once
#include <gnuradio/decim_block.hpp>

#include <utility>

namespace gr {
namespace hip {
class fir_filter_cascade_ccf : public decim_block
{
public:
    using stage = std::pair<std::vector<float>, int>; // (taps, decimation)
    using sptr = std::shared_ptr<fir_filter_cascade_ccf>;
    static sptr make(const std::vector<stage>& stages)
    {
        auto p = std::make_shared<fir_filter_cascade_ccf>(stages);
        p->add_port(port<gr_complex>::make("in", port_direction_t::INPUT));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT));
        return p;
    }
    explicit fir_filter_cascade_ccf(const std::vector<stage>& stages);
    ~fir_filter_cascade_ccf() override;
    bool start() override;
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;

    const std::vector<stage>& stages() const { return _stages; }
    // Whether a chain qualifies (host arithmetic only): total decimation 8 or 16, finite taps,
    // and a composite filter of at most 256 output rows of history (ceil((len(heq)-1)/D) <= 256).
    static bool supported(const std::vector<stage>& stages);
    std::string kernel() const; // after start()
    uint64_t launches() const { return _launches; }

    // Per-launch kernel timing with HIP events on the launch stream, as fir_filter_ccf's.
    void enable_timing(bool on) { _timing = on; }
    double kernel_ms();
    uint64_t timed_samples() const { return _timed_samples; } // outputs of the timed launches

private:
    void release();
    std::vector<stage> _stages;
    int _dev = -1;
    void* _plan = nullptr;
    size_t _hist_len = 0;
    void* _hist[2] = { nullptr, nullptr };
    bool _zero_hist = true;
    int _cur = 0;
    uint64_t _launches = 0;
    bool _timing = false;
    std::vector<std::pair<void*, void*>> _ev;
    size_t _ev_used = 0;
    uint64_t _timed_samples = 0;
};
} // namespace hip
} // namespace gr
