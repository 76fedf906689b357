// gr::hip::fir_filter_ccf -- the MI355X hot path (BASELINE config C3/C5).
// Complex fp32 stream, real fp32 taps, optional decimation D (a gr::decim_block: the
// runtime clamps the call to D readable items per output and consumes D*n_produced).
// The block owns the device tap plan and two (ntaps-1)-sample history buffers it
// ping-pongs between work() calls, because the block API has no history (reference
// runtime/include/gnuradio/sync_block.hpp:36-86). Device state is created on the first
// start() on the partition thread (right device and stream) and the history is zeroed on
// every start() (a fresh stream). Algorithm: nsh_fir_algo (AUTO = MFMA for D = 1).
#pragma once
#include <gnuradio/decim_block.hpp>

namespace gr {
namespace hip {
class fir_filter_ccf : public decim_block
{
public:
    using sptr = std::shared_ptr<fir_filter_ccf>;
    static sptr make(const std::vector<float>& taps, int decim = 1, int algo = 0)
    {
        auto p = std::make_shared<fir_filter_ccf>(taps, decim, algo);
        p->add_port(port<gr_complex>::make("in", port_direction_t::INPUT));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT));
        return p;
    }
    fir_filter_ccf(const std::vector<float>& taps, int decim, int algo);
    ~fir_filter_ccf() override;
    bool start() override;
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    int decimation() const { return _decim; }
    const std::vector<float>& taps() const { return _taps; }
    int requested_algo() const { return _algo; } // as given to make() (0 = AUTO)
    bool has_initial_history() const { return !_init_hist.empty(); }
    int algo() const; // resolved algorithm (after start())
    std::string kernel() const; // the kernel its work() launches (after start())
    uint64_t launches() const { return _launches; }

    // History loaded at start() instead of zeros: the ntaps-1 samples that precede this
    // block's first input (a time shard's halo, regenerated or received by the caller).
    void set_initial_history(const std::vector<gr_complex>& h) { _init_hist = h; }

    // Per-launch kernel timing with HIP events on the launch stream (bench/profiling): every
    // `stride`-th launch is timed (its own dispatch records the pair, nsh_time_next_launch).
    void enable_timing(bool on, int stride = 1)
    {
        _timing = on;
        _stride = stride > 0 ? stride : 1;
    }
    uint64_t timed_launches() const { return _timed_launches; }
    // Sum of kernel durations (ms) and output samples over every timed launch since the block
    // was made (cumulative across runs: a caller takes differences around the runs it times).
    // Reading it synchronises on the launches' events and folds them into the total; between
    // reads a run costs only its two event records per launch.
    double kernel_ms();
    uint64_t timed_samples() const { return _timed_samples; }

private:
    void release();
    std::vector<gr_complex> _init_hist;
    bool _timing = false;
    int _stride = 1;
    uint64_t _timed_launches = 0;
    std::vector<std::pair<void*, void*>> _ev;  // (start, stop) per launch, reused
    size_t _ev_used = 0;
    double _done_ms = 0; // kernel time of the launches folded so far
    uint64_t _timed_samples = 0;
    std::vector<float> _taps;
    int _decim, _algo;
    int _dev = -1;
    void* _plan = nullptr;
    void* _hist[2] = { nullptr, nullptr };
    bool _zero_hist = true; // the next call reads a null history (zeros): set by start()
    int _cur = 0;
    uint64_t _launches = 0;
};
} // namespace hip
} // namespace gr
