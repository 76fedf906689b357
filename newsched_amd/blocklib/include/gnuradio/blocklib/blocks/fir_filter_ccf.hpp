// blocks::fir_filter_ccf: CPU restatement of GNU Radio's fir_filter_ccf (complex stream,
// real taps, optional decimation), y[m] = sum_k h[k] x[m D - k], zero initial history.
// Absent from the reference; this is the CPU-baseline FIR the bench
// times on the host cores (thread per block, 8192-item vmcircbuf edges), vectorised for
// AVX-512/AVX2 by function multiversioning dispatched on CPU features (cpu_isa() names the
// variant this process runs), fp32 accumulation in tap order. A gr::decim_block: the runtime
// clamps and consumes D items per output.
#pragma once
#include <gnuradio/decim_block.hpp>

namespace gr {
namespace blocks {
class fir_filter_ccf : public decim_block
{
public:
    using sptr = std::shared_ptr<fir_filter_ccf>;
    static sptr make(const std::vector<float>& taps, int decim = 1)
    {
        auto p = std::make_shared<fir_filter_ccf>(taps, decim);
        p->add_port(port<gr_complex>::make("in", port_direction_t::INPUT));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT));
        return p;
    }
    fir_filter_ccf(const std::vector<float>& taps, int decim);
    bool start() override;
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    // work()'s arithmetic on plain arrays: n_out outputs from n_out * D inputs, history carried
    // over from the previous call (zeros before the first). The CPU baseline times it alone.
    void filter(const gr_complex* in, gr_complex* out, int n_out);
    const std::vector<float>& taps() const { return _taps; }
    int decimation() const { return _decim; }

private:
    std::vector<float> _taps;  // h[0..L)
    int _decim;
    std::vector<gr_complex> _ext; // [history (L-1) | current input]
};
// The vector ISA the CPU blocks dispatched to in this process ("avx512f+fma", "avx2+fma", ...).
const char* cpu_isa();
} // namespace blocks
} // namespace gr
