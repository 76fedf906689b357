// gr::hip::fft_vcc (1024-point, forward or inverse, unnormalised) and
// gr::hip::channelizer_vcc (fft -> multiply by w -> ifft, fused; BASELINE config C4).
// Items are vectors of 1024 complex samples (port dims {1024}, 8192 B per item).
#pragma once
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace hip {
class fft_vcc : public sync_block
{
public:
    using sptr = std::shared_ptr<fft_vcc>;
    static sptr make(size_t fft_size = 1024, bool forward = true)
    {
        auto p = std::make_shared<fft_vcc>(fft_size, forward);
        p->add_port(port<gr_complex>::make("in", port_direction_t::INPUT, { fft_size }));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT, { fft_size }));
        return p;
    }
    fft_vcc(size_t fft_size, bool forward);
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    bool forward() const { return _forward; }
    size_t fft_size() const { return 1024; }

private:
    bool _forward;
};

class channelizer_vcc : public sync_block
{
public:
    using sptr = std::shared_ptr<channelizer_vcc>;
    static sptr make(const std::vector<gr_complex>& w)
    {
        auto p = std::make_shared<channelizer_vcc>(w);
        p->add_port(port<gr_complex>::make("in", port_direction_t::INPUT, { 1024 }));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT, { 1024 }));
        return p;
    }
    explicit channelizer_vcc(const std::vector<gr_complex>& w);
    const std::vector<gr_complex>& w() const { return _w; }
    ~channelizer_vcc() override;
    bool start() override;
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;

private:
    std::vector<gr_complex> _w;
    void* _wdev = nullptr;
};
} // namespace hip
} // namespace gr
