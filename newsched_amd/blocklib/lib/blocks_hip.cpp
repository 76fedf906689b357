// gr::hip::* block work() implementations: argument plumbing from block_work_io to the
// libnsh_hip.so C-ABI on the thread's HIP stream. Nonzero codes throw (hip::check).
#include <gnuradio/run_trace.hpp>
#include <gnuradio/blocklib/hip/arith.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
#include <gnuradio/blocklib/hip/fft.hpp>
#include <gnuradio/blocklib/hip/fir_filter_cascade_ccf.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/blocklib/hip/synth_source.hpp>
#include <gnuradio/hip_context.hpp>

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "nsh_hip.h"

namespace gr {
namespace hip {

work_return_code_t copy::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const size_t n = (size_t)out[0].n_items;
    for (size_t l = 0; l < d_load; ++l)
        check(nsh_copy(in[0].buffer->read_ptr(), out[0].buffer->write_ptr(), n * d_batch_size * sizeof(gr_complex),
                       current_stream()),
              "hip::copy");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

template <>
work_return_code_t multiply_const<gr_complex>::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    check(nsh_mul_const_cc((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(),
                           (int64_t)out[0].n_items * (int64_t)d_vlen, d_k.real(), d_k.imag(), current_stream()),
          "hip::multiply_const_cc");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

template <>
work_return_code_t multiply_const<float>::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    check(nsh_mul_const_ff((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(),
                           (int64_t)out[0].n_items * (int64_t)d_vlen, d_k, current_stream()),
          "hip::multiply_const_ff");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}
template class multiply_const<gr_complex>;
template class multiply_const<float>;

multiply_const_vcc::multiply_const_vcc(const std::vector<gr_complex>& k) : sync_block("multiply_const_vcc (hip)"), d_k(k)
{
    if (k.empty()) throw std::invalid_argument("hip::multiply_const_vcc: k must not be empty");
}
multiply_const_vcc::~multiply_const_vcc()
{
    if (d_kdev) nsh_free(d_kdev);
}
bool multiply_const_vcc::start()
{
    if (!d_kdev) { // the constant lives on the device of the thread that runs the block
        check(nsh_malloc(current_device(), d_k.size() * sizeof(gr_complex), &d_kdev), "hip::multiply_const_vcc");
        check(nsh_memcpy_async(d_kdev, d_k.data(), d_k.size() * sizeof(gr_complex), NSH_H2D, current_stream()),
              "hip::multiply_const_vcc");
        check(nsh_stream_sync(current_stream()), "hip::multiply_const_vcc");
    }
    return sync_block::start();
}
work_return_code_t multiply_const_vcc::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    check(nsh_mul_const_vcc((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(),
                            (const float*)d_kdev, (int)d_k.size(), out[0].n_items, current_stream()),
          "hip::multiply_const_vcc");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

work_return_code_t multiply_const_chain_cc::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    std::vector<float> k;
    k.reserve(2 * d_ks.size());
    for (auto& c : d_ks) {
        k.push_back(c.real());
        k.push_back(c.imag());
    }
    check(nsh_mul_const_chain_cc((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(),
                                 (int64_t)out[0].n_items * (int64_t)d_vlen, k.data(), (int)d_ks.size(), current_stream()),
          "hip::multiply_const_chain_cc");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

template <int OP>
work_return_code_t arith_cc<OP>::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const int64_t n = (int64_t)out[0].n_items * (int64_t)_vlen;
    float* o = (float*)out[0].buffer->write_ptr();
    void* s = current_stream();
    if (_nports == 1) {
        check(nsh_copy(in[0].buffer->read_ptr(), o, (size_t)n * 8, s), "hip::arith_cc");
    } else {
        for (size_t p = 1; p < _nports; ++p) {
            const float* a = p == 1 ? (const float*)in[0].buffer->read_ptr() : o;
            const float* b = (const float*)in[p].buffer->read_ptr();
            check(OP == 0 ? nsh_add_cc(a, b, o, n, s) : nsh_mul_cc(a, b, o, n, s), OP == 0 ? "hip::add_cc" : "hip::multiply_cc");
        }
    }
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}
template class arith_cc<0>;
template class arith_cc<1>;

// ---- FIR ---------------------------------------------------------------------------
fir_filter_ccf::fir_filter_ccf(const std::vector<float>& taps, int decim, int algo)
    : decim_block("fir_filter_ccf (hip)", (unsigned)decim), _taps(taps), _decim(decim), _algo(algo)
{
    if (taps.empty()) throw std::invalid_argument("hip::fir_filter_ccf: no taps");
    if (decim != 1 && decim != 2 && decim != 4 && decim != 8 && decim != 16)
        throw std::invalid_argument("hip::fir_filter_ccf: decimation must be 1, 2, 4, 8 or 16");
}

fir_filter_ccf::~fir_filter_ccf() { release(); }

void fir_filter_ccf::release()
{
    for (auto& e : _ev) {
        nsh_event_destroy(e.first);
        nsh_event_destroy(e.second);
    }
    _ev.clear();
    _ev_used = 0;
    if (_plan) nsh_fir_plan_destroy(_plan);
    for (auto& h : _hist)
        if (h) nsh_free(h);
    _plan = nullptr;
    _hist[0] = _hist[1] = nullptr;
}

int fir_filter_ccf::algo() const { return _plan ? nsh_fir_plan_algo(_plan) : _algo; }
std::string fir_filter_ccf::kernel() const { return _plan ? nsh_fir_plan_kernel(_plan) : std::string(); }

bool fir_filter_ccf::start()
{
    const int dev = current_device();
    if (_plan && dev != _dev) release();
    const size_t hbytes = std::max<size_t>(_taps.size() - 1, 1) * sizeof(gr_complex);
    if (!_plan) {
        _dev = dev;
        check(nsh_fir_plan_create(dev, _taps.data(), (int)_taps.size(), _decim, _algo, &_plan), "hip::fir_filter_ccf plan");
        check(nsh_malloc(dev, hbytes, &_hist[0]), "hip::fir_filter_ccf history");
        check(nsh_malloc(dev, hbytes, &_hist[1]), "hip::fir_filter_ccf history");
    }
    void* s = current_stream();
    // the run's first call reads a null history (zeros in the kernel): no memset launches per run;
    // every call writes its hist_out in full, so the ping-pong buffers need no clearing
    _zero_hist = true;
    if (!_init_hist.empty()) {
        if (_init_hist.size() != _taps.size() - 1)
            throw std::invalid_argument("hip::fir_filter_ccf: initial history must have ntaps-1 samples");
        check(nsh_memcpy_async(_hist[0], _init_hist.data(), hbytes, NSH_H2D, s), "hip::fir_filter_ccf history load");
        check(nsh_stream_sync(s), "hip::fir_filter_ccf history load"); // host vector must outlive the copy
        _zero_hist = false;
    }
    _cur = 0;
    // the events of earlier runs are folded into the total when it is read (kernel_ms), not here:
    // nothing per run but the two records per launch; a long unread series is folded at 4096
    if (_ev_used >= 4096) kernel_ms();
    return block::start();
}

// Kernel timing: the launch records its own start / stop events (nsh_time_next_launch) unless
// NSH_FIR_TIMING=records asks for the two event records around the call (A/B of the two forms).
static bool timing_by_records()
{
    static const bool r = [] {
        const char* v = std::getenv("NSH_FIR_TIMING");
        return v && std::string(v) == "records";
    }();
    return r;
}

work_return_code_t fir_filter_ccf::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const int n_out = out[0].n_items; // decim_block::do_work: in[0].n_items == D * n_out
    void* s = current_stream();
    std::pair<void*, void*>* ev = nullptr;
    if (_timing && _launches % (uint64_t)_stride == 0) {
        if (_ev_used == _ev.size()) {
            std::pair<void*, void*> p{ nullptr, nullptr };
            check(nsh_event_create(&p.first), "hip::fir_filter_ccf timing");
            check(nsh_event_create(&p.second), "hip::fir_filter_ccf timing");
            _ev.push_back(p);
        }
        ev = &_ev[_ev_used++];
        if (timing_by_records())
            check(nsh_event_record(ev->first, s), "hip::fir_filter_ccf timing");
        else // the launch records both events itself (nsh_time_next_launch)
            check(nsh_time_next_launch(ev->first, ev->second), "hip::fir_filter_ccf timing");
    }
    NSR_RT(4);
    check(nsh_fir_ccf(_plan, (const float*)in[0].buffer->read_ptr(), _zero_hist ? nullptr : (const float*)_hist[_cur],
                      (float*)_hist[_cur ^ 1], (float*)out[0].buffer->write_ptr(), n_out, s),
          "hip::fir_filter_ccf");
    _zero_hist = false;
    if (ev) {
        if (timing_by_records()) check(nsh_event_record(ev->second, s), "hip::fir_filter_ccf timing");
        _timed_samples += (uint64_t)n_out;
        ++_timed_launches;
    }
    NSR_RT(5);
    _cur ^= 1;
    ++_launches;
    out[0].n_produced = n_out;
    return work_return_code_t::WORK_OK;
}

double fir_filter_ccf::kernel_ms()
{
    for (size_t i = 0; i < _ev_used; ++i) {
        float ms = 0;
        check(nsh_event_sync(_ev[i].second), "hip::fir_filter_ccf timing");
        check(nsh_event_elapsed_ms(_ev[i].first, _ev[i].second, &ms), "hip::fir_filter_ccf timing");
        _done_ms += ms;
    }
    _ev_used = 0; // folded: the events are reused by the next launches
    return _done_ms;
}

// ---- fused decimating FIR chain -----------------------------------------------------
namespace {
int total_decim(const std::vector<fir_filter_cascade_ccf::stage>& st)
{
    int64_t d = 1;
    for (auto& s : st) d *= s.second > 0 ? s.second : 0;
    return d > 64 ? 64 : (int)d;
}
} // namespace

bool fir_filter_cascade_ccf::supported(const std::vector<stage>& st)
{
    if (st.empty()) return false;
    const int D = total_decim(st);
    if (D != 8 && D != 16) return false;
    int64_t len = 1, dacc = 1; // composite length 1 + sum (L_s - 1) prod_{t<s} D_t
    for (auto& s : st) {
        if (s.first.empty()) return false;
        for (float v : s.first)
            if (!std::isfinite(v)) return false;
        len += (int64_t)(s.first.size() - 1) * dacc;
        dacc *= s.second;
    }
    return (len - 1 + D - 1) / D <= 256; // nsh_fir_cascade_plan_create's limit
}

fir_filter_cascade_ccf::fir_filter_cascade_ccf(const std::vector<stage>& stages)
    : decim_block("fir_filter_cascade_ccf (hip)", (unsigned)total_decim(stages)), _stages(stages)
{
    if (!supported(stages))
        throw std::invalid_argument("hip::fir_filter_cascade_ccf: needs total decimation 8 or 16, finite taps and "
                                    "ceil((len(heq)-1)/D) <= 256");
}

fir_filter_cascade_ccf::~fir_filter_cascade_ccf() { release(); }

void fir_filter_cascade_ccf::release()
{
    for (auto& e : _ev) {
        nsh_event_destroy(e.first);
        nsh_event_destroy(e.second);
    }
    _ev.clear();
    _ev_used = 0;
    if (_plan) nsh_fir_cascade_plan_destroy(_plan);
    for (auto& h : _hist)
        if (h) nsh_free(h);
    _plan = nullptr;
    _hist[0] = _hist[1] = nullptr;
}

std::string fir_filter_cascade_ccf::kernel() const { return _plan ? nsh_fir_cascade_kernel(_plan) : std::string(); }

bool fir_filter_cascade_ccf::start()
{
    const int dev = current_device();
    if (_plan && dev != _dev) release();
    if (!_plan) {
        _dev = dev;
        std::vector<const float*> tp;
        std::vector<int> nt, dc;
        for (auto& s : _stages) {
            tp.push_back(s.first.data());
            nt.push_back((int)s.first.size());
            dc.push_back(s.second);
        }
        check(nsh_fir_cascade_plan_create(dev, tp.data(), nt.data(), dc.data(), (int)_stages.size(), &_plan),
              "hip::fir_filter_cascade_ccf plan");
        _hist_len = (size_t)nsh_fir_cascade_hist_len(_plan);
        const size_t hbytes = std::max<size_t>(_hist_len, 1) * sizeof(gr_complex);
        check(nsh_malloc(dev, hbytes, &_hist[0]), "hip::fir_filter_cascade_ccf history");
        check(nsh_malloc(dev, hbytes, &_hist[1]), "hip::fir_filter_cascade_ccf history");
    }
    _zero_hist = true; // a fresh stream: the first call reads a null (zero) history
    _cur = 0;
    _ev_used = 0;
    _timed_samples = 0;
    return block::start();
}

work_return_code_t fir_filter_cascade_ccf::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    const int n_out = out[0].n_items; // decim_block::do_work: in[0].n_items == D * n_out
    void* s = current_stream();
    std::pair<void*, void*>* ev = nullptr;
    if (_timing) {
        if (_ev_used == _ev.size()) {
            std::pair<void*, void*> p{ nullptr, nullptr };
            check(nsh_event_create(&p.first), "hip::fir_filter_cascade_ccf timing");
            check(nsh_event_create(&p.second), "hip::fir_filter_cascade_ccf timing");
            _ev.push_back(p);
        }
        ev = &_ev[_ev_used++];
        if (timing_by_records())
            check(nsh_event_record(ev->first, s), "hip::fir_filter_cascade_ccf timing");
        else // the launch records both events itself (nsh_time_next_launch)
            check(nsh_time_next_launch(ev->first, ev->second), "hip::fir_filter_cascade_ccf timing");
    }
    check(nsh_fir_cascade_ccf(_plan, (const float*)in[0].buffer->read_ptr(),
                              _zero_hist ? nullptr : (const float*)_hist[_cur], (float*)_hist[_cur ^ 1],
                              (float*)out[0].buffer->write_ptr(), n_out, s),
          "hip::fir_filter_cascade_ccf");
    _zero_hist = false;
    if (ev) {
        if (timing_by_records()) check(nsh_event_record(ev->second, s), "hip::fir_filter_cascade_ccf timing");
        _timed_samples += (uint64_t)n_out;
    }
    _cur ^= 1;
    ++_launches;
    out[0].n_produced = n_out;
    return work_return_code_t::WORK_OK;
}

double fir_filter_cascade_ccf::kernel_ms()
{
    double total = 0;
    for (size_t i = 0; i < _ev_used; ++i) {
        float ms = 0;
        check(nsh_event_sync(_ev[i].second), "hip::fir_filter_cascade_ccf timing");
        check(nsh_event_elapsed_ms(_ev[i].first, _ev[i].second, &ms), "hip::fir_filter_cascade_ccf timing");
        total += ms;
    }
    return total;
}

// ---- FFT ---------------------------------------------------------------------------
fft_vcc::fft_vcc(size_t fft_size, bool forward) : sync_block(forward ? "fft_vcc (hip)" : "ifft_vcc (hip)"), _forward(forward)
{
    if (fft_size != 1024) throw std::invalid_argument("hip::fft_vcc: only 1024-point transforms are implemented");
}

work_return_code_t fft_vcc::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    check(nsh_fft1024_c2c((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(), out[0].n_items,
                          _forward ? 0 : 1, current_stream()),
          "hip::fft_vcc");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

channelizer_vcc::channelizer_vcc(const std::vector<gr_complex>& w) : sync_block("channelizer_vcc (hip)"), _w(w)
{
    if (w.size() != 1024) throw std::invalid_argument("hip::channelizer_vcc: w must have 1024 bins");
}
channelizer_vcc::~channelizer_vcc()
{
    if (_wdev) nsh_free(_wdev);
}
bool channelizer_vcc::start()
{
    if (!_wdev) {
        check(nsh_malloc(current_device(), _w.size() * sizeof(gr_complex), &_wdev), "hip::channelizer_vcc");
        check(nsh_memcpy_async(_wdev, _w.data(), _w.size() * sizeof(gr_complex), NSH_H2D, current_stream()),
              "hip::channelizer_vcc");
        check(nsh_stream_sync(current_stream()), "hip::channelizer_vcc");
    }
    return sync_block::start();
}
work_return_code_t channelizer_vcc::work(std::vector<block_work_input>& in, std::vector<block_work_output>& out)
{
    check(nsh_channelizer1024((const float*)in[0].buffer->read_ptr(), (float*)out[0].buffer->write_ptr(),
                              (const float*)_wdev, out[0].n_items, current_stream()),
          "hip::channelizer_vcc");
    out[0].n_produced = out[0].n_items;
    return work_return_code_t::WORK_OK;
}

// ---- synthetic source ----------------------------------------------------------------
work_return_code_t synth_source::work(std::vector<block_work_input>&, std::vector<block_work_output>& out)
{
    int64_t n = (int64_t)out[0].n_items * (int64_t)_vlen; // samples
    if (_limit) {
        const uint64_t left = _first + _limit - _index;
        if (left == 0) {
            out[0].n_produced = 0;
            return work_return_code_t::WORK_DONE;
        }
        n = std::min<int64_t>(n, (int64_t)left);
    }
    check(nsh_synth_cf32((float*)out[0].buffer->write_ptr(), n, _index, _seed, current_stream()), "hip::synth_source");
    _index += (uint64_t)n;
    out[0].n_produced = (int)(n / (int64_t)_vlen);
    if (_limit && _index >= _first + _limit) return work_return_code_t::WORK_DONE;
    return work_return_code_t::WORK_OK;
}

} // namespace hip
} // namespace gr
