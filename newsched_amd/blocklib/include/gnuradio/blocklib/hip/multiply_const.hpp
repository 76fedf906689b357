// gr::hip::multiply_const<T> for gr_complex (cc) and float (ff): out = k * in on the
// device (replaces cuda::multiply_const, reference blocklib/cuda/include/gnuradio/
// blocklib/cuda/multiply_const.hpp:8-45 + lib/multiply_const.cu:1-18 -- float only, and
// its make() never stores k, Appendix A). Same per-product rounding as the CPU block.
#pragma once
#include <gnuradio/hip_fusion.hpp>
#include <gnuradio/sync_block.hpp>
#include <type_traits>

namespace gr {
namespace hip {
template <class T>
class multiply_const : public sync_block, public elementwise_cc
{
public:
    using sptr = std::shared_ptr<multiply_const>;
    static sptr make(const T k, const size_t vlen = 1)
    {
        auto p = std::make_shared<multiply_const>(k, vlen);
        p->add_port(port<T>::make("input", port_direction_t::INPUT, std::vector<size_t>{ vlen }));
        p->add_port(port<T>::make("output", port_direction_t::OUTPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    multiply_const(T k, size_t vlen) : sync_block("multiply_const (hip)"), d_k(k), d_vlen(vlen) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    T k() const { return d_k; }
    bool elementwise_stages(std::vector<gr_complex>& ks) const override
    {
        if constexpr (std::is_same_v<T, gr_complex>) {
            ks.push_back(d_k);
            return true;
        } else {
            return false;
        }
    }

private:
    T d_k;
    size_t d_vlen;
};
using multiply_const_cc = multiply_const<gr_complex>;
using multiply_const_ff = multiply_const<float>;

// Fused chain of multiply_const_cc stages in one pass over HBM (BASELINE config C2):
// identical results to the unfused chain (each stage's products rounded in order), 16 B
// per sample of traffic instead of 16 B per stage. scheduler_hip builds these itself from
// chains of separate elementwise blocks (hip_fusion.hpp); no stages = a copy.
class multiply_const_chain_cc : public sync_block, public elementwise_cc
{
public:
    using sptr = std::shared_ptr<multiply_const_chain_cc>;
    static sptr make(const std::vector<gr_complex>& ks, size_t vlen = 1)
    {
        auto p = std::make_shared<multiply_const_chain_cc>(ks, vlen);
        p->add_port(port<gr_complex>::make("input", port_direction_t::INPUT, std::vector<size_t>{ vlen }));
        p->add_port(port<gr_complex>::make("output", port_direction_t::OUTPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    multiply_const_chain_cc(const std::vector<gr_complex>& ks, size_t vlen)
        : sync_block("multiply_const_chain (hip)"), d_ks(ks), d_vlen(vlen)
    {
    }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    const std::vector<gr_complex>& ks() const { return d_ks; }
    bool elementwise_stages(std::vector<gr_complex>& ks) const override
    {
        ks.insert(ks.end(), d_ks.begin(), d_ks.end());
        return true;
    }

private:
    std::vector<gr_complex> d_ks;
    size_t d_vlen;
};

// y[i][j] = x[i][j] * k[j] on items of vlen = k.size() complex samples (GNU Radio's
// multiply_const_vcc; the reference has only the scalar multiply_const<T>). Not an
// elementwise_cc stage (its constant depends on the position in the item); scheduler_hip
// fuses fft_vcc -> multiply_const_vcc -> fft_vcc(inverse) into one channelizer_vcc launch.
class multiply_const_vcc : public sync_block
{
public:
    using sptr = std::shared_ptr<multiply_const_vcc>;
    static sptr make(const std::vector<gr_complex>& k)
    {
        auto p = std::make_shared<multiply_const_vcc>(k);
        p->add_port(port<gr_complex>::make("input", port_direction_t::INPUT, std::vector<size_t>{ k.size() }));
        p->add_port(port<gr_complex>::make("output", port_direction_t::OUTPUT, std::vector<size_t>{ k.size() }));
        return p;
    }
    explicit multiply_const_vcc(const std::vector<gr_complex>& k);
    ~multiply_const_vcc() override;
    bool start() override;
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    const std::vector<gr_complex>& k() const { return d_k; }

private:
    std::vector<gr_complex> d_k;
    void* d_kdev = nullptr;
};
} // namespace hip
} // namespace gr
