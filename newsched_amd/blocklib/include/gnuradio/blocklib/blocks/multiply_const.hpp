// blocks::multiply_const<T> (reference blocklib/blocks/include/gnuradio/blocklib/blocks/
// multiply_const.hpp:8-43, blocklib/blocks/lib/multiply_const.cpp:17-86). The complex
// product rounds each partial product (std::complex<float> / VOLK generic formula); the
// CPU path is the baseline and the parity partner of gr::hip::multiply_const_cc.
#pragma once
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace blocks {
template <class T>
class multiply_const : public sync_block
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
    multiply_const(T k, size_t vlen) : sync_block("multiply_const"), d_k(k), d_vlen(vlen) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;
    T k() const { return d_k; }

private:
    T d_k;
    size_t d_vlen;
};
using multiply_const_ss = multiply_const<int16_t>;
using multiply_const_ii = multiply_const<int32_t>;
using multiply_const_ff = multiply_const<float>;
using multiply_const_cc = multiply_const<gr_complex>;
} // namespace blocks
} // namespace gr
