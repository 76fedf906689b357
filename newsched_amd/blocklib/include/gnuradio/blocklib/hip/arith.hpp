// gr::hip::add_cc / multiply_cc: elementwise over 2 complex device streams.
#pragma once
#include <gnuradio/sync_block.hpp>

namespace gr {
namespace hip {
template <int OP> // 0 add, 1 multiply
class arith_cc : public sync_block
{
public:
    using sptr = std::shared_ptr<arith_cc>;
    static sptr make(size_t nports = 2, size_t vlen = 1)
    {
        auto p = std::make_shared<arith_cc>(nports, vlen);
        for (size_t i = 0; i < nports; ++i)
            p->add_port(port<gr_complex>::make("in" + std::to_string(i), port_direction_t::INPUT, std::vector<size_t>{ vlen }));
        p->add_port(port<gr_complex>::make("out", port_direction_t::OUTPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    arith_cc(size_t nports, size_t vlen) : sync_block(OP == 0 ? "add_cc (hip)" : "multiply_cc (hip)"), _nports(nports), _vlen(vlen)
    {
        if (nports < 1) throw std::invalid_argument("arith_cc: need at least one input");
    }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override;

private:
    size_t _nports, _vlen;
};
using add_cc = arith_cc<0>;
using multiply_cc = arith_cc<1>;
} // namespace hip
} // namespace gr
