// blocks::vector_sink<T> (reference blocklib/blocks/include/gnuradio/blocklib/blocks/
// vector_sink.hpp, blocklib/blocks/lib/vector_sink.cpp:28-40): appends everything it
// reads; data() returns it. Cleared when a run starts.
#pragma once
#include <gnuradio/sync_block.hpp>
#include <mutex>

namespace gr {
namespace blocks {
template <class T>
class vector_sink : public sync_block
{
public:
    using sptr = std::shared_ptr<vector_sink>;
    static sptr make(const size_t vlen = 1, const size_t reserve_items = 1024)
    {
        auto p = std::make_shared<vector_sink>(vlen, reserve_items);
        p->add_port(port<T>::make("input", port_direction_t::INPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    explicit vector_sink(const size_t vlen = 1, const size_t reserve_items = 1024) : sync_block("vector_sink"), d_vlen(vlen)
    {
        d_data.reserve(vlen * reserve_items);
    }
    bool start() override
    {
        std::lock_guard<std::mutex> g(_m);
        d_data.clear();
        return sync_block::start();
    }
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>&) override
    {
        const T* iptr = static_cast<const T*>(in[0].buffer->read_ptr());
        std::lock_guard<std::mutex> g(_m);
        d_data.insert(d_data.end(), iptr, iptr + (size_t)in[0].n_items * d_vlen);
        in[0].n_consumed = in[0].n_items;
        return work_return_code_t::WORK_OK;
    }
    std::vector<T> data()
    {
        std::lock_guard<std::mutex> g(_m);
        return d_data;
    }

private:
    std::mutex _m;
    std::vector<T> d_data;
    size_t d_vlen;
};
using vector_sink_b = vector_sink<uint8_t>;
using vector_sink_s = vector_sink<int16_t>;
using vector_sink_i = vector_sink<int32_t>;
using vector_sink_f = vector_sink<float>;
using vector_sink_c = vector_sink<gr_complex>;
} // namespace blocks
} // namespace gr
