// blocks::vector_source<T> (reference blocklib/blocks/include/gnuradio/blocklib/blocks/
// vector_source.hpp, blocklib/blocks/lib/vector_source.cpp:38-82): emits `data` once
// (then WORK_DONE) or repeatedly; vlen items. The offset re-arms in start().
#pragma once
#include <algorithm>
#include <cstring>
#include <gnuradio/sync_block.hpp>
#include <stdexcept>

namespace gr {
namespace blocks {
template <class T>
class vector_source : public sync_block
{
public:
    using sptr = std::shared_ptr<vector_source>;
    static sptr make(const std::vector<T>& data, bool repeat = false, unsigned int vlen = 1,
                     const std::vector<tag_t>& tags = {})
    {
        auto p = std::make_shared<vector_source>(data, repeat, vlen, tags);
        p->add_port(port<T>::make("output", port_direction_t::OUTPUT, std::vector<size_t>{ vlen }));
        return p;
    }
    vector_source(const std::vector<T>& data, bool repeat, unsigned int vlen, const std::vector<tag_t>& tags)
        : sync_block("vector_source"), d_data(data), d_repeat(repeat), d_vlen(vlen), d_tags(tags)
    {
        if (vlen == 0 || data.size() % vlen != 0) throw std::invalid_argument("data length must be a multiple of vlen");
    }
    bool start() override
    {
        d_offset = 0;
        return sync_block::start();
    }
    work_return_code_t work(std::vector<block_work_input>&, std::vector<block_work_output>& out) override
    {
        T* optr = static_cast<T*>(out[0].buffer->write_ptr());
        const size_t want = (size_t)out[0].n_items * d_vlen;
        if (d_repeat) {
            if (d_data.empty()) return work_return_code_t::WORK_DONE;
            size_t done = 0;
            while (done < want) {
                const size_t n = std::min(want - done, d_data.size() - d_offset);
                std::memcpy(optr + done, d_data.data() + d_offset, n * sizeof(T));
                done += n;
                d_offset = (d_offset + n) % d_data.size();
            }
            out[0].n_produced = out[0].n_items;
            return work_return_code_t::WORK_OK;
        }
        if (d_offset >= d_data.size()) {
            out[0].n_produced = 0;
            return work_return_code_t::WORK_DONE;
        }
        const size_t n = std::min(d_data.size() - d_offset, want);
        std::memcpy(optr, d_data.data() + d_offset, n * sizeof(T));
        d_offset += n;
        out[0].n_produced = (int)(n / d_vlen);
        return work_return_code_t::WORK_OK;
    }

private:
    std::vector<T> d_data;
    bool d_repeat;
    size_t d_offset = 0;
    size_t d_vlen;
    std::vector<tag_t> d_tags;
};
using vector_source_b = vector_source<uint8_t>;
using vector_source_s = vector_source<int16_t>;
using vector_source_i = vector_source<int32_t>;
using vector_source_f = vector_source<float>;
using vector_source_c = vector_source<gr_complex>;
} // namespace blocks
} // namespace gr
