// Stream tags (reference runtime/include/gnuradio/tag.hpp:8-41): absolute item offset plus
// key/value/srcid payloads. Host-side only; hip_buffer keeps _total_read/_total_written
// exact so offsets stay meaningful across device edges.
#pragma once
#include <cstdint>
#include <gnuradio/pmtf.hpp>

namespace gr {

enum class tag_propagation_policy_t {
    TPP_DONT = 0,       // scheduler does not propagate
    TPP_ALL_TO_ALL = 1, // every input's tags go to every output
    TPP_ONE_TO_ONE = 2, // input n -> output n
    TPP_CUSTOM = 3      // block does it itself
};

class tag_t
{
public:
    uint64_t offset;
    pmtf::pmt_sptr key;
    pmtf::pmt_sptr value;
    pmtf::pmt_sptr srcid;
    tag_t(uint64_t offset_, pmtf::pmt_sptr key_, pmtf::pmt_sptr value_, pmtf::pmt_sptr srcid_ = nullptr)
        : offset(offset_), key(std::move(key_)), value(std::move(value_)), srcid(std::move(srcid_))
    {
    }
    bool operator==(const tag_t& o) const { return offset == o.offset && key == o.key && value == o.value && srcid == o.srcid; }
    bool operator!=(const tag_t& o) const { return !(*this == o); }
};

} // namespace gr
