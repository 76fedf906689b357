// A set of blocks run by one thread (reference schedulers/mt/include/gnuradio/schedulers/
// mt/block_group_properties.hpp:8-61).
#pragma once
#include <gnuradio/block.hpp>
#include <vector>

namespace gr {
namespace schedulers {

class block_group_properties
{
public:
    block_group_properties(const std::vector<block_sptr>& blocks, const std::string& name = "",
                           const std::vector<unsigned int>& affinity_mask = {})
        : _blocks(blocks), _name(name), _affinity_mask(affinity_mask)
    {
        if (_name.empty() && !_blocks.empty()) _name = _blocks[0]->name();
    }
    void set_processor_affinity(const std::vector<unsigned int>& mask) { _affinity_mask = mask; }
    void unset_processor_affinity() { _affinity_mask.clear(); }
    std::vector<unsigned int> processor_affinity() const { return _affinity_mask; }
    std::vector<block_sptr>& blocks() { return _blocks; }
    const std::string& name() const { return _name; }

private:
    std::vector<block_sptr> _blocks;
    std::string _name;
    std::vector<unsigned int> _affinity_mask;
};

} // namespace schedulers
} // namespace gr
