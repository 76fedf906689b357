// Anything that accepts scheduler messages: a block-group thread, a scheduler
// (reference runtime/include/gnuradio/neighbor_interface.hpp).
#pragma once
#include <gnuradio/scheduler_message.hpp>

namespace gr {
struct neighbor_interface {
    virtual ~neighbor_interface() = default;
    virtual void push_message(scheduler_message_sptr msg) = 0;
};
using neighbor_interface_sptr = std::shared_ptr<neighbor_interface>;
} // namespace gr
