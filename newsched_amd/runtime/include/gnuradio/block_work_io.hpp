// work() argument structs and return codes (reference
// runtime/include/gnuradio/block_work_io.hpp:15-54).
#pragma once
#include <gnuradio/buffer.hpp>

namespace gr {

struct block_work_input {
    int n_items;          // items readable
    buffer_sptr buffer;
    int n_consumed;       // set by the block (or sync_block::do_work)
    block_work_input(int n, buffer_sptr b) : n_items(n), buffer(std::move(b)), n_consumed(-1) {}
};

struct block_work_output {
    int n_items;          // items writable
    buffer_sptr buffer;
    int n_produced;       // set by the block
    block_work_output(int n, buffer_sptr b) : n_items(n), buffer(std::move(b)), n_produced(-1) {}
};

enum class work_return_code_t {
    WORK_ERROR = -100,
    WORK_INSUFFICIENT_OUTPUT_ITEMS = -3,
    WORK_INSUFFICIENT_INPUT_ITEMS = -2,
    WORK_DONE = -1,
    WORK_OK = 0,
};

} // namespace gr
