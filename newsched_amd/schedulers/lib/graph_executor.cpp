// One scheduling pass over a block group (reference schedulers/mt/lib/graph_executor.cpp).
#include <gnuradio/schedulers/mt/graph_executor.hpp>

#include <climits>
#include <stdexcept>

namespace gr {
namespace schedulers {

namespace {
void notify(const port_sptr& p, scheduler_action_t a, nodeid_t id)
{
    p->notify_connected_ports(std::make_shared<scheduler_action>(a, id));
}
} // namespace

bool graph_executor::all_finished(const std::vector<block_sptr>& blocks) const
{
    for (auto& b : blocks)
        if (!_finished.count(b->id())) return false;
    return true;
}

// Every step runs even if an earlier one throws (a failed cross-process edge throws from
// set_writer_done): an input left without its reader-done flag would hold the upstream block
// forever. The first error is rethrown at the end.
void graph_executor::finish(const block_sptr& b)
{
    if (!_finished.insert(b->id()).second) return;
    std::exception_ptr first;
    auto step = [&first](auto&& f) {
        try {
            f();
        } catch (...) {
            if (!first) first = std::current_exception();
        }
    };
    for (auto& p : b->output_stream_ports()) {
        for (auto& buf : _bufman->get_output_buffers(p)) step([&] { buf->set_writer_done(); });
        step([&] { notify(p, scheduler_action_t::NOTIFY_INPUT, b->id()); });
    }
    for (auto& p : b->input_stream_ports()) {
        step([&] { _bufman->get_input_buffer(p)->set_reader_done(); });
        step([&] { notify(p, scheduler_action_t::NOTIFY_OUTPUT, b->id()); });
    }
    if (first) std::rethrow_exception(first);
}

std::map<nodeid_t, executor_iteration_status> graph_executor::run_one_iteration(std::vector<block_sptr> blocks)
{
    using S = executor_iteration_status;
    std::map<nodeid_t, S> st;
    if (blocks.empty()) blocks = d_blocks;

    for (auto& b : blocks) { // group order (topological in the GPU domain)
        const nodeid_t id = b->id();
        if (_finished.count(id)) {
            st[id] = S::DONE;
            continue;
        }
        const auto in_ports = b->input_stream_ports();
        const auto out_ports = b->output_stream_ports();

        // ---- inputs --------------------------------------------------------------
        std::vector<block_work_input> win;
        win.reserve(in_ports.size());
        bool ready = true, exhausted = false;
        for (auto& p : in_ports) {
            auto buf = _bufman->get_input_buffer(p);
            buffer_info_t ri{};
            if (!buf->read_info(ri)) {
                ready = false;
                break;
            }
            if (ri.n_items < s_min_items_to_process) {
                ready = false;
                // writer finished and nothing left (re-read: the writer may have posted
                // its last items just before flagging done)
                if (buf->writer_done() && buf->read_info(ri) && ri.n_items < s_min_items_to_process) exhausted = true;
                break;
            }
            win.emplace_back(ri.n_items, buf);
        }
        if (exhausted) {
            finish(b);
            st[id] = S::DONE;
            continue;
        }
        if (!ready) {
            st[id] = S::BLKD_IN;
            continue;
        }

        // ---- outputs (fan-out: the primary buffer is handed to work(), the rest get
        //      copy_items; buffers whose reader has finished are skipped) ----------------
        bool all_readers_done = !out_ports.empty();
        for (auto& p : out_ports)
            for (auto& buf : _bufman->get_output_buffers(p))
                if (!buf->reader_done()) all_readers_done = false;
        if (all_readers_done) {
            finish(b);
            st[id] = S::DONE;
            continue;
        }
        std::vector<block_work_output> wout;
        std::vector<std::vector<buffer_sptr>> live(out_ports.size());
        wout.reserve(out_ports.size());
        for (size_t i = 0; i < out_ports.size() && ready; ++i) {
            int max_out = INT_MAX;
            for (auto& buf : _bufman->get_output_buffers(out_ports[i])) {
                if (buf->reader_done()) continue;
                buffer_info_t wi{};
                if (!buf->write_info(wi) || wi.n_items < s_min_buf_items) {
                    ready = false;
                    break;
                }
                max_out = std::min(max_out, wi.n_items);
                live[i].push_back(buf);
            }
            if (!ready) break;
            if (live[i].empty()) { // every reader of this port is gone: discard into the first
                live[i].push_back(_bufman->get_output_buffers(out_ports[i])[0]);
                buffer_info_t wi{};
                live[i][0]->write_info(wi);
                max_out = wi.n_items;
                if (max_out < s_min_buf_items) ready = false;
            }
            wout.emplace_back(max_out, live[i][0]);
        }
        if (!ready) {
            st[id] = S::BLKD_OUT;
            continue;
        }

        // ---- work ------------------------------------------------------------------
        work_return_code_t ret;
        while (true) {
            if (_hooks.before) _hooks.before(b);
            try {
                ret = b->do_work(win, wout);
            } catch (...) {
                if (_hooks.after) _hooks.after(b, -1);
                throw;
            }
            if (_hooks.after)
                _hooks.after(b, (ret == work_return_code_t::WORK_OK || ret == work_return_code_t::WORK_DONE) && !wout.empty()
                                    ? std::max(wout[0].n_produced, 0)
                                    : 0);
            if (ret == work_return_code_t::WORK_OK || ret == work_return_code_t::WORK_DONE) break;
            if (ret == work_return_code_t::WORK_INSUFFICIENT_INPUT_ITEMS) {
                if (wout.empty()) break;
                wout[0].n_items >>= 1; // ask for less output (reference :125-130)
                if (wout[0].n_items < 4) break;
                continue;
            }
            throw std::runtime_error("block " + b->alias() + " returned " +
                                     (ret == work_return_code_t::WORK_ERROR ? "WORK_ERROR" : "WORK_INSUFFICIENT_OUTPUT_ITEMS"));
        }

        if (ret == work_return_code_t::WORK_INSUFFICIENT_INPUT_ITEMS) {
            bool writers_done = !in_ports.empty();
            for (auto& p : in_ports)
                if (!_bufman->get_input_buffer(p)->writer_done()) writers_done = false;
            if (writers_done) { // end of stream: leftover input cannot form an output
                finish(b);
                st[id] = S::DONE;
            } else {
                st[id] = S::BLKD_IN;
            }
            continue;
        }

        // ---- advance buffers, propagate tags, wake neighbours --------------------------
        bool progress = false;
        for (size_t i = 0; i < in_ports.size(); ++i) {
            auto buf = win[i].buffer;
            const int consumed = std::max(win[i].n_consumed, 0);
            if (buf->has_tags()) {
                const auto pol = b->tag_propagation_policy();
                for (size_t o = 0; o < out_ports.size(); ++o)
                    if (pol == tag_propagation_policy_t::TPP_ALL_TO_ALL ||
                        (pol == tag_propagation_policy_t::TPP_ONE_TO_ONE && o == i))
                        for (auto& ob : _bufman->get_output_buffers(out_ports[o])) ob->propagate_tags(buf, consumed);
                buf->prune_tags(consumed);
            }
            if (consumed > 0) {
                buf->post_read(consumed);
                progress = true;
                notify(in_ports[i], scheduler_action_t::NOTIFY_OUTPUT, id);
            }
        }
        for (size_t i = 0; i < out_ports.size(); ++i) {
            const int produced = std::max(wout[i].n_produced, 0);
            if (produced <= 0) continue;
            for (size_t j = 1; j < live[i].size(); ++j) live[i][j]->copy_items(live[i][0], produced);
            for (auto& buf : live[i]) buf->post_write(produced);
            progress = true;
            notify(out_ports[i], scheduler_action_t::NOTIFY_INPUT, id);
        }
        if (ret == work_return_code_t::WORK_DONE) {
            finish(b);
            st[id] = S::DONE;
        } else {
            st[id] = progress ? S::READY : S::BLKD_IN;
        }
    }
    return st;
}

} // namespace schedulers
} // namespace gr
