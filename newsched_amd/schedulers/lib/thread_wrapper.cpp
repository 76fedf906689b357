// Block-group thread (reference schedulers/mt/lib/thread_wrapper.cpp:9-191).
#include <gnuradio/run_trace.hpp>
#include <gnuradio/schedulers/mt/thread_wrapper.hpp>

#include <pthread.h>
#include <sched.h>

namespace gr {
namespace schedulers {

thread_wrapper::thread_wrapper(int id, block_group_properties bgp, buffer_manager::sptr bufman,
                               flowgraph_monitor_sptr fgmon, thread_hooks hooks, finished_cb on_finished,
                               int thread_index)
    : d_block_group(bgp), d_blocks(bgp.blocks()), d_fgmon(std::move(fgmon)), _hooks(std::move(hooks)),
      _on_finished(std::move(on_finished)), _id(id), _thread_index(thread_index)
{
    _exec = std::make_unique<graph_executor>(bgp.name());
    _exec->initialize(std::move(bufman), d_blocks, _hooks.on_work);
    d_thread = std::thread(thread_body, this);
}

thread_wrapper::~thread_wrapper()
{
    if (d_thread.joinable()) {
        d_thread_stopped = true;
        push_message(std::make_shared<scheduler_action>(scheduler_action_t::EXIT, 0));
        d_thread.join();
    }
}

void thread_wrapper::start() { push_message(std::make_shared<scheduler_action>(scheduler_action_t::NOTIFY_ALL, 0)); }

void thread_wrapper::stop()
{
    if (!d_thread.joinable()) return;
    push_message(std::make_shared<scheduler_action>(scheduler_action_t::EXIT, 0));
    d_thread.join();
    for (auto& b : d_blocks) b->stop();
}

bool thread_wrapper::handle_work_notification()
{
    auto s = _exec->run_one_iteration(d_blocks);
    bool ready = false;
    for (auto& kv : s) {
        if (kv.second == executor_iteration_status::DONE) continue;
        if (kv.second == executor_iteration_status::READY) ready = true;
    }
    if (_run_active && _exec->all_finished(d_blocks)) {
        NSR_RT(6);
        if (_hooks.on_flush) _hooks.on_flush(); // drain this partition's HIP stream
        NSR_RT(7);
        _run_active = false;
        for (auto& b : d_blocks) d_fgmon->push_message(fg_monitor_message(fg_monitor_message_t::DONE, _id, b->id()));
        if (_on_finished) _on_finished(_thread_index);
        return false;
    }
    return ready;
}

void thread_wrapper::thread_body(thread_wrapper* top)
{
    const std::string tname = (top->d_block_group.name() + std::to_string(top->d_blocks.empty() ? 0 : top->d_blocks[0]->id())).substr(0, 15);
    pthread_setname_np(pthread_self(), tname.c_str());
    if (!top->d_block_group.processor_affinity().empty()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (unsigned c : top->d_block_group.processor_affinity()) CPU_SET(c, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    try {
        if (top->_hooks.on_thread_start) top->_hooks.on_thread_start();
    } catch (...) {
        top->d_fgmon->report_error(std::current_exception());
    }

    bool blocking = true;
    while (!top->d_thread_stopped) {
        scheduler_message_sptr msg;
        bool do_work = false;
        bool got = blocking ? top->msgq.pop(msg, top->_hooks.queue_spin_us) : top->msgq.try_pop(msg);
        while (got) {
            if (msg->type() == scheduler_message_t::SCHEDULER_ACTION) {
                switch (std::static_pointer_cast<scheduler_action>(msg)->action()) {
                case scheduler_action_t::NOTIFY_ALL: // a run starts: re-arm on this thread
                    NSR_RT(2);
                    top->_exec->reset_run_state();
                    for (auto& b : top->d_blocks) b->start();
                    NSR_RT(3);
                    top->_run_active = true;
                    do_work = true;
                    break;
                case scheduler_action_t::NOTIFY_INPUT:
                case scheduler_action_t::NOTIFY_OUTPUT:
                    do_work = true;
                    break;
                case scheduler_action_t::DONE: // external request to wind down
                    do_work = true;
                    break;
                case scheduler_action_t::EXIT:
                    top->d_thread_stopped = true;
                    break;
                }
            } else if (msg->type() == scheduler_message_t::MSGPORT_MESSAGE) {
                auto m = std::static_pointer_cast<msgport_message>(msg);
                if (m->callback()) m->callback()(m->message());
            }
            got = top->msgq.try_pop(msg);
        }
        if (top->d_thread_stopped) break;

        bool ready = false;
        if (do_work || !blocking) {
            if (top->_run_active) {
                try {
                    ready = top->handle_work_notification();
                } catch (...) {
                    top->d_fgmon->report_error(std::current_exception());
                    // finish everything so neighbours drain and the run completes
                    top->_exec->finish_all();
                    top->_run_active = false;
                    try {
                        if (top->_hooks.on_flush) top->_hooks.on_flush();
                    } catch (...) {
                    }
                    if (top->_on_finished) top->_on_finished(top->_thread_index);
                    ready = false;
                }
            }
        }
        blocking = !ready;
    }
}

} // namespace schedulers
} // namespace gr
