// One block-group thread (reference schedulers/mt/include/gnuradio/schedulers/mt/
// thread_wrapper.hpp, schedulers/mt/lib/thread_wrapper.cpp:9-191). Persistent across
// runs: NOTIFY_ALL starts a run (re-arming per-run state on this thread), the thread
// iterates its blocks while notifications arrive or progress is made, and when all its
// blocks have finished it runs its flush hook (HIP stream drain) and reports to its
// scheduler. EXIT ends the thread.
#pragma once
#include <atomic>
#include <functional>
#include <gnuradio/concurrent_queue.hpp>
#include <gnuradio/flowgraph_monitor.hpp>
#include <gnuradio/neighbor_interface.hpp>
#include <gnuradio/schedulers/mt/block_group_properties.hpp>
#include <gnuradio/schedulers/mt/graph_executor.hpp>
#include <thread>

namespace gr {
namespace schedulers {

struct thread_hooks {
    std::function<void()> on_thread_start; // e.g. bind device + partition stream
    std::function<void()> on_flush;        // e.g. drain the partition stream
    int queue_spin_us = 0;                 // spin this long on an empty queue before sleeping
    work_hooks on_work;                    // around every do_work() call (e.g. kernel timing)
};

class thread_wrapper : public neighbor_interface, public std::enable_shared_from_this<thread_wrapper>
{
public:
    using sptr = std::shared_ptr<thread_wrapper>;
    using finished_cb = std::function<void(int thread_index)>;

    static sptr make(int id, block_group_properties bgp, buffer_manager::sptr bufman, flowgraph_monitor_sptr fgmon,
                     thread_hooks hooks = {}, finished_cb on_finished = nullptr, int thread_index = 0)
    {
        return std::make_shared<thread_wrapper>(id, bgp, bufman, fgmon, hooks, on_finished, thread_index);
    }
    thread_wrapper(int id, block_group_properties bgp, buffer_manager::sptr bufman, flowgraph_monitor_sptr fgmon,
                   thread_hooks hooks, finished_cb on_finished, int thread_index);
    ~thread_wrapper() override;

    int id() const { return _id; }
    const std::string& name() const { return d_block_group.name(); }
    void push_message(scheduler_message_sptr msg) override { msgq.push(msg); }

    void start(); // begin a run
    void stop();  // end the thread (joins)
    void wait() {}

private:
    static void thread_body(thread_wrapper* top);
    bool handle_work_notification();

    concurrent_queue<scheduler_message_sptr> msgq;
    std::thread d_thread;
    std::atomic<bool> d_thread_stopped{ false };
    std::unique_ptr<graph_executor> _exec;
    block_group_properties d_block_group;
    std::vector<block_sptr> d_blocks;
    flowgraph_monitor_sptr d_fgmon;
    thread_hooks _hooks;
    finished_cb _on_finished;
    int _id;
    int _thread_index;
    bool _run_active = false;
    bool _started = false;
};

} // namespace schedulers
} // namespace gr
