// Run-completion tracker (reference runtime/include/gnuradio/flowgraph_monitor.hpp,
// runtime/lib/flowgraph_monitor.cpp).
//
// The reference monitor reacts to the first DONE by sleeping 100 ms and then telling
// every thread to report FLUSHED, without draining in-flight data (:27-31). Here every
// block-group thread drains: a block finishes when it returns WORK_DONE, when an input's
// writer has finished and the input is empty, or when every reader of its outputs has
// finished; a thread whose blocks are all finished synchronises its HIP stream and
// reports to its scheduler, which sends FLUSHED here once all its threads have. wait()
// returns when every scheduler has flushed -- no fixed sleep anywhere.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace gr {

enum class fg_monitor_message_t { UNKNOWN, DONE, FLUSHED, KILL };

class fg_monitor_message
{
public:
    fg_monitor_message(fg_monitor_message_t t = fg_monitor_message_t::UNKNOWN, int64_t schedid = -1, int64_t blkid = -1)
        : _type(t), _blkid(blkid), _schedid(schedid)
    {
    }
    fg_monitor_message_t type() const { return _type; }
    int64_t schedid() const { return _schedid; }
    int64_t blkid() const { return _blkid; }

private:
    fg_monitor_message_t _type;
    int64_t _blkid;
    int64_t _schedid;
};

class scheduler;

class flowgraph_monitor
{
public:
    explicit flowgraph_monitor(std::vector<std::shared_ptr<scheduler>>& scheds) : d_schedulers(scheds) {}
    // drop the scheduler references (schedulers hold the monitor: break the cycle)
    void release()
    {
        std::lock_guard<std::mutex> g(_m);
        d_schedulers.clear();
    }
    virtual ~flowgraph_monitor() = default;

    virtual void push_message(fg_monitor_message msg);
    void start();                                    // arm for a new run
    void stop() { push_message(fg_monitor_message(fg_monitor_message_t::KILL, 0, 0)); }
    void wait();                                     // block until all flushed (or killed)
    // wait() first polls for this long (us) before sleeping: the caller's thread is idle
    // anyway, and a futex wake-up after the last scheduler flushed costs several us per run
    void set_wait_spin_us(int us) { _wait_spin_us = us; }
    bool run_complete();
    void report_error(std::exception_ptr e);         // a worker thread failed
    std::exception_ptr error();
    uint64_t done_blocks();                          // WORK_DONE reports this run
    bool replace_scheduler(std::shared_ptr<scheduler> original,
                           const std::vector<std::shared_ptr<scheduler>> replacements);

private:
    std::vector<std::shared_ptr<scheduler>> d_schedulers;
    std::mutex _m;
    std::condition_variable _cv;
    std::map<int64_t, bool> _flushed;
    bool _killed = false;
    std::atomic<bool> _complete{ false };
    int _wait_spin_us = 0;
    uint64_t _done_blocks = 0;
    std::exception_ptr _error;
};

using flowgraph_monitor_sptr = std::shared_ptr<flowgraph_monitor>;

} // namespace gr
