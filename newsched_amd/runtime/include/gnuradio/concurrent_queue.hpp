// Blocking multi-producer / single-consumer queue (reference
// runtime/include/gnuradio/concurrent_queue.hpp:16-61). notify_one: there is exactly one
// consumer per queue.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>

namespace gr {
template <typename T>
class concurrent_queue
{
public:
    bool push(const T& v)
    {
        {
            std::lock_guard<std::mutex> g(_m);
            _q.push_back(v);
            _n.store(_q.size(), std::memory_order_release);
        }
        _cv.notify_one();
        return true;
    }
    bool try_pop(T& out)
    {
        std::lock_guard<std::mutex> g(_m);
        if (_q.empty()) return false;
        out = std::move(_q.front());
        _q.pop_front();
        _n.store(_q.size(), std::memory_order_release);
        return true;
    }
    // Blocking pop. The consumer first spins for up to spin_us microseconds on an atomic count
    // (a message typically follows within tens of microseconds -- the next notification of a
    // running flowgraph), then sleeps on the condition variable: a futex wake-up costs several
    // microseconds on every hand-off between the scheduler threads.
    bool pop(T& out, int spin_us = 0)
    {
        if (spin_us > 0 && _n.load(std::memory_order_acquire) == 0) {
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
            while (_n.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
                __builtin_ia32_pause();
        }
        std::unique_lock<std::mutex> l(_m);
        _cv.wait(l, [this] { return !_q.empty(); });
        out = std::move(_q.front());
        _q.pop_front();
        _n.store(_q.size(), std::memory_order_release);
        return true;
    }
    template <class Rep, class Per>
    bool pop_for(T& out, std::chrono::duration<Rep, Per> d)
    {
        std::unique_lock<std::mutex> l(_m);
        if (!_cv.wait_for(l, d, [this] { return !_q.empty(); })) return false;
        out = std::move(_q.front());
        _q.pop_front();
        _n.store(_q.size(), std::memory_order_release);
        return true;
    }
    void clear()
    {
        std::lock_guard<std::mutex> g(_m);
        _q.clear();
        _n.store(0, std::memory_order_release);
    }
    size_t size()
    {
        std::lock_guard<std::mutex> g(_m);
        return _q.size();
    }

private:
    std::atomic<size_t> _n{ 0 };
    std::deque<T> _q;
    std::mutex _m;
    std::condition_variable _cv;
};
} // namespace gr
