// Blocking multi-producer / single-consumer queue (reference
// runtime/include/gnuradio/concurrent_queue.hpp:16-61). notify_one: there is exactly one
// consumer per queue.
#pragma once
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
        return true;
    }
    bool pop(T& out)
    {
        std::unique_lock<std::mutex> l(_m);
        _cv.wait(l, [this] { return !_q.empty(); });
        out = std::move(_q.front());
        _q.pop_front();
        return true;
    }
    template <class Rep, class Per>
    bool pop_for(T& out, std::chrono::duration<Rep, Per> d)
    {
        std::unique_lock<std::mutex> l(_m);
        if (!_cv.wait_for(l, d, [this] { return !_q.empty(); })) return false;
        out = std::move(_q.front());
        _q.pop_front();
        return true;
    }
    void clear()
    {
        std::lock_guard<std::mutex> g(_m);
        _q.clear();
    }
    size_t size()
    {
        std::lock_guard<std::mutex> g(_m);
        return _q.size();
    }

private:
    std::deque<T> _q;
    std::mutex _m;
    std::condition_variable _cv;
};
} // namespace gr
