// Probe builds only (-DNSR_RUN_TRACE=1, tools/probe/run_trace.py): steady-clock stamps at fixed
// points of one flowgraph run, to split a run's host overhead. Compiled out otherwise.
#pragma once
#if NSR_RUN_TRACE
#include <atomic>
#include <chrono>
#include <cstdint>
namespace gr {
inline std::atomic<int64_t> g_run_trace[16];
inline void run_trace(int k)
{
    g_run_trace[k].store(std::chrono::duration_cast<std::chrono::nanoseconds>(
                             std::chrono::steady_clock::now().time_since_epoch()).count(),
                         std::memory_order_relaxed);
}
} // namespace gr
#define NSR_RT(k) ::gr::run_trace(k)
#else
#define NSR_RT(k) ((void)0)
#endif
