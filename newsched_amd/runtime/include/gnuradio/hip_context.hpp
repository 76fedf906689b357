// Per-thread HIP execution context for work() calls.
//
// Every gr::hip block launches on hip::current_stream(). The GPU scheduler domain
// (gr::schedulers::scheduler_hip) binds one stream for its whole partition before its
// thread runs any block, so all kernels of a partition are stream-ordered and no work()
// ever synchronises (the reference syncs every work() and post_write: blocklib/cuda/lib/
// copy.cpp:58, runtime/lib/cudabuffer.cu:175). A hip block placed on an ordinary
// scheduler_mt thread gets a private stream created on first use, synchronised when that
// thread flushes.
#pragma once
#include <stdexcept>
#include <string>

namespace gr {
namespace hip {

void* current_stream();          // never null; creates the thread's stream on first use
int current_device();
void bind_thread(int device, void* stream); // stream owned by the caller
void unbind_thread();
bool thread_has_stream();
void sync_thread_stream();       // drain this thread's stream, if it has one

// Throw std::runtime_error("<what>: <nsh_last_error()>") when rc != 0.
void check(int rc, const char* what);

} // namespace hip
} // namespace gr
