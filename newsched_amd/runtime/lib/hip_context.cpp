// Thread-local HIP stream binding for work() calls (see hip_context.hpp).
#include <gnuradio/hip_context.hpp>

#include "nsh_hip.h"

namespace gr {
namespace hip {

namespace {
struct thread_ctx {
    int device = 0;
    void* stream = nullptr;
    bool owned = false;
    ~thread_ctx()
    {
        if (owned && stream) {
            nsh_stream_sync(stream);
            nsh_stream_destroy(stream);
        }
    }
};
thread_local thread_ctx t_ctx;
} // namespace

void check(int rc, const char* what)
{
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + nsh_last_error());
}

void* current_stream()
{
    if (!t_ctx.stream) {
        check(nsh_set_device(t_ctx.device), "hip::current_stream set_device");
        check(nsh_stream_create(t_ctx.device, &t_ctx.stream), "hip::current_stream");
        t_ctx.owned = true;
    }
    return t_ctx.stream;
}

int current_device() { return t_ctx.device; }

void bind_thread(int device, void* stream)
{
    if (t_ctx.owned && t_ctx.stream) {
        nsh_stream_sync(t_ctx.stream);
        nsh_stream_destroy(t_ctx.stream);
    }
    t_ctx.device = device;
    t_ctx.stream = stream;
    t_ctx.owned = false;
    check(nsh_set_device(device), "hip::bind_thread");
}

void unbind_thread()
{
    if (!t_ctx.owned) {
        t_ctx.stream = nullptr;
    }
}

bool thread_has_stream() { return t_ctx.stream != nullptr; }

void sync_thread_stream()
{
    if (t_ctx.stream) check(nsh_stream_sync(t_ctx.stream), "hip::sync_thread_stream");
}

} // namespace hip
} // namespace gr
