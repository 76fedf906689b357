// GPU scheduler domain (see scheduler_hip.hpp).
#include <chrono>
#include <gnuradio/hip_context.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>

#include "nsh_hip.h"

namespace gr {
namespace schedulers {

scheduler_hip::scheduler_hip(const std::string name, int device, size_t fixed_buf_size)
    : scheduler_mt(name, fixed_buf_size), _device(device)
{
    hip::check(nsh_stream_create(device, &_stream), "scheduler_hip: stream");
    _default_buf_factory = hip_buffer::make;
    _default_buf_properties = hip_buffer_properties::make(hip_buffer_type::D2D, device);
}

scheduler_hip::~scheduler_hip()
{
    for (auto& t : _threads) t->stop(); // threads use the stream: stop them first
    _threads.clear();
    release_fused();
    if (_stream) {
        nsh_stream_sync(_stream);
        nsh_stream_destroy(_stream);
    }
}

void scheduler_hip::release_fused()
{
    // fused blocks are owned here; their ports point at this scheduler's threads
    for (auto& f : _plan.fused)
        for (auto& p : f->all_ports()) p->set_parent_intf(nullptr);
    _plan.undo(); // the user's blocks get their original port links back
    _plan = hip::fusion_result();
}

void scheduler_hip::initialize(flat_graph_sptr fg, flowgraph_monitor_sptr fgmon, neighbor_interface_map nbr)
{
    for (auto& t : _threads) t->stop();
    _threads.clear();
    release_fused();
    if (_fusion) {
        _plan = hip::fuse_elementwise_cc(fg);
        auto ch = hip::fuse_channelizer(_plan.graph);
        _plan.graph = ch.graph;
        _plan.fused.insert(_plan.fused.end(), ch.fused.begin(), ch.fused.end());
        _plan.chains.insert(_plan.chains.end(), ch.chains.begin(), ch.chains.end());
        _plan.cut.insert(_plan.cut.end(), ch.cut.begin(), ch.cut.end());
        _plan.added.insert(_plan.added.end(), ch.added.begin(), ch.added.end());
        if (_fir_fusion) {
            auto fc = hip::fuse_fir_cascade(_plan.graph);
            _plan.graph = fc.graph;
            _plan.fused.insert(_plan.fused.end(), fc.fused.begin(), fc.fused.end());
            _plan.chains.insert(_plan.chains.end(), fc.chains.begin(), fc.chains.end());
            _plan.cut.insert(_plan.cut.end(), fc.cut.begin(), fc.cut.end());
            _plan.added.insert(_plan.added.end(), fc.added.begin(), fc.added.end());
        }
        fg = _plan.graph;
    }
    scheduler_mt::initialize(fg, fgmon, nbr);
}

std::vector<block_group_properties> scheduler_hip::plan_groups(flat_graph_sptr fg)
{
    // The whole partition is one group, producers first.
    auto order = fg->topological_sort(fg->calc_used_blocks());
    if (order.empty()) return {};
    return { block_group_properties(order, name()) };
}

thread_hooks scheduler_hip::hooks_for_group(const block_group_properties&)
{
    thread_hooks h;
    const int dev = _device;
    void* s = _stream;
    h.on_thread_start = [dev, s] { hip::bind_thread(dev, s); };
    const int spin_us = _flush_spin_us;
    h.on_flush = [s, spin_us] {
        if (spin_us > 0) {
            const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
            int q;
            while ((q = nsh_stream_query(s)) == 1 && std::chrono::steady_clock::now() < until)
                for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
            hip::check(q < 0 ? q : 0, "scheduler_hip: flush");
            if (q == 0) return;
        }
        hip::check(nsh_stream_sync(s), "scheduler_hip: flush");
    };
    // one thread per GPU partition: spinning briefly on its queue takes the futex wake-up out
    // of each run's start (the notification arrives within microseconds of the last one)
    h.queue_spin_us = 200;
    return h;
}

} // namespace schedulers
} // namespace gr
