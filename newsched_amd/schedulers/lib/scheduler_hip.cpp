// GPU scheduler domain (see scheduler_hip.hpp).
#include <atomic>
#include <chrono>
#include <gnuradio/hip_context.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <map>
#include <mutex>

#include "nsh_hip.h"

namespace gr {
namespace schedulers {

// Per-block event pairs of the timed work() calls. Written by the partition thread inside a run,
// read (folded) by the caller between runs; the mutex keeps the two apart anyway.
struct scheduler_hip::launch_timer {
    struct pairs {
        std::string alias;
        std::vector<std::pair<void*, void*>> ev; // pool; [0, used) armed or recorded since the last fold
        std::vector<uint64_t> items;             // per recorded pair
        size_t used = 0;
        kernel_stat done;                        // folded totals
        uint64_t done_unrecorded = 0;            // pairs a block's own timing displaced
    };
    std::atomic<bool> on{ false };
    std::mutex m;
    std::map<nodeid_t, pairs> blocks;
    uint64_t count_before = 0;

    ~launch_timer()
    {
        for (auto& kv : blocks)
            for (auto& e : kv.second.ev) {
                nsh_event_destroy(e.first);
                nsh_event_destroy(e.second);
            }
    }
    void fold(pairs& p)
    {
        for (size_t i = 0; i < p.used; ++i) {
            float ms = 0;
            hip::check(nsh_event_sync(p.ev[i].second), "scheduler_hip: kernel timing");
            if (nsh_event_elapsed_ms(p.ev[i].first, p.ev[i].second, &ms) != 0) {
                // never recorded: a block armed a pair of its own over ours (its own kernel timing,
                // e.g. hip::fir_filter_ccf::enable_timing) and the launch took that one. Not counted,
                // and the pair is replaced so no stale time can be read from it later.
                nsh_event_destroy(p.ev[i].first);
                nsh_event_destroy(p.ev[i].second);
                p.ev[i] = { nullptr, nullptr };
                hip::check(nsh_event_create(&p.ev[i].first), "scheduler_hip: kernel timing");
                hip::check(nsh_event_create(&p.ev[i].second), "scheduler_hip: kernel timing");
                ++p.done_unrecorded;
                continue;
            }
            p.done.kernel_ms += ms;
            p.done.launches += 1;
            p.done.items += p.items[i];
        }
        p.used = 0;
        p.items.clear();
    }
    void before(const block_sptr& b)
    {
        if (!on.load(std::memory_order_relaxed)) return;
        std::lock_guard<std::mutex> g(m);
        auto& p = blocks[b->id()];
        if (p.alias.empty()) p.alias = b->alias();
        if (p.used >= 4096) fold(p); // a long unread series
        if (p.used == p.ev.size()) {
            std::pair<void*, void*> e{ nullptr, nullptr };
            hip::check(nsh_event_create(&e.first), "scheduler_hip: kernel timing");
            hip::check(nsh_event_create(&e.second), "scheduler_hip: kernel timing");
            p.ev.push_back(e);
        }
        hip::check(nsh_timed_launches(&count_before), "scheduler_hip: kernel timing");
        hip::check(nsh_time_next_launch(p.ev[p.used].first, p.ev[p.used].second), "scheduler_hip: kernel timing");
    }
    void after(const block_sptr& b, int produced)
    {
        if (!on.load(std::memory_order_relaxed)) return;
        std::lock_guard<std::mutex> g(m);
        uint64_t now = 0;
        nsh_time_next_launch(nullptr, nullptr); // whatever happened, nothing stays armed
        hip::check(nsh_timed_launches(&now), "scheduler_hip: kernel timing");
        auto it = blocks.find(b->id());
        if (it == blocks.end() || now == count_before || produced < 0) return; // nothing launched: pair unused
        it->second.items.push_back((uint64_t)produced);
        ++it->second.used;
    }
};

void scheduler_hip::set_kernel_timing(bool on) { _timer->on.store(on); }

std::vector<scheduler_hip::kernel_stat> scheduler_hip::kernel_stats()
{
    std::lock_guard<std::mutex> g(_timer->m);
    std::vector<kernel_stat> out;
    for (auto& kv : _timer->blocks) {
        _timer->fold(kv.second);
        if (kv.second.done.launches == 0) continue;
        kernel_stat k = kv.second.done;
        k.block = kv.second.alias;
        out.push_back(k);
    }
    return out;
}

void scheduler_hip::reset_kernel_stats()
{
    std::lock_guard<std::mutex> g(_timer->m);
    for (auto& kv : _timer->blocks) {
        kv.second.used = 0;
        kv.second.items.clear();
        kv.second.done = kernel_stat();
    }
}

scheduler_hip::scheduler_hip(const std::string name, int device, size_t fixed_buf_size)
    : scheduler_mt(name, fixed_buf_size), _timer(std::make_shared<launch_timer>()), _device(device)
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
    auto t = _timer;
    h.on_work.before = [t](const block_sptr& b) { t->before(b); };
    h.on_work.after = [t](const block_sptr& b, int produced) { t->after(b, produced); };
    return h;
}

} // namespace schedulers
} // namespace gr
