// GPU scheduler domain for MI355X: one host thread + one hipStream per partition.
//
// The partition's blocks run on a single thread in topological order with the partition
// stream bound (gr::hip::bind_thread), so every kernel of the partition is stream-ordered
// and no work() call or buffer operation synchronises with the host. Edges default to
// device-resident hip_buffer (D2D) sized for large work() calls: the default
// fixed_buf_size is 64 MiB (buffers of 2 * 64 MiB), i.e. up to 8 Mi complex samples per
// call, versus the reference's 32 KiB / 4096-sample chunks (scheduler_mt.hpp:22,
// vmcircbuf.cpp:83). On flush the thread drains the stream before reporting, so the run
// only completes when the device is idle. One scheduler_hip per GPU (device index).
//
// Before buffers are allocated, initialize() fuses every maximal chain of elementwise
// device blocks (multiply_const_cc, copy, multiply_const_chain_cc joined by D2D edges)
// into one block with one launch per work() call (gnuradio/hip_fusion.hpp), and
// fft -> multiply_const_vcc -> ifft into the channelizer; those results are bit-identical.
// Chains of decimating fir_filter_ccf blocks with total decimation 8 or 16 become one
// fir_filter_cascade_ccf: NOT bit-identical -- within fp32 transform rounding relative to each
// 512-row frame's input level (nsh_hip.h, nsh_fir_cascade_ccf); inf/NaN frames reproduce the
// chain's non-finite pattern. It is on by default and a make() argument, so a flowgraph that
// needs the staged blocks' exact outputs says so where the scheduler is built:
// scheduler_hip::make("hip", dev, buf, /*fir_fusion=*/false) (or set_fir_fusion(false) before
// the flowgraph is validated). set_fusion(false) keeps every block and edge as connected.
#pragma once
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_fusion.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

namespace gr {
namespace schedulers {

class scheduler_hip : public scheduler_mt
{
public:
    using sptr = std::shared_ptr<scheduler_hip>;
    static sptr make(const std::string name = "hip", int device = 0, size_t fixed_buf_size = 64u << 20,
                     bool fir_fusion = true)
    {
        auto s = std::make_shared<scheduler_hip>(name, device, fixed_buf_size);
        s->set_fir_fusion(fir_fusion);
        return s;
    }
    scheduler_hip(const std::string name = "hip", int device = 0, size_t fixed_buf_size = 64u << 20);
    ~scheduler_hip() override;

    int device() const { return _device; }
    void* stream() const { return _stream; }

    void initialize(flat_graph_sptr fg, flowgraph_monitor_sptr fgmon,
                    neighbor_interface_map block_sched_map = neighbor_interface_map()) override;
    // Elementwise fusion on (default) or off; takes effect at the next initialize().
    void set_fusion(bool on) { _fusion = on; }
    bool fusion() const { return _fusion; }
    // The FIR-chain pass (hip::fuse_fir_cascade; within tolerance, not bit-identical) on (default)
    // or off; applies when fusion() is on.
    void set_fir_fusion(bool on) { _fir_fusion = on; }
    bool fir_fusion() const { return _fir_fusion; }
    // End-of-run wait: poll the stream for up to `us` microseconds before blocking in
    // hipStreamSynchronize (0 = block at once, the default). A blocking wait wakes some
    // microseconds after the stream drains; polling sees it at once, for a busy host core during
    // the run's last kernel. Takes effect at the next initialize().
    void set_flush_spin_us(int us) { _flush_spin_us = us; }
    int flush_spin_us() const { return _flush_spin_us; }
    // What the last initialize() fused: blocks that replaced chains, and the chains.
    const hip::fusion_result& fusion_plan() const { return _plan; }

    // Kernel timing of the partition's work() calls (off by default; switch it between runs).
    // Each call gets an event pair that its kernel launch records as part of its own dispatch
    // (nsh_time_next_launch, no extra stream packets); a call that launches nothing (nop blocks,
    // sinks) is not counted (nsh_timed_launches). kernel_stats() waits for the recorded events
    // and returns the totals per block (fused blocks under their own alias) since the last
    // reset_kernel_stats(); call it between runs.
    struct kernel_stat {
        std::string block;
        double kernel_ms = 0;   // summed start-to-end time of the timed launches
        uint64_t launches = 0;  // work() calls that launched (and recorded their pair)
        uint64_t items = 0;     // items those calls produced on their first output
    };
    void set_kernel_timing(bool on);
    std::vector<kernel_stat> kernel_stats();
    void reset_kernel_stats();

protected:
    thread_hooks hooks_for_group(const block_group_properties&) override;
    std::vector<block_group_properties> plan_groups(flat_graph_sptr fg) override;

private:
    void release_fused();
    struct launch_timer;
    std::shared_ptr<launch_timer> _timer;
    int _device;
    void* _stream = nullptr;
    bool _fusion = true;
    bool _fir_fusion = true;
    int _flush_spin_us = 0;
    hip::fusion_result _plan;
};

} // namespace schedulers
} // namespace gr
