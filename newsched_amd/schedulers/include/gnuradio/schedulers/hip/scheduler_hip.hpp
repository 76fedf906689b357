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
#pragma once
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

namespace gr {
namespace schedulers {

class scheduler_hip : public scheduler_mt
{
public:
    using sptr = std::shared_ptr<scheduler_hip>;
    static sptr make(const std::string name = "hip", int device = 0, size_t fixed_buf_size = 64u << 20)
    {
        return std::make_shared<scheduler_hip>(name, device, fixed_buf_size);
    }
    scheduler_hip(const std::string name = "hip", int device = 0, size_t fixed_buf_size = 64u << 20);
    ~scheduler_hip() override;

    int device() const { return _device; }
    void* stream() const { return _stream; }

protected:
    thread_hooks hooks_for_group(const block_group_properties&) override;
    std::vector<block_group_properties> plan_groups(flat_graph_sptr fg) override;

private:
    int _device;
    void* _stream = nullptr;
};

} // namespace schedulers
} // namespace gr
