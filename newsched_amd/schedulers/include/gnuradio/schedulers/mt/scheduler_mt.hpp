// Thread-per-block-group CPU scheduler (reference schedulers/mt/include/gnuradio/
// schedulers/mt/scheduler_mt.hpp:11-75, schedulers/mt/lib/scheduler_mt.cpp:6-137).
// make(name, fixed_buf_size = 32768); add_block_group(); blocks not in a group get a
// thread each. The default edge buffer is vmcirc_buffer.
#pragma once
#include <gnuradio/domain.hpp>
#include <gnuradio/graph_utils.hpp>
#include <gnuradio/scheduler.hpp>
#include <gnuradio/schedulers/mt/block_group_properties.hpp>
#include <gnuradio/schedulers/mt/thread_wrapper.hpp>
#include <gnuradio/vmcircbuf.hpp>
#include <mutex>

namespace gr {
namespace schedulers {

class scheduler_mt : public scheduler
{
public:
    using sptr = std::shared_ptr<scheduler_mt>;
    static sptr make(const std::string name = "multi_threaded", const unsigned int fixed_buf_size = 32768)
    {
        return std::make_shared<scheduler_mt>(name, fixed_buf_size);
    }
    scheduler_mt(const std::string name = "multi_threaded", const size_t fixed_buf_size = 32768)
        : scheduler(name), s_fixed_buf_size(fixed_buf_size)
    {
        _default_buf_factory = vmcirc_buffer::make;
        _default_buf_properties = vmcirc_buffer_properties::make(vmcirc_buffer_type::AUTO);
    }
    ~scheduler_mt() override;

    void push_message(scheduler_message_sptr msg) override;
    void add_block_group(const std::vector<block_sptr>& blocks, const std::string& name = "",
                         const std::vector<unsigned int>& affinity_mask = {});
    void initialize(flat_graph_sptr fg, flowgraph_monitor_sptr fgmon,
                    neighbor_interface_map block_sched_map = neighbor_interface_map()) override;
    void prepare_run() override;
    void start() override;
    void stop() override;
    void wait() override;
    void run();

    buffer_manager::sptr buffers() const { return _bufman; }
    size_t num_threads() const { return _threads.size(); }

protected:
    // Per-thread hooks; scheduler_hip binds its stream here.
    // Default: a CPU thread that ran hip blocks drains its private stream on flush.
    virtual thread_hooks hooks_for_group(const block_group_properties&);
    // Block groups actually used; scheduler_hip folds the partition into one.
    virtual std::vector<block_group_properties> plan_groups(flat_graph_sptr fg);
    void thread_finished(int thread_index);

    std::vector<thread_wrapper::sptr> _threads;
    const size_t s_fixed_buf_size;
    std::map<nodeid_t, neighbor_interface_sptr> _block_thread_map;
    std::vector<block_group_properties> _block_groups;
    buffer_manager::sptr _bufman;
    flowgraph_monitor_sptr _fgmon;
    std::vector<block_sptr> _blocks;
    std::mutex _fin_mtx;
    size_t _n_finished = 0;
    bool _prepared = false; // prepare_run() done for the next start()
};

} // namespace schedulers
} // namespace gr
