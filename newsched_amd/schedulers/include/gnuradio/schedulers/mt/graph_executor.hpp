// Runs one pass over a thread's blocks: gathers buffer state, calls do_work(), advances
// buffers, notifies neighbours (reference schedulers/mt/lib/graph_executor.cpp:7-221 --
// THE caller of work()). Differences: per-block completion for drain-based termination;
// WORK_ERROR / WORK_INSUFFICIENT_OUTPUT_ITEMS throw instead of spinning forever (:102-131).
#pragma once
#include <gnuradio/block.hpp>
#include <gnuradio/executor.hpp>
#include <gnuradio/schedulers/mt/buffer_management.hpp>
#include <functional>
#include <map>
#include <set>

namespace gr {
namespace schedulers {

// Called on the executing thread around each do_work() call: before(b), then after(b, n) with the
// items the call produced on its first output (0 for a sink, -1 when do_work threw). scheduler_hip
// times its partition's kernel launches with them.
struct work_hooks {
    std::function<void(const block_sptr&)> before;
    std::function<void(const block_sptr&, int)> after;
};

class graph_executor : public executor
{
public:
    explicit graph_executor(const std::string& name) : executor(name) {}

    void initialize(buffer_manager::sptr bufman, std::vector<block_sptr> blocks, work_hooks hooks = {})
    {
        _bufman = std::move(bufman);
        d_blocks = std::move(blocks);
        _hooks = std::move(hooks);
    }

    std::map<nodeid_t, executor_iteration_status> run_one_iteration(std::vector<block_sptr> blocks = {});

    void reset_run_state() { _finished.clear(); }
    // Mark every block finished (error path): flags its buffers so neighbours drain.
    // the error path's wind-down (a work() call threw): every block is finished even when one
    // of them throws again on the way (a remote edge whose setup failed rethrows its error at
    // each use); the first error is already with the flowgraph monitor
    void finish_all()
    {
        for (auto& b : d_blocks) {
            try {
                finish(b);
            } catch (...) {
            }
        }
    }
    bool all_finished(const std::vector<block_sptr>& blocks) const;
    const std::vector<block_sptr>& blocks() const { return d_blocks; }

private:
    void finish(const block_sptr& b);
    std::vector<block_sptr> d_blocks;
    buffer_manager::sptr _bufman;
    work_hooks _hooks;
    std::set<nodeid_t> _finished;
    static constexpr int s_min_items_to_process = 1;
    static constexpr int s_min_buf_items = 1;
};

} // namespace schedulers
} // namespace gr
