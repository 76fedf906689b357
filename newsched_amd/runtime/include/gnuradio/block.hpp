// Signal-processing block base (reference runtime/include/gnuradio/block.hpp:24-104).
// work() is the plugin point the MI355X path fills with HIP kernels; do_work() wraps it
// (sync_block clamps item counts). start()/stop()/done() bracket a run; unlike the
// reference (which never calls start()), this runtime calls start() on every block when a
// flowgraph starts, so blocks can (re)arm per-run state such as FIR history.
#pragma once
#include <gnuradio/block_work_io.hpp>
#include <gnuradio/gpdict.hpp>
#include <gnuradio/node.hpp>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace gr {

class scheduler;

class block : public gr::node, public std::enable_shared_from_this<block>
{
public:
    using sptr = std::shared_ptr<block>;
    explicit block(const std::string& name)
        : node(name), d_tag_propagation_policy(tag_propagation_policy_t::TPP_ALL_TO_ALL)
    {
    }
    ~block() override = default;

    virtual bool start()
    {
        d_running = true;
        return true;
    }
    virtual bool stop()
    {
        d_running = false;
        return true;
    }
    virtual bool done()
    {
        d_running = false;
        return true;
    }
    bool running() const { return d_running; }

    sptr base() { return shared_from_this(); }
    tag_propagation_policy_t tag_propagation_policy() const { return d_tag_propagation_policy; }
    void set_tag_propagation_policy(tag_propagation_policy_t p) { d_tag_propagation_policy = p; }

    virtual work_return_code_t work(std::vector<block_work_input>& work_input,
                                    std::vector<block_work_output>& work_output)
    {
        throw std::runtime_error("work function has been called but not implemented");
    }
    virtual work_return_code_t do_work(std::vector<block_work_input>& work_input,
                                       std::vector<block_work_output>& work_output)
    {
        return work(work_input, work_output);
    }

    // Output items per input item (1 for sync blocks, 1/D for decim_block) and the output
    // granularity; buffer managers size edges from them.
    virtual double relative_rate() const { return 1.0; }
    int output_multiple() const { return d_output_multiple; }
    void set_output_multiple(int m) { d_output_multiple = m > 0 ? m : 1; }

    // weak: the scheduler owns its blocks (a strong back-reference would leak both)
    void set_scheduler(std::shared_ptr<scheduler> s) { p_scheduler = s; }
    std::shared_ptr<scheduler> get_scheduler() const { return p_scheduler.lock(); }

    gpdict attributes;

protected:
    std::weak_ptr<scheduler> p_scheduler;

private:
    bool d_running = false;
    tag_propagation_policy_t d_tag_propagation_policy;
    int d_output_multiple = 1;
};

using block_sptr = block::sptr;
using block_vector_t = std::vector<block_sptr>;
using block_viter_t = std::vector<block_sptr>::iterator;

} // namespace gr
