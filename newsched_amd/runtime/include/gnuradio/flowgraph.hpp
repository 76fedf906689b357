// Top-level flowgraph (reference runtime/include/gnuradio/flowgraph.hpp,
// runtime/lib/flowgraph.cpp). validate()/partition() build buffers and threads once;
// start()/wait() may be repeated (each run re-arms blocks via block::start()).
#pragma once
#include <gnuradio/domain.hpp>
#include <gnuradio/flowgraph_monitor.hpp>
#include <gnuradio/graph.hpp>
#include <gnuradio/scheduler.hpp>

namespace gr {

class flowgraph : public graph
{
public:
    using sptr = std::shared_ptr<flowgraph>;
    static sptr make() { return std::make_shared<flowgraph>(); }
    flowgraph() { set_alias("flowgraph"); }
    ~flowgraph() override;

    void set_scheduler(scheduler_sptr sched);
    void set_schedulers(std::vector<scheduler_sptr> scheds);
    void add_scheduler(scheduler_sptr sched);
    void clear_schedulers();
    void partition(std::vector<domain_conf>& confs);
    void validate();
    void start();
    void stop();
    void wait();   // rethrows the first exception raised by a work() call
    void run();
    // wait() polls for up to `us` microseconds before sleeping (0: sleep at once). Worth it for
    // short repeated runs: it takes the futex wake-up of the waiting thread out of each run.
    void set_wait_spin_us(int us)
    {
        d_wait_spin_us = us;
        if (d_fgmon) d_fgmon->set_wait_spin_us(us);
    }

private:
    int d_wait_spin_us = 0;
    std::vector<scheduler_sptr> d_schedulers;
    flat_graph_sptr d_flat_graph;
    std::vector<flat_graph_sptr> d_flat_subgraphs;
    flowgraph_monitor_sptr d_fgmon;
    bool d_started = false;
};

using flowgraph_sptr = flowgraph::sptr;

} // namespace gr
