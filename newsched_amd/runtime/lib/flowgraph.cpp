// flowgraph + flowgraph_monitor (reference runtime/lib/flowgraph.cpp,
// runtime/lib/flowgraph_monitor.cpp; drain-based completion, see flowgraph_monitor.hpp).
#include <gnuradio/run_trace.hpp>
#include <gnuradio/domain_adapter_remote.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/graph_utils.hpp>

#include <algorithm>
#include <chrono>

namespace gr {

// ---- flowgraph_monitor ---------------------------------------------------------------
void flowgraph_monitor::push_message(fg_monitor_message msg)
{
    std::lock_guard<std::mutex> g(_m);
    switch (msg.type()) {
    case fg_monitor_message_t::DONE: ++_done_blocks; break;
    case fg_monitor_message_t::FLUSHED:
        _flushed[msg.schedid()] = true;
        NSR_RT(8);
        break;
    case fg_monitor_message_t::KILL: _killed = true; break;
    default: break;
    }
    if (_killed || run_complete()) _complete.store(true, std::memory_order_release);
    _cv.notify_all();
}

void flowgraph_monitor::start()
{
    std::lock_guard<std::mutex> g(_m);
    _flushed.clear();
    _killed = false;
    _complete.store(false, std::memory_order_release);
    _done_blocks = 0;
    _error = nullptr;
}

bool flowgraph_monitor::run_complete()
{
    for (auto& s : d_schedulers)
        if (!_flushed.count(s->id())) return false;
    return true;
}

void flowgraph_monitor::wait()
{
    if (_wait_spin_us > 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(_wait_spin_us);
        while (!_complete.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < until)
            __builtin_ia32_pause();
    }
    std::unique_lock<std::mutex> l(_m);
    _cv.wait(l, [this] { return _killed || run_complete(); });
}

void flowgraph_monitor::report_error(std::exception_ptr e)
{
    std::lock_guard<std::mutex> g(_m);
    if (!_error) _error = e;
}

std::exception_ptr flowgraph_monitor::error()
{
    std::lock_guard<std::mutex> g(_m);
    return _error;
}

uint64_t flowgraph_monitor::done_blocks()
{
    std::lock_guard<std::mutex> g(_m);
    return _done_blocks;
}

bool flowgraph_monitor::replace_scheduler(std::shared_ptr<scheduler> original,
                                          const std::vector<std::shared_ptr<scheduler>> replacements)
{
    std::lock_guard<std::mutex> g(_m);
    auto it = std::find(d_schedulers.begin(), d_schedulers.end(), original);
    if (it == d_schedulers.end()) return false;
    d_schedulers.erase(it);
    d_schedulers.insert(d_schedulers.end(), replacements.begin(), replacements.end());
    return true;
}

// ---- flowgraph -------------------------------------------------------------------------
flowgraph::~flowgraph()
{
    for (auto& s : d_schedulers) {
        try {
            s->stop();
        } catch (...) {
        }
    }
    // Ownership cycles of a finished flowgraph: block ports point at their thread
    // (neighbor interface) which owns the blocks; the monitor and the schedulers point at
    // each other. Break them so threads, buffers and domain adapters (whose destructors
    // close cross-process edges gracefully) are released with the flowgraph.
    auto unhook = [](graph& g) {
        for (auto& e : g.edges())
            for (auto* n : { e->src().node().get(), e->dst().node().get() })
                if (n)
                    for (auto& p : n->all_ports()) p->set_parent_intf(nullptr);
        for (auto& n : g.orphan_nodes())
            for (auto& p : n->all_ports()) p->set_parent_intf(nullptr);
    };
    for (auto& fgs : d_flat_subgraphs)
        if (fgs) unhook(*fgs);
    if (d_flat_graph) unhook(*d_flat_graph);
    unhook(*this);
    if (d_fgmon) d_fgmon->release();
}

void flowgraph::set_scheduler(scheduler_sptr s) { set_schedulers({ std::move(s) }); }
void flowgraph::set_schedulers(std::vector<scheduler_sptr> s)
{
    d_schedulers = std::move(s);
    int id = 1;
    for (auto& x : d_schedulers) x->set_id(id++);
}
void flowgraph::add_scheduler(scheduler_sptr s)
{
    d_schedulers.push_back(std::move(s));
    int id = 1;
    for (auto& x : d_schedulers) x->set_id(id++);
}
void flowgraph::clear_schedulers() { d_schedulers.clear(); }

void flowgraph::partition(std::vector<domain_conf>& confs)
{
    // Domains run by another process (remote_domain) are neither monitored nor started
    // here; this process runs the local ones and its halves of the crossings.
    d_schedulers.erase(std::remove_if(d_schedulers.begin(), d_schedulers.end(),
                                      [](const scheduler_sptr& s) {
                                          return std::dynamic_pointer_cast<remote_domain>(s) != nullptr;
                                      }),
                       d_schedulers.end());
    d_fgmon = std::make_shared<flowgraph_monitor>(d_schedulers);
    d_fgmon->set_wait_spin_us(d_wait_spin_us);
    auto parts = graph_utils::partition(base(), d_schedulers, confs);
    d_flat_subgraphs.clear();
    for (auto& p : parts) {
        if (std::dynamic_pointer_cast<remote_domain>(p.scheduler)) continue;
        d_flat_subgraphs.push_back(flat_graph::make_flat(p.subgraph));
        p.scheduler->initialize(d_flat_subgraphs.back(), d_fgmon, p.neighbor_map);
    }
}

void flowgraph::validate()
{
    if (d_schedulers.empty()) throw std::runtime_error("flowgraph::validate: no scheduler specified");
    d_fgmon = std::make_shared<flowgraph_monitor>(d_schedulers);
    d_fgmon->set_wait_spin_us(d_wait_spin_us);
    d_flat_graph = flat_graph::make_flat(base());
    for (auto& s : d_schedulers) s->initialize(d_flat_graph, d_fgmon);
}

void flowgraph::start()
{
    if (d_schedulers.empty()) throw std::runtime_error("No Scheduler Specified.");
    if (!d_fgmon) validate();
    d_fgmon->start();
    for (auto& s : d_schedulers) s->prepare_run(); // every domain's edges re-armed first
    for (auto& s : d_schedulers) s->start();
    d_started = true;
}

void flowgraph::stop()
{
    for (auto& s : d_schedulers) s->stop();
    if (d_fgmon) d_fgmon->stop();
    d_started = false;
}

void flowgraph::wait()
{
    if (!d_started) return;
    d_fgmon->wait();
    for (auto& s : d_schedulers) s->wait();
    d_started = false;
    if (auto e = d_fgmon->error()) std::rethrow_exception(e);
}

void flowgraph::run()
{
    NSR_RT(0);
    start();
    NSR_RT(1);
    wait();
    NSR_RT(9);
}

} // namespace gr
