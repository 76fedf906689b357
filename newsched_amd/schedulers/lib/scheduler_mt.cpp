// Thread-per-block-group scheduler (reference schedulers/mt/lib/scheduler_mt.cpp:6-137).
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

#include <algorithm>
#include <gnuradio/hip_context.hpp>

namespace gr {
namespace schedulers {

scheduler_mt::~scheduler_mt()
{
    for (auto& t : _threads) t->stop();
}

void scheduler_mt::push_message(scheduler_message_sptr msg)
{
    if (msg->blkid() == 0) { // 0 addresses every thread
        for (auto& t : _threads) t->push_message(msg);
    } else {
        auto it = _block_thread_map.find((nodeid_t)msg->blkid());
        if (it != _block_thread_map.end()) it->second->push_message(msg);
    }
}

thread_hooks scheduler_mt::hooks_for_group(const block_group_properties&)
{
    thread_hooks h;
    h.on_flush = [] { hip::sync_thread_stream(); };
    return h;
}

void scheduler_mt::add_block_group(const std::vector<block_sptr>& blocks, const std::string& name,
                                   const std::vector<unsigned int>& affinity_mask)
{
    _block_groups.emplace_back(blocks, name, affinity_mask);
}

std::vector<block_group_properties> scheduler_mt::plan_groups(flat_graph_sptr fg)
{
    auto blocks = fg->calc_used_blocks();
    std::vector<block_group_properties> groups;
    for (auto& bg : _block_groups) {
        std::vector<block_sptr> mine;
        for (auto& b : bg.blocks()) {
            auto it = std::find(blocks.begin(), blocks.end(), b);
            if (it != blocks.end()) {
                mine.push_back(b);
                blocks.erase(it);
            }
        }
        if (!mine.empty()) groups.emplace_back(mine, bg.name(), bg.processor_affinity());
    }
    for (auto& b : blocks) groups.emplace_back(std::vector<block_sptr>{ b }); // thread per block
    return groups;
}

void scheduler_mt::initialize(flat_graph_sptr fg, flowgraph_monitor_sptr fgmon, neighbor_interface_map)
{
    for (auto& t : _threads) t->stop();
    _threads.clear();
    _block_thread_map.clear();
    _fgmon = fgmon;
    _blocks = fg->calc_used_blocks();
    for (auto& b : _blocks) b->set_scheduler(base());

    _bufman = std::make_shared<buffer_manager>(s_fixed_buf_size);
    _bufman->initialize_buffers(fg, _default_buf_factory, _default_buf_properties);

    auto groups = plan_groups(fg);
    int idx = 0;
    for (auto& g : groups) {
        auto t = thread_wrapper::make(id(), g, _bufman, fgmon, hooks_for_group(g),
                                      [this](int i) { thread_finished(i); }, idx++);
        _threads.push_back(t);
        for (auto& b : g.blocks()) {
            for (auto& p : b->all_ports()) p->set_parent_intf(t);
            _block_thread_map[b->id()] = t;
        }
    }
}

void scheduler_mt::thread_finished(int)
{
    bool all = false;
    {
        std::lock_guard<std::mutex> g(_fin_mtx);
        all = ++_n_finished == _threads.size();
    }
    if (all && _fgmon) _fgmon->push_message(fg_monitor_message(fg_monitor_message_t::FLUSHED, id()));
}

void scheduler_mt::prepare_run()
{
    _prepared = true;
    {
        std::lock_guard<std::mutex> g(_fin_mtx);
        _n_finished = 0;
    }
    if (_bufman)
        for (auto& b : _bufman->all_buffers()) {
            b->reset_flags();
            b->discard_unread();
        }
}

void scheduler_mt::start()
{
    if (!_prepared) prepare_run(); // started directly (not through flowgraph::start)
    _prepared = false;
    if (_threads.empty()) {
        if (_fgmon) _fgmon->push_message(fg_monitor_message(fg_monitor_message_t::FLUSHED, id()));
        return;
    }
    for (auto& t : _threads) t->start();
}

void scheduler_mt::stop()
{
    for (auto& t : _threads) t->stop();
}

void scheduler_mt::wait()
{
    for (auto& b : _blocks) b->done();
}

void scheduler_mt::run()
{
    start();
    if (_fgmon) _fgmon->wait();
    wait();
}

} // namespace schedulers
} // namespace gr
