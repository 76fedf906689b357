// Scheduler plugin base (reference runtime/include/gnuradio/scheduler.hpp).
#pragma once
#include <gnuradio/buffer.hpp>
#include <gnuradio/flat_graph.hpp>
#include <gnuradio/flowgraph_monitor.hpp>
#include <gnuradio/logging.hpp>
#include <gnuradio/neighbor_interface_info.hpp>
#include <gnuradio/scheduler_message.hpp>

namespace gr {

class scheduler : public std::enable_shared_from_this<scheduler>, public neighbor_interface
{
public:
    explicit scheduler(const std::string& name) : _name(name)
    {
        _logger = logging::get_logger(name, "default");
        _debug_logger = logging::get_logger(name + "_dbg", "debug");
    }
    ~scheduler() override = default;
    std::shared_ptr<scheduler> base() { return shared_from_this(); }

    virtual void initialize(flat_graph_sptr fg, flowgraph_monitor_sptr fgmon,
                            neighbor_interface_map scheduler_adapter_map = neighbor_interface_map()) = 0;
    void push_message(scheduler_message_sptr msg) override = 0;
    // Re-arm run state that other schedulers' threads can observe (buffer done flags). The
    // flowgraph calls prepare_run() on every scheduler before it starts any of them: a scheduler
    // that reset its edges' flags in start() could clear a flag a neighbour domain's thread had
    // already acted on, or leave a stale one for a thread that started first.
    virtual void prepare_run() {}
    virtual void start() = 0;
    virtual void stop() = 0;
    virtual void wait() = 0;

    std::string name() const { return _name; }
    int id() const { return _id; }
    void set_id(int id) { _id = id; }

    virtual void set_default_buffer_factory(const buffer_factory_function& bff,
                                            std::shared_ptr<buffer_properties> bp = nullptr)
    {
        _default_buf_factory = bff;
        _default_buf_properties = std::move(bp);
    }

protected:
    logger_sptr _logger;
    logger_sptr _debug_logger;
    buffer_factory_function _default_buf_factory = nullptr;
    std::shared_ptr<buffer_properties> _default_buf_properties = nullptr;

private:
    std::string _name;
    int _id = 0;
};

using scheduler_sptr = std::shared_ptr<scheduler>;

} // namespace gr
