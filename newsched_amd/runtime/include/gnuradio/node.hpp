// Graph node: name, alias, unique id and ports (reference
// runtime/include/gnuradio/node.hpp:26-160).
#pragma once
#include <atomic>
#include <gnuradio/logging.hpp>
#include <gnuradio/port.hpp>
#include <string>
#include <vector>

namespace gr {

using nodeid_t = uint32_t;

struct nodeid_generator {
    static nodeid_t get_id()
    {
        static std::atomic<nodeid_t> next{ 1 }; // 0 addresses "all threads" in messages
        return next++;
    }
};

class node
{
public:
    using sptr = std::shared_ptr<node>;
    node() : d_name(""), d_id(0) {}
    explicit node(const std::string& name) : d_name(name), d_id(nodeid_generator::get_id()) {}
    virtual ~node() = default;

    std::vector<port_sptr>& all_ports() { return d_all_ports; }
    std::vector<port_sptr>& input_ports() { return d_input_ports; }
    std::vector<port_sptr>& output_ports() { return d_output_ports; }
    std::vector<port_sptr> input_stream_ports() const { return stream_ports(d_input_ports); }
    std::vector<port_sptr> output_stream_ports() const { return stream_ports(d_output_ports); }
    std::vector<size_t> sizeof_input_stream_ports() const { return sizes(d_input_ports); }
    std::vector<size_t> sizeof_output_stream_ports() const { return sizes(d_output_ports); }

    std::string& name() { return d_name; }
    std::string& alias() { return d_alias; }
    nodeid_t id() const { return d_id; }
    void set_id(nodeid_t id) { d_id = id; }
    void set_alias(const std::string& alias)
    {
        d_alias = alias;
        _logger = logging::get_logger(alias, "default");
        _debug_logger = logging::get_logger(alias + "_dbg", "debug");
    }

    port_sptr get_port(const std::string& name)
    {
        for (auto& p : d_all_ports)
            if (p->name() == name) return p;
        return nullptr;
    }
    message_port_sptr get_message_port(const std::string& name)
    {
        return std::dynamic_pointer_cast<message_port>(get_port(name));
    }
    port_sptr get_port(unsigned int index, port_type_t type, port_direction_t dir)
    {
        for (auto& p : d_all_ports)
            if (p->type() == type && p->direction() == dir && p->index() == (int)index) return p;
        return nullptr;
    }

    // Public so factories (X::make) can declare ports after construction, as the
    // reference's blocks do through their own static make().
    void add_port(port_sptr p)
    {
        d_all_ports.push_back(p);
        if (p->direction() == port_direction_t::INPUT) {
            if (p->type() == port_type_t::STREAM) p->set_index((int)input_stream_ports().size());
            d_input_ports.push_back(p);
        } else if (p->direction() == port_direction_t::OUTPUT) {
            if (p->type() == port_type_t::STREAM) p->set_index((int)output_stream_ports().size());
            d_output_ports.push_back(p);
        }
    }

protected:
    std::string d_name;
    std::string d_alias;
    nodeid_t d_id;
    std::vector<port_sptr> d_all_ports;
    std::vector<port_sptr> d_input_ports;
    std::vector<port_sptr> d_output_ports;
    logger_sptr _logger;
    logger_sptr _debug_logger;

private:
    static std::vector<port_sptr> stream_ports(const std::vector<port_sptr>& v)
    {
        std::vector<port_sptr> r;
        for (auto& p : v)
            if (p->type() == port_type_t::STREAM) r.push_back(p);
        return r;
    }
    static std::vector<size_t> sizes(const std::vector<port_sptr>& v)
    {
        std::vector<size_t> r;
        for (auto& p : v)
            if (p->type() == port_type_t::STREAM) r.push_back(p->data_size());
        return r;
    }
};

using node_sptr = node::sptr;
using node_vector_t = std::vector<node_sptr>;

} // namespace gr
