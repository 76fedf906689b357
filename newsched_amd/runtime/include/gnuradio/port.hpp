// Block ports (reference runtime/include/gnuradio/port.hpp:27-268). A port knows its item
// size, its index among the block's stream ports, the ports it is connected to, and the
// thread interface that owns its block; notify_connected_ports() is how a work() call
// wakes the neighbouring block-group threads.
#pragma once
#include <algorithm>
#include <gnuradio/neighbor_interface.hpp>
#include <gnuradio/parameter_types.hpp>
#include <memory>
#include <stdexcept>
#include <string>
#include <typeindex>
#include <vector>

namespace gr {

enum class port_type_t { STREAM, MESSAGE };
enum class port_direction_t { INPUT, OUTPUT, BIDIRECTONAL };

class port_base : public std::enable_shared_from_this<port_base>
{
public:
    using sptr = std::shared_ptr<port_base>;

    static sptr make(const std::string& name, port_direction_t dir, param_type_t dtype = param_type_t::CFLOAT,
                     port_type_t ptype = port_type_t::STREAM, const std::vector<size_t>& dims = { 1 },
                     int multiplicity = 1)
    {
        return std::make_shared<port_base>(name, dir, dtype, ptype, dims, multiplicity);
    }

    port_base(const std::string& name, port_direction_t dir, param_type_t dtype = param_type_t::CFLOAT,
              port_type_t ptype = port_type_t::STREAM, const std::vector<size_t>& dims = { 1 },
              int multiplicity = 1)
        : _name(name), _direction(dir), _data_type(dtype), _port_type(ptype), _dims(dims),
          _multiplicity(multiplicity)
    {
        _datasize = parameter_functions::param_size_info(dtype);
        _itemsize = _datasize;
        for (size_t d : _dims) _itemsize *= d; // item = scalar x prod(dims)
    }

    port_base(const std::string& name, port_direction_t dir, size_t itemsize,
              port_type_t ptype = port_type_t::STREAM, int multiplicity = 1)
        : _name(name), _direction(dir), _data_type(param_type_t::UNTYPED), _port_type(ptype),
          _multiplicity(multiplicity), _datasize(itemsize), _itemsize(itemsize)
    {
    }
    virtual ~port_base() = default;

    std::string name() const { return _name; }
    std::string alias() const { return _alias; }
    void set_alias(const std::string& a) { _alias = a; }
    void set_index(int i) { _index = i; }
    int index() const { return _index; }
    port_type_t type() const { return _port_type; }
    param_type_t data_type() const { return _data_type; }
    port_direction_t direction() const { return _direction; }
    size_t data_size() const { return _datasize; }
    size_t itemsize() const { return _itemsize; }
    std::vector<size_t> dims() const { return _dims; }
    sptr base() { return shared_from_this(); }

    void set_parent_intf(neighbor_interface_sptr intf) { _parent_intf = std::move(intf); }
    neighbor_interface_sptr parent_intf() const { return _parent_intf; }

    // Wake the threads owning every connected port.
    void notify_connected_ports(scheduler_message_sptr msg)
    {
        for (auto& w : _connected_ports)
            if (auto p = w.lock()) p->push_message(msg);
    }

    virtual void push_message(scheduler_message_sptr msg)
    {
        if (!_parent_intf) throw std::runtime_error("port " + _name + " has no parent interface");
        _parent_intf->push_message(std::move(msg));
    }

    // Peers are held weakly: each port is owned by its node, and two connected ports holding
    // each other strongly would keep both (and everything they reference) alive forever.
    void connect(sptr other)
    {
        for (auto& w : _connected_ports)
            if (w.lock() == other) return;
        _connected_ports.push_back(other);
    }
    void disconnect(const sptr& other)
    {
        _connected_ports.erase(std::remove_if(_connected_ports.begin(), _connected_ports.end(),
                                              [&](const std::weak_ptr<port_base>& w) {
                                                  auto p = w.lock();
                                                  return !p || p == other;
                                              }),
                               _connected_ports.end());
    }
    std::vector<sptr> connected_ports() const
    {
        std::vector<sptr> r;
        for (auto& w : _connected_ports)
            if (auto p = w.lock()) r.push_back(std::move(p));
        return r;
    }

protected:
    std::string _name;
    std::string _alias;
    port_direction_t _direction;
    param_type_t _data_type;
    port_type_t _port_type;
    int _index = -1;
    std::vector<size_t> _dims;
    int _multiplicity;
    size_t _datasize = 0;
    size_t _itemsize = 0;
    std::vector<std::weak_ptr<port_base>> _connected_ports;
    neighbor_interface_sptr _parent_intf = nullptr;
};

using port_sptr = port_base::sptr;
using port_vector_t = std::vector<port_sptr>;

// Typed stream port: item size = sizeof(T) * prod(dims).
template <class T>
class port : public port_base
{
public:
    static std::shared_ptr<port<T>> make(const std::string& name, port_direction_t dir,
                                         const std::vector<size_t>& dims = {}, int multiplicity = 1)
    {
        return std::make_shared<port<T>>(name, dir, dims, multiplicity);
    }
    port(const std::string& name, port_direction_t dir, const std::vector<size_t>& dims = {}, int multiplicity = 1)
        : port_base(name, dir, parameter_functions::get_param_type_from_typeinfo(std::type_index(typeid(T))),
                    port_type_t::STREAM, dims, multiplicity)
    {
    }
};

// Byte-sized stream port for type-agnostic blocks (copy, head, null_*).
class untyped_port : public port_base
{
public:
    static std::shared_ptr<untyped_port> make(const std::string& name, port_direction_t dir, size_t itemsize,
                                              int multiplicity = 1)
    {
        return std::make_shared<untyped_port>(name, dir, itemsize, multiplicity);
    }
    untyped_port(const std::string& name, port_direction_t dir, size_t itemsize, int multiplicity = 1)
        : port_base(name, dir, itemsize, port_type_t::STREAM, multiplicity)
    {
    }
};

// Message port: control plane only, kept so blocks can declare them.
class message_port : public port_base
{
public:
    using sptr = std::shared_ptr<message_port>;
    static sptr make(const std::string& name, port_direction_t dir, int multiplicity = 1)
    {
        return std::make_shared<message_port>(name, dir, multiplicity);
    }
    message_port(const std::string& name, port_direction_t dir, int multiplicity = 1)
        : port_base(name, dir, 0, port_type_t::MESSAGE, multiplicity)
    {
    }
    message_port_callback_fcn callback() const { return _cb; }
    void register_callback(message_port_callback_fcn f) { _cb = std::move(f); }
    void post(pmtf::pmt_sptr msg) { notify_connected_ports(std::make_shared<msgport_message>(msg, _cb)); }
    void push_message(scheduler_message_sptr msg) override
    {
        std::static_pointer_cast<msgport_message>(msg)->set_callback(_cb);
        port_base::push_message(std::move(msg));
    }

private:
    message_port_callback_fcn _cb;
};
using message_port_sptr = message_port::sptr;

} // namespace gr
