// Edges between (node, port) endpoints, carrying the optional custom buffer factory
// (reference runtime/include/gnuradio/edge.hpp, runtime/lib/edge.cpp).
#pragma once
#include <gnuradio/buffer.hpp>
#include <gnuradio/node.hpp>
#include <ostream>
#include <utility>
#include <vector>

namespace gr {

template <class A, class B>
class endpoint : public std::pair<A, B>
{
public:
    endpoint() = default;
    endpoint(A a, B b) : std::pair<A, B>(std::move(a), std::move(b)) {}
    virtual ~endpoint() = default;
};

class node_endpoint : public endpoint<node_sptr, port_sptr>
{
public:
    node_endpoint() = default;
    node_endpoint(node_sptr n, port_sptr p) : endpoint<node_sptr, port_sptr>(std::move(n), std::move(p)) {}
    node_sptr node() const { return this->first; }
    port_sptr port() const { return this->second; }
    std::string identifier() const { return first->alias() + ":" + second->name(); }
};

inline bool operator==(const node_endpoint& a, const node_endpoint& b)
{
    return a.node() == b.node() && a.port() == b.port();
}
inline std::ostream& operator<<(std::ostream& os, const node_endpoint& e) { return os << e.identifier(); }

class edge
{
public:
    using sptr = std::shared_ptr<edge>;
    static sptr make(const node_endpoint& src, const node_endpoint& dst) { return std::make_shared<edge>(src, dst); }
    static sptr make(node_sptr sb, port_sptr sp, node_sptr db, port_sptr dp)
    {
        return std::make_shared<edge>(node_endpoint(sb, sp), node_endpoint(db, dp));
    }
    edge(const node_endpoint& src, const node_endpoint& dst) : _src(src), _dst(dst) {}
    edge(node_sptr sb, port_sptr sp, node_sptr db, port_sptr dp) : _src(sb, sp), _dst(db, dp) {}
    virtual ~edge() = default;

    node_endpoint src() const { return _src; }
    node_endpoint dst() const { return _dst; }
    std::string identifier() const { return _src.identifier() + "->" + _dst.identifier(); }
    size_t itemsize() const { return _src.port()->itemsize(); }

    // Select the buffer implementation for this edge (e.g. HIP_BUFFER_ARGS_D2D).
    void set_custom_buffer(buffer_factory_function f, std::shared_ptr<buffer_properties> p = nullptr)
    {
        _buffer_factory = std::move(f);
        _buffer_properties = std::move(p);
    }
    bool has_custom_buffer() const { return _buffer_factory != nullptr; }
    buffer_factory_function buffer_factory() const { return _buffer_factory; }
    std::shared_ptr<buffer_properties> buf_properties() const { return _buffer_properties; }

protected:
    node_endpoint _src, _dst;
    buffer_factory_function _buffer_factory = nullptr;
    std::shared_ptr<buffer_properties> _buffer_properties = nullptr;
};

inline bool operator==(const edge& a, const edge& b) { return a.src() == b.src() && a.dst() == b.dst(); }
inline std::ostream& operator<<(std::ostream& os, const edge& e) { return os << e.identifier(); }

using edge_sptr = edge::sptr;
using edge_vector_t = std::vector<edge_sptr>;

} // namespace gr
