// Domain adapters: the node + buffer that replaces an edge crossing between two
// schedulers (reference runtime/include/gnuradio/domain_adapter.hpp:13-97).
#pragma once
#include <gnuradio/buffer.hpp>
#include <gnuradio/graph.hpp>
#include <gnuradio/node.hpp>
#include <tuple>

namespace gr {

enum class buffer_location_t { LOCAL = 0, REMOTE };
enum class buffer_preference_t { UPSTREAM, DOWNSTREAM };
enum class da_request_t : uint32_t { WRITE_INFO = 0, READ_INFO, POST_WRITE, POST_READ, GET_REMOTE_BUFFER };
enum class da_response_t : uint32_t { OK = 0, ERROR = 1 };

class domain_adapter : public node, public buffer
{
public:
    ~domain_adapter() override = default;
    void set_buffer(buffer_sptr b) { _buffer = std::move(b); }
    buffer_sptr buffer() { return _buffer; }
    buffer_location_t buffer_location() const { return _buffer_loc; }
    void set_buffer_location(buffer_location_t l) { _buffer_loc = l; }
    // Called by the buffer manager once a LOCAL adapter's edge buffer exists.
    virtual void buffer_ready() {}

protected:
    domain_adapter(buffer_location_t loc, const std::string& name = "domain_adapter") : node(name), _buffer_loc(loc) {}
    buffer_sptr _buffer = nullptr;
    buffer_location_t _buffer_loc;
};
using domain_adapter_sptr = std::shared_ptr<domain_adapter>;

class domain_adapter_conf
{
public:
    virtual ~domain_adapter_conf() = default;
    // Returns (adapter attached to the upstream block's output, adapter feeding the
    // downstream block's input). NOTE: the reference returns the pair the other way round
    // relative to how graph_utils consumes it (domain_adapter_direct.hpp:241-256 vs
    // graph_utils.cpp:166-177); this runtime fixes the order here.
    virtual std::pair<domain_adapter_sptr, domain_adapter_sptr>
    make_domain_adapter_pair(port_sptr upstream_port, port_sptr downstream_port, const std::string& name = "")
    {
        throw std::runtime_error("Cannot create domain adapter pair from base class");
    }
    // One half of a crossing whose other end lives in another process
    // (domain_adapter_remote.hpp). local_port: the local block's port at the crossing.
    virtual std::shared_ptr<domain_adapter>
    make_remote_adapter(port_sptr local_port, bool local_is_upstream, int crossing, const std::string& name = "")
    {
        throw std::runtime_error("this domain_adapter_conf cannot cross process boundaries");
    }

protected:
    explicit domain_adapter_conf(buffer_preference_t p) : _buf_pref(p) {}
    buffer_preference_t _buf_pref;
};
using domain_adapter_conf_sptr = std::shared_ptr<domain_adapter_conf>;
using domain_adapter_conf_per_edge = std::vector<std::tuple<edge_sptr, domain_adapter_conf_sptr>>;

} // namespace gr
