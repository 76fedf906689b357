// In-process domain adapter pair (reference runtime/include/gnuradio/
// domain_adapter_direct.hpp:10-258). One adapter of the pair owns the real edge buffer
// (LOCAL, chosen by buffer_preference_t); the other forwards every buffer call to it
// (REMOTE). Both share a `direct_sync` slot through which the REMOTE side fetches the
// buffer on first use. Work notifications crossing the domain boundary are forwarded to
// the block on the far side, and writer/reader completion flags resolve to the shared
// buffer, so drain-based termination works across domains (the reference test for this
// path is disabled, schedulers/mt/test/qa_scheduler_mt.cpp:40-78).
#pragma once
#include <condition_variable>
#include <cstring>
#include <gnuradio/domain_adapter.hpp>
#include <mutex>

namespace gr {

class direct_sync
{
public:
    static std::shared_ptr<direct_sync> make() { return std::make_shared<direct_sync>(); }
    void set(buffer_sptr b)
    {
        {
            std::lock_guard<std::mutex> g(_m);
            _buf = std::move(b);
        }
        _cv.notify_all();
    }
    buffer_sptr get()
    {
        std::unique_lock<std::mutex> l(_m);
        _cv.wait(l, [this] { return _buf != nullptr; });
        return _buf;
    }

private:
    std::mutex _m;
    std::condition_variable _cv;
    buffer_sptr _buf;
};
using direct_sync_sptr = std::shared_ptr<direct_sync>;

class domain_adapter_direct : public domain_adapter
{
public:
    using sptr = std::shared_ptr<domain_adapter_direct>;

    // other_port: the block port this adapter faces; the adapter gets the opposite
    // direction and the same item size.
    static sptr make(direct_sync_sptr sync, port_sptr other_port, buffer_location_t loc)
    {
        auto p = std::shared_ptr<domain_adapter_direct>(new domain_adapter_direct(std::move(sync), loc));
        const bool faces_input = other_port->direction() == port_direction_t::INPUT;
        p->add_port(untyped_port::make(faces_input ? "output" : "input",
                                       faces_input ? port_direction_t::OUTPUT : port_direction_t::INPUT,
                                       other_port->itemsize()));
        return p;
    }

    void set_peer(std::weak_ptr<domain_adapter_direct> peer) { _peer = std::move(peer); }

    void* read_ptr() override { return target()->read_ptr(); }
    void* write_ptr() override { return target()->write_ptr(); }
    bool read_info(buffer_info_t& i) override { return target()->read_info(i); }
    bool write_info(buffer_info_t& i) override { return target()->write_info(i); }
    void post_read(int n) override { target()->post_read(n); }
    void post_write(int n) override { target()->post_write(n); }
    void copy_items(buffer_sptr from, int n) override { target()->copy_items(std::move(from), n); }
    gr::buffer* tag_target() override { return target().get(); }
    void set_writer_done() override { target()->set_writer_done(); }
    void set_reader_done() override { target()->set_reader_done(); }
    bool writer_done() const override { return const_cast<domain_adapter_direct*>(this)->target()->writer_done(); }
    bool reader_done() const override { return const_cast<domain_adapter_direct*>(this)->target()->reader_done(); }
    void reset_flags() override
    {
        if (_buffer_loc == buffer_location_t::LOCAL && _buffer) _buffer->reset_flags();
    }
    void discard_unread() override
    {
        if (_buffer_loc == buffer_location_t::LOCAL && _buffer) _buffer->discard_unread();
    }

    // Forward a notification that arrived at this adapter's port to the far side.
    struct forwarder : neighbor_interface {
        std::weak_ptr<domain_adapter_direct> self;
        void push_message(scheduler_message_sptr msg) override
        {
            auto s = self.lock();
            if (!s) return;
            auto peer = s->_peer.lock();
            if (!peer) return;
            for (auto& p : peer->all_ports()) p->notify_connected_ports(msg);
        }
    };
    void install_forwarder()
    {
        auto f = std::make_shared<forwarder>();
        f->self = std::static_pointer_cast<domain_adapter_direct>(shared_from_node());
        for (auto& p : all_ports()) p->set_parent_intf(f);
    }

    void set_self(std::weak_ptr<domain_adapter_direct> s) { _self = std::move(s); }

private:
    domain_adapter_direct(direct_sync_sptr sync, buffer_location_t loc)
        : domain_adapter(loc, "domain_adapter_direct"), _sync(std::move(sync))
    {
    }
    std::shared_ptr<node> shared_from_node() { return _self.lock(); }
    buffer_sptr target()
    {
        if (_buffer_loc == buffer_location_t::LOCAL) {
            if (!_buffer) throw std::runtime_error("domain_adapter_direct: LOCAL buffer not set");
            return _buffer;
        }
        if (!_remote) _remote = _sync->get();
        return _remote;
    }

    direct_sync_sptr _sync;
    buffer_sptr _remote;
    std::weak_ptr<domain_adapter_direct> _peer;
    std::weak_ptr<domain_adapter_direct> _self;

public:
    // LOCAL side publishes its buffer to the REMOTE side when the buffer manager sets it.
    void publish() { _sync->set(_buffer); }
    void buffer_ready() override { publish(); }
};

class domain_adapter_direct_conf : public domain_adapter_conf
{
public:
    using sptr = std::shared_ptr<domain_adapter_direct_conf>;
    static sptr make(buffer_preference_t pref = buffer_preference_t::DOWNSTREAM)
    {
        return std::make_shared<domain_adapter_direct_conf>(pref);
    }
    explicit domain_adapter_direct_conf(buffer_preference_t pref) : domain_adapter_conf(pref) {}

    std::pair<domain_adapter_sptr, domain_adapter_sptr>
    make_domain_adapter_pair(port_sptr upstream_port, port_sptr downstream_port, const std::string& name = "") override
    {
        auto sync = direct_sync::make();
        const bool down_local = _buf_pref == buffer_preference_t::DOWNSTREAM;
        auto up = domain_adapter_direct::make(sync, upstream_port,
                                              down_local ? buffer_location_t::REMOTE : buffer_location_t::LOCAL);
        auto down = domain_adapter_direct::make(sync, downstream_port,
                                                down_local ? buffer_location_t::LOCAL : buffer_location_t::REMOTE);
        up->set_self(up);
        down->set_self(down);
        up->set_peer(down);
        down->set_peer(up);
        up->install_forwarder();
        down->install_forwarder();
        if (!name.empty()) {
            up->set_alias(name + "_up");
            down->set_alias(name + "_down");
        }
        return { up, down };
    }
};

} // namespace gr
