// Cross-process domain adapters (see domain_adapter_remote.hpp for the design).
#include <gnuradio/domain_adapter_remote.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/hip_context.hpp>

#include "nsh_hip.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>

namespace gr {
namespace remote {

namespace {
enum msg_type : uint32_t { M_HELLO = 0x4e534831u, M_DATA = 2, M_DONE = 3, M_READER_DONE = 4, M_CLOSE = 5 };
struct msg {
    uint32_t type;
    uint32_t aux;
    uint64_t n;
};
struct hello {
    uint32_t magic;     // M_HELLO
    int32_t crossing;
    uint64_t item_size;
    int32_t is_device;  // this side's ring end is device memory
    int32_t device;
    int32_t want;       // 0 auto, 1 rccl, 2 socket (sender's request)
    int32_t chosen;     // receiver's answer: 1 rccl, 2 socket
    int64_t max_chunk;  // receiver's answer: items per message
    char pci[32];       // PCI bus id of `device` ("" for host rings): ordinals differ per
                        // process under per-rank HIP_VISIBLE_DEVICES, bus ids do not
};
using clk = std::chrono::steady_clock;
double since(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

// ---- tags on the wire: the tags of a DATA message's items travel with it ----------------
// record = u64 offset relative to the message's first item, then key, value, srcid as
// [u8 variant index | 255 = null][payload]; payloads: bool u8, int64 / double 8 B, string
// and float vector u32 count + bytes (the PMT stand-in's value types, pmtf.hpp).
template <class T>
void put_raw(std::string& b, const T& v)
{
    b.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
void put_pmt(std::string& b, const pmtf::pmt_sptr& p)
{
    if (!p) {
        b.push_back((char)255);
        return;
    }
    const auto& v = p->value();
    b.push_back((char)v.index());
    switch (v.index()) {
    case 0: break;
    case 1: b.push_back(std::get<bool>(v) ? 1 : 0); break;
    case 2: put_raw(b, std::get<int64_t>(v)); break;
    case 3: put_raw(b, std::get<double>(v)); break;
    case 4: {
        const auto& str = std::get<std::string>(v);
        put_raw(b, (uint32_t)str.size());
        b.append(str);
        break;
    }
    case 5: {
        const auto& f = std::get<std::vector<float>>(v);
        put_raw(b, (uint32_t)f.size());
        b.append(reinterpret_cast<const char*>(f.data()), f.size() * sizeof(float));
        break;
    }
    }
}
struct reader {
    const std::string& b;
    size_t i = 0;
    template <class T>
    T raw()
    {
        if (i + sizeof(T) > b.size()) throw std::runtime_error("remote edge: truncated tag record");
        T v;
        std::memcpy(&v, b.data() + i, sizeof(T));
        i += sizeof(T);
        return v;
    }
    pmtf::pmt_sptr pmt()
    {
        const uint8_t k = raw<uint8_t>();
        switch (k) {
        case 255: return nullptr;
        case 0: return std::make_shared<pmtf::pmt_base>();
        case 1: return pmtf::make(raw<uint8_t>() != 0);
        case 2: return pmtf::make(raw<int64_t>());
        case 3: return pmtf::make(raw<double>());
        case 4: {
            const uint32_t n = raw<uint32_t>();
            if (i + n > b.size()) throw std::runtime_error("remote edge: truncated tag record");
            std::string str(b.data() + i, n);
            i += n;
            return pmtf::make(std::move(str));
        }
        case 5: {
            const uint32_t n = raw<uint32_t>();
            if (i + (size_t)n * sizeof(float) > b.size()) throw std::runtime_error("remote edge: truncated tag record");
            std::vector<float> f(n);
            std::memcpy(f.data(), b.data() + i, (size_t)n * sizeof(float));
            i += (size_t)n * sizeof(float);
            return pmtf::make(std::move(f));
        }
        default: throw std::runtime_error("remote edge: bad tag value type");
        }
    }
};
} // namespace

// ---- control / data socket ------------------------------------------------------------
class channel
{
public:
    explicit channel(int fd) : _fd(fd)
    {
        int one = 1;
        setsockopt(_fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    }
    ~channel()
    {
        if (_fd >= 0) ::close(_fd);
    }
    void send_bytes(const void* p, size_t n)
    {
        auto* c = static_cast<const char*>(p);
        while (n) {
            const ssize_t k = ::send(_fd, c, n, MSG_NOSIGNAL);
            if (k < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("remote edge: send: ") + std::strerror(errno));
            }
            c += k;
            n -= (size_t)k;
        }
    }
    // false on orderly EOF before the first byte
    bool recv_bytes(void* p, size_t n)
    {
        auto* c = static_cast<char*>(p);
        const size_t want = n;
        while (n) {
            const ssize_t k = ::recv(_fd, c, n, 0);
            if (k == 0) {
                if (n == want) return false;
                throw std::runtime_error("remote edge: peer closed mid-message");
            }
            if (k < 0) {
                if (errno == EINTR) continue;
                throw std::runtime_error(std::string("remote edge: recv: ") + std::strerror(errno));
            }
            c += k;
            n -= (size_t)k;
        }
        return true;
    }
    void send_msg(uint32_t type, uint64_t n = 0)
    {
        msg m{ type, 0, n };
        std::lock_guard<std::mutex> g(_send_m);
        send_bytes(&m, sizeof(m));
    }
    // message + payload as one unit with respect to other senders on this socket
    template <typename F>
    void send_msg_with(uint32_t type, uint64_t n, F&& payload, uint32_t aux = 0)
    {
        msg m{ type, aux, n };
        std::lock_guard<std::mutex> g(_send_m);
        send_bytes(&m, sizeof(m));
        payload();
    }
    bool recv_msg(msg& m) { return recv_bytes(&m, sizeof(m)); }
    bool readable(int timeout_ms)
    {
        pollfd pfd{ _fd, POLLIN, 0 };
        return ::poll(&pfd, 1, timeout_ms) > 0 && (pfd.revents & (POLLIN | POLLHUP));
    }
    void shutdown_both() { ::shutdown(_fd, SHUT_RDWR); }
    void shutdown_write() { ::shutdown(_fd, SHUT_WR); }
    // read and drop until the peer closes (or the timeout): closing a socket with unread
    // bytes resets the connection and can destroy data the peer has not read yet
    void drain_until_eof(double timeout_s)
    {
        char buf[4096];
        const auto t0 = clk::now();
        while (since(t0) < timeout_s) {
            if (!readable(100)) continue;
            const ssize_t k = ::recv(_fd, buf, sizeof(buf), 0);
            if (k <= 0) return;
        }
    }

private:
    int _fd;
    std::mutex _send_m;
};

namespace {
sockaddr_in resolve(const std::string& host, int port)
{
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
        addrinfo hints{}, *res = nullptr;
        hints.ai_family = AF_INET;
        if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
            throw std::runtime_error("remote edge: cannot resolve " + host);
        a.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
        freeaddrinfo(res);
    }
    return a;
}

int listen_on(const std::string& host, int port)
{
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw std::runtime_error("remote edge: socket");
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a = resolve(host, port);
    if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 4) != 0) {
        const int e = errno;
        ::close(fd);
        throw std::runtime_error("remote edge: cannot listen on " + host + ":" + std::to_string(port) + ": " +
                                 std::strerror(e));
    }
    return fd;
}

std::shared_ptr<channel> accept_one(int lfd, double timeout_s)
{
    pollfd pfd{ lfd, POLLIN, 0 };
    const int r = ::poll(&pfd, 1, (int)(timeout_s * 1000));
    if (r <= 0) throw std::runtime_error("remote edge: no peer connected within the timeout");
    const int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) throw std::runtime_error(std::string("remote edge: accept: ") + std::strerror(errno));
    return std::make_shared<channel>(fd);
}

std::shared_ptr<channel> connect_retry(const std::string& host, int port, double timeout_s,
                                       const std::atomic<bool>& cancel)
{
    const auto t0 = clk::now();
    const sockaddr_in a = resolve(host, port);
    for (;;) {
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) throw std::runtime_error("remote edge: socket");
        if (::connect(fd, reinterpret_cast<const sockaddr*>(&a), sizeof(a)) == 0) return std::make_shared<channel>(fd);
        ::close(fd);
        if (cancel.load()) throw std::runtime_error("remote edge: cancelled");
        if (since(t0) > timeout_s)
            throw std::runtime_error("remote edge: cannot connect to " + host + ":" + std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}
} // namespace

// ---- data transports -------------------------------------------------------------------
class transport
{
public:
    virtual ~transport() = default;
    virtual const char* kind() const = 0;
    // bytes on the calling thread's stream (device) or directly (host)
    virtual void send(channel& ch, const void* p, size_t bytes) = 0;
    virtual void recv(channel& ch, void* p, size_t bytes) = 0;
};

// Bytes over the control socket. Device memory is staged through a pinned bounce buffer
// (one synchronous D2H/H2D per message): the path for host rings and for two processes
// sharing one GPU, where RCCL cannot be used.
class socket_transport : public transport
{
public:
    explicit socket_transport(bool device) : _device(device) {}
    ~socket_transport() override
    {
        if (_bounce) nsh_host_free(_bounce);
    }
    const char* kind() const override { return _device ? "socket(staged)" : "socket"; }
    void send(channel& ch, const void* p, size_t bytes) override
    {
        if (!_device) {
            ch.send_bytes(p, bytes);
            return;
        }
        ensure(bytes);
        void* s = hip::current_stream();
        hip::check(nsh_memcpy_async(_bounce, p, bytes, NSH_D2H, s), "remote edge: stage D2H");
        hip::check(nsh_stream_sync(s), "remote edge: stage sync");
        ch.send_bytes(_bounce, bytes);
    }
    void recv(channel& ch, void* p, size_t bytes) override
    {
        if (!_device) {
            if (!ch.recv_bytes(p, bytes)) throw std::runtime_error("remote edge: peer closed");
            return;
        }
        ensure(bytes);
        if (!ch.recv_bytes(_bounce, bytes)) throw std::runtime_error("remote edge: peer closed");
        void* s = hip::current_stream();
        hip::check(nsh_memcpy_async(p, _bounce, bytes, NSH_H2D, s), "remote edge: stage H2D");
        hip::check(nsh_stream_sync(s), "remote edge: stage sync"); // bounce reused next message
    }

private:
    void ensure(size_t bytes)
    {
        if (bytes <= _cap) return;
        if (_bounce) nsh_host_free(_bounce);
        _bounce = nullptr;
        hip::check(nsh_host_alloc(bytes, &_bounce), "remote edge: bounce buffer");
        _cap = bytes;
    }
    bool _device;
    void* _bounce = nullptr;
    size_t _cap = 0;
};

// RCCL point-to-point on the partition streams (device rings on different GPUs). librccl
// is loaded on first use so that host-only builds and tests do not need it.
class rccl_transport : public transport
{
    struct api {
        void* h = nullptr;
        int (*get_unique_id)(void*) = nullptr;
        void* comm_init_rank = nullptr; // int ncclCommInitRank(ncclComm_t*, int, ncclUniqueId, int)
        int (*send)(const void*, size_t, int, int, void*, void*) = nullptr;
        int (*recv)(void*, size_t, int, int, void*, void*) = nullptr;
        int (*comm_destroy)(void*) = nullptr;
        const char* (*err_str)(int) = nullptr;
    };
    static api& lib()
    {
        static api a;
        static std::once_flag once;
        std::call_once(once, [] {
            a.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!a.h) a.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!a.h) return;
            a.get_unique_id = (int (*)(void*))dlsym(a.h, "ncclGetUniqueId");
            a.comm_destroy = (int (*)(void*))dlsym(a.h, "ncclCommDestroy");
            a.err_str = (const char* (*)(int))dlsym(a.h, "ncclGetErrorString");
            a.send = (int (*)(const void*, size_t, int, int, void*, void*))dlsym(a.h, "ncclSend");
            a.recv = (int (*)(void*, size_t, int, int, void*, void*))dlsym(a.h, "ncclRecv");
            a.comm_init_rank = dlsym(a.h, "ncclCommInitRank");
        });
        if (!a.h || !a.get_unique_id || !a.send || !a.recv || !a.comm_destroy || !a.comm_init_rank)
            throw std::runtime_error("remote edge: librccl.so.1 not loadable");
        return a;
    }
    void ck(int r, const char* what)
    {
        if (r != 0)
            throw std::runtime_error(std::string("remote edge: ") + what + ": " +
                                     (lib().err_str ? lib().err_str(r) : std::to_string(r)));
    }

public:
    struct uid { // ncclUniqueId: 128 bytes, passed by value
        char b[128];
    };
    using init_fn = int (*)(void**, int, uid, int);

    rccl_transport(channel& ch, bool sender, int device) : _sender(sender)
    {
        auto& L = lib();
        hip::check(nsh_set_device(device), "remote edge: set device");
        uid id{};
        if (sender) {
            ck(L.get_unique_id(&id), "ncclGetUniqueId");
            ch.send_bytes(&id, sizeof(id));
        } else if (!ch.recv_bytes(&id, sizeof(id))) {
            throw std::runtime_error("remote edge: peer closed during RCCL setup");
        }
        auto init = reinterpret_cast<init_fn>(L.comm_init_rank);
        ck(init(&_comm, 2, id, sender ? 0 : 1), "ncclCommInitRank");
    }
    ~rccl_transport() override
    {
        if (_comm) lib().comm_destroy(_comm);
    }
    const char* kind() const override { return "rccl"; }
    void send(channel&, const void* p, size_t bytes) override
    {
        ck(lib().send(p, bytes, /*ncclInt8*/ 0, /*peer*/ 1, _comm, hip::current_stream()), "ncclSend");
    }
    void recv(channel&, void* p, size_t bytes) override
    {
        ck(lib().recv(p, bytes, /*ncclInt8*/ 0, /*peer*/ 0, _comm, hip::current_stream()), "ncclRecv");
    }

private:
    bool _sender;
    void* _comm = nullptr;
};

} // namespace remote

// ---- adapter ---------------------------------------------------------------------------
namespace {
// Port parent: wakes the receive thread when the downstream block frees ring space; other
// notifications crossing the adapter need no action (the sender forwards in post_write).
struct adapter_port_intf : neighbor_interface {
    std::mutex* m;
    std::condition_variable* cv;
    void push_message(scheduler_message_sptr) override
    {
        std::lock_guard<std::mutex> g(*m);
        cv->notify_all();
    }
};
std::mutex g_listen_m;
std::map<std::pair<int, int>, int>& listen_fds() // (port, crossing) -> listening fd
{
    static std::map<std::pair<int, int>, int> m;
    return m;
}
} // namespace

domain_adapter_remote::domain_adapter_remote(remote_role role, int crossing, const remote_edge_options& opt)
    : domain_adapter(buffer_location_t::LOCAL, role == remote_role::SEND ? "da_remote_send" : "da_remote_recv"),
      _role(role), _crossing(crossing), _opt(opt)
{
}

domain_adapter_remote::sptr domain_adapter_remote::make(remote_role role, port_sptr other_port, int crossing,
                                                        const remote_edge_options& opt)
{
    auto p = sptr(new domain_adapter_remote(role, crossing, opt));
    const bool faces_input = other_port->direction() == port_direction_t::INPUT;
    p->add_port(untyped_port::make(faces_input ? "output" : "input",
                                   faces_input ? port_direction_t::OUTPUT : port_direction_t::INPUT,
                                   other_port->itemsize()));
    auto intf = std::make_shared<adapter_port_intf>();
    intf->m = &p->_m;
    intf->cv = &p->_cv;
    for (auto& pt : p->all_ports()) pt->set_parent_intf(intf);
    p->_isz = other_port->itemsize();
    if (role == remote_role::RECV) {
        // listen now (partition time), accept later: the peer can connect whenever it
        // reaches this crossing, whatever order either process initialises its edges in
        const int port = opt.base_port + crossing;
        std::lock_guard<std::mutex> g(g_listen_m);
        auto key = std::make_pair(port, crossing);
        if (!listen_fds().count(key)) listen_fds()[key] = remote::listen_on(opt.host, port);
    }
    return p;
}

domain_adapter_remote::~domain_adapter_remote()
{
    if (_role == remote_role::SEND) {
        _closing.store(true);
        if (_thr.joinable()) _thr.join(); // setup
        if (_ch && _ready.load()) {
            try {
                _ch->send_msg(remote::M_CLOSE);
                _ch->shutdown_write();
                _ch->drain_until_eof(_opt.timeout_s); // receiver closes after CLOSE
            } catch (...) {
            }
        }
    } else if (_thr.joinable()) {
        // The receive thread ends at the sender's CLOSE (the sender may still be finishing
        // its run after this process's reader is done: keep consuming until then), or at
        // the timeout.
        const auto t0 = std::chrono::steady_clock::now();
        while (!_thread_done.load() &&
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < _opt.timeout_s)
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        _closing.store(true);
    }
    if (_ch) _ch->shutdown_both();
    {
        std::lock_guard<std::mutex> g(_m);
        _cv.notify_all();
    }
    if (_thr.joinable()) _thr.join();
    _tr.reset(); // RCCL communicator before the stream
    if (_scratch) {
        if (_stream)
            nsh_free(_scratch);
        else
            std::free(_scratch);
    }
    if (_stream) {
        nsh_stream_sync(_stream);
        nsh_stream_destroy(_stream);
    }
    if (_role == remote_role::RECV) {
        std::lock_guard<std::mutex> g(g_listen_m);
        auto key = std::make_pair(_opt.base_port + _crossing, _crossing);
        auto it = listen_fds().find(key);
        if (it != listen_fds().end()) {
            ::close(it->second);
            listen_fds().erase(it);
        }
    }
}

bool domain_adapter_remote::local_is_device_side() const
{
    auto hb = std::dynamic_pointer_cast<hip_buffer>(_buffer);
    if (!hb) return false;
    // SEND reads the ring, RECV writes it
    if (_role == remote_role::SEND) return hb->buffer_type() != hip_buffer_type::D2H;
    return hb->buffer_type() != hip_buffer_type::H2D;
}

std::string domain_adapter_remote::transport_kind() const { return _tr ? _tr->kind() : "unconnected"; }

void domain_adapter_remote::check_failed() const
{
    if (_failed.load()) {
        if (_err) std::rethrow_exception(_err);
        throw std::runtime_error("remote edge failed");
    }
}

void domain_adapter_remote::buffer_ready()
{
    if (!_buffer) throw std::runtime_error("domain_adapter_remote: no buffer");
    const bool dev_side = local_is_device_side();
    _device = _opt.device;
    if (auto hb = std::dynamic_pointer_cast<hip_buffer>(_buffer)) _device = hb->device();
    if (_device < 0 && dev_side) _device = hip::current_device();

    auto setup = [this, dev_side]() {
        using namespace remote;
        hello mine{};
        mine.magic = M_HELLO;
        mine.crossing = _crossing;
        mine.item_size = _isz;
        mine.is_device = dev_side ? 1 : 0;
        mine.device = _device;
        mine.want = _opt.transport == "rccl" ? 1 : _opt.transport == "socket" ? 2 : 0;
        if (dev_side && _device >= 0) hip::check(nsh_device_pci_id(_device, mine.pci, (int)sizeof(mine.pci)), "remote edge: pci id");
        hello peer{};
        if (_role == remote_role::SEND) {
            _ch = connect_retry(_opt.host, _opt.base_port + _crossing, _opt.timeout_s, _closing);
            _ch->send_bytes(&mine, sizeof(mine));
            if (!_ch->recv_bytes(&peer, sizeof(peer))) throw std::runtime_error("remote edge: peer closed in handshake");
            if (peer.magic != M_HELLO || peer.crossing != _crossing || peer.item_size != _isz)
                throw std::runtime_error("remote edge: handshake mismatch on crossing " + std::to_string(_crossing));
            _max_chunk = (int)peer.max_chunk;
            if (peer.chosen == 1)
                _tr = std::make_shared<rccl_transport>(*_ch, true, _device);
            else
                _tr = std::make_shared<socket_transport>(dev_side);
        } else {
            int lfd;
            {
                std::lock_guard<std::mutex> g(g_listen_m);
                lfd = listen_fds().at(std::make_pair(_opt.base_port + _crossing, _crossing));
            }
            _ch = accept_one(lfd, _opt.timeout_s);
            if (!_ch->recv_bytes(&peer, sizeof(peer))) throw std::runtime_error("remote edge: peer closed in handshake");
            if (peer.magic != M_HELLO || peer.crossing != _crossing || peer.item_size != _isz)
                throw std::runtime_error("remote edge: handshake mismatch on crossing " + std::to_string(_crossing));
            // messages must fit the empty ring in one contiguous span
            buffer_info_t wi{};
            _buffer->write_info(wi);
            mine.max_chunk = wi.n_items;
            peer.pci[sizeof(peer.pci) - 1] = 0;
            const bool rccl_ok = dev_side && peer.is_device && mine.pci[0] && peer.pci[0] &&
                                 std::strncmp(peer.pci, mine.pci, sizeof(mine.pci)) != 0;
            const int want = peer.want ? peer.want : mine.want;
            if (want == 1 && !rccl_ok)
                throw std::runtime_error("remote edge: rccl transport needs device rings on two different GPUs");
            mine.chosen = (want != 2 && rccl_ok) ? 1 : 2;
            _ch->send_bytes(&mine, sizeof(mine));
            _max_chunk = (int)mine.max_chunk;
            if (mine.chosen == 1) {
                _tr = std::make_shared<rccl_transport>(*_ch, false, _device);
            } else {
                _tr = std::make_shared<socket_transport>(dev_side);
            }
        }
        if (_max_chunk <= 0) throw std::runtime_error("remote edge: receiver ring has no space");
        _ready.store(true);
    };

    if (_role == remote_role::SEND) {
        _thr = std::thread([this, setup] {
            try {
                setup();
            } catch (...) {
                _err = std::current_exception();
                _failed.store(true);
            }
        });
    } else {
        _thr = std::thread([this, setup, dev_side] {
            try {
                if (dev_side) {
                    hip::check(nsh_stream_create(_device, &_stream), "remote edge: stream");
                    hip::bind_thread(_device, _stream);
                }
                setup();
                recv_loop();
            } catch (...) {
                if (!_closing.load()) {
                    _err = std::current_exception();
                    _failed.store(true);
                }
            }
            if (dev_side) hip::unbind_thread();
            _thread_done.store(true);
            notify_downstream(); // let a waiting reader observe the failure / end
        });
    }
}

void domain_adapter_remote::notify_downstream()
{
    try {
        for (auto& p : all_ports())
            p->notify_connected_ports(std::make_shared<scheduler_action>(scheduler_action_t::NOTIFY_INPUT, id()));
    } catch (const std::exception&) {
        // the downstream scheduler is already gone (flowgraph torn down): nothing to wake
    }
}

void domain_adapter_remote::recv_loop()
{
    using namespace remote;
    msg m{};
    while (!_closing.load()) {
        if (!_ch->recv_msg(m)) return; // peer closed
        if (m.type == M_CLOSE) {
            _ch->shutdown_both(); // the sender drains until EOF: release it now
            return;
        }
        if (m.type == M_DONE) {
            _remote_done.fetch_add(1);
            notify_downstream();
            continue;
        }
        if (m.type != M_DATA) throw std::runtime_error("remote edge: unexpected message");
        const int n = (int)m.n;
        const size_t bytes = (size_t)n * _isz;
        std::vector<tag_t> tags; // m.aux tags, offsets relative to this message's first item
        if (m.aux) {
            const uint32_t len = [&] {
                uint32_t l = 0;
                if (!_ch->recv_bytes(&l, sizeof(l))) throw std::runtime_error("remote edge: peer closed in tags");
                return l;
            }();
            std::string blob(len, '\0');
            if (len && !_ch->recv_bytes(&blob[0], len)) throw std::runtime_error("remote edge: peer closed in tags");
            reader rd{ blob };
            for (uint32_t k = 0; k < m.aux; ++k) {
                const uint64_t rel = rd.raw<uint64_t>();
                auto key = rd.pmt();
                auto value = rd.pmt();
                auto srcid = rd.pmt();
                tags.emplace_back(rel, std::move(key), std::move(value), std::move(srcid));
            }
        }
        // Data after the k-th DONE belongs to run k+1: it waits until this process has
        // started that run (so runs do not mix), then for n contiguous writable items, or
        // is discarded if this run's reader has already finished.
        const uint64_t data_run = _remote_done.load() + 1;
        void* dst = nullptr;
        for (;;) {
            if (_runs.load() < data_run) {
                std::unique_lock<std::mutex> l(_m);
                _cv.wait_for(l, std::chrono::milliseconds(1));
                if (_closing.load()) return;
                continue;
            }
            if (_reader_finished.load() >= data_run) break;
            buffer_info_t wi{};
            if (_buffer->write_info(wi) && wi.n_items >= n) {
                dst = wi.ptr;
                break;
            }
            std::unique_lock<std::mutex> l(_m);
            _cv.wait_for(l, std::chrono::milliseconds(1));
            if (_closing.load()) return;
        }
        if (!dst) { // reader finished: the bytes still have to be received
            if (_scratch_bytes < bytes) {
                if (_scratch) {
                    if (_stream)
                        nsh_free(_scratch);
                    else
                        std::free(_scratch);
                }
                _scratch = nullptr;
                if (_stream)
                    hip::check(nsh_malloc(_device, bytes, &_scratch), "remote edge: scratch");
                else
                    _scratch = std::malloc(bytes);
                _scratch_bytes = bytes;
            }
            _tr->recv(*_ch, _scratch, bytes);
            continue;
        }
        _tr->recv(*_ch, dst, bytes);
        const uint64_t w0 = _buffer->total_written(); // the items' absolute offsets start here
        for (auto& t : tags) {
            t.offset += w0;
            _buffer->add_tag(std::move(t));
        }
        _buffer->post_write(n);
        _moved.fetch_add((uint64_t)n);
        notify_downstream();
    }
}

void domain_adapter_remote::pump()
{
    if (_thr.joinable()) _thr.join(); // setup finished (first use)
    check_failed();
    for (;;) {
        buffer_info_t ri{};
        if (!_buffer->read_info(ri) || ri.n_items <= 0) break;
        const int m = std::min(ri.n_items, _max_chunk);
        // the tags of these m items travel in the same message (offsets relative to its first item)
        const uint64_t r0 = _buffer->total_read();
        const auto tags = _buffer->tags_in_window(0, (uint64_t)m);
        std::string blob;
        for (auto& t : tags) {
            remote::put_raw(blob, (uint64_t)(t.offset - r0));
            remote::put_pmt(blob, t.key);
            remote::put_pmt(blob, t.value);
            remote::put_pmt(blob, t.srcid);
        }
        _ch->send_msg_with(
            remote::M_DATA, (uint64_t)m,
            [&] {
                if (!tags.empty()) {
                    const uint32_t len = (uint32_t)blob.size();
                    _ch->send_bytes(&len, sizeof(len));
                    _ch->send_bytes(blob.data(), blob.size());
                }
                _tr->send(*_ch, ri.ptr, (size_t)m * _isz);
            },
            (uint32_t)tags.size());
        _buffer->prune_tags(m); // sent with their items
        _buffer->post_read(m);
        _moved.fetch_add((uint64_t)m);
    }
}

void domain_adapter_remote::poll_reverse()
{
    // only READER_DONE travels upstream; called on the sender's partition thread
    if (!_ready.load()) return;
    while (_ch->readable(0)) {
        remote::msg m{};
        if (!_ch->recv_msg(m)) return;
        if (m.type == remote::M_READER_DONE) _remote_done.fetch_add(1);
    }
}

// -- buffer interface --
void* domain_adapter_remote::read_ptr()
{
    check_failed();
    return _buffer->read_ptr();
}
void* domain_adapter_remote::write_ptr() { return _buffer->write_ptr(); }
bool domain_adapter_remote::read_info(buffer_info_t& i)
{
    check_failed();
    return _buffer->read_info(i);
}
bool domain_adapter_remote::write_info(buffer_info_t& i) { return _buffer->write_info(i); }
void domain_adapter_remote::post_read(int n) { _buffer->post_read(n); }
void domain_adapter_remote::post_write(int n)
{
    _buffer->post_write(n);
    if (_role == remote_role::SEND) pump();
}
void domain_adapter_remote::copy_items(buffer_sptr from, int n)
{
    _buffer->copy_items(std::move(from), n);
    if (_role == remote_role::SEND) pump();
}
void domain_adapter_remote::set_writer_done()
{
    _buffer->set_writer_done();
    if (_role == remote_role::SEND) {
        pump();
        _ch->send_msg(remote::M_DONE);
    }
}
void domain_adapter_remote::set_reader_done()
{
    _buffer->set_reader_done();
    if (_role == remote_role::RECV) _reader_finished.store(_runs.load());
    if (_role == remote_role::RECV && _ready.load() && !_failed.load()) {
        try {
            _ch->send_msg(remote::M_READER_DONE);
        } catch (...) {
        }
        std::lock_guard<std::mutex> g(_m);
        _cv.notify_all();
    }
}
bool domain_adapter_remote::writer_done() const
{
    if (_role == remote_role::SEND) return _buffer->writer_done();
    check_failed();
    return _remote_done.load() >= _runs.load();
}
bool domain_adapter_remote::reader_done() const
{
    if (_role == remote_role::RECV) return _buffer->reader_done();
    const_cast<domain_adapter_remote*>(this)->poll_reverse();
    return _remote_done.load() >= _runs.load();
}
void domain_adapter_remote::reset_flags()
{
    if (_buffer) _buffer->reset_flags();
    _runs.fetch_add(1);
}

domain_adapter_sptr domain_adapter_remote_conf::make_remote_adapter(port_sptr local_port, bool local_is_upstream,
                                                                    int crossing, const std::string& name)
{
    auto a = domain_adapter_remote::make(local_is_upstream ? remote_role::SEND : remote_role::RECV, local_port,
                                         crossing, _opt);
    if (!name.empty()) a->set_alias(name);
    _made.push_back(a);
    return a;
}

} // namespace gr
