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

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <set>
#include <cstdio>
#include <stdexcept>

namespace gr {
namespace remote {

namespace {
enum msg_type : uint32_t {
    M_HELLO = 0x4e534832u, // "NSH2": hellos carry role, pid and nonce

    M_DATA = 2,
    M_DONE = 3,
    M_READER_DONE = 4,
    M_CLOSE = 5,
    M_SLOT_FREE = 6 // p2p: receiver -> sender, landing slot n may be written again
};
struct msg {
    uint32_t type;
    uint32_t aux;
    uint64_t n;
};
// transport codes in hello.want / hello.chosen
enum tr_code : int32_t { T_AUTO = 0, T_RCCL = 1, T_SOCKET = 2, T_P2P = 3, T_DEFERRED_TEST = 4 };
struct hello {
    uint32_t magic;     // M_HELLO
    int32_t crossing;
    uint64_t item_size;
    int32_t is_device;  // this side's ring end is device memory
    int32_t device;
    int32_t want;       // tr_code (sender's request)
    int32_t chosen;     // receiver's answer (tr_code, never T_AUTO)
    int64_t max_chunk;  // receiver's answer: items per message
    char pci[32];       // PCI bus id of `device` ("" for host rings): ordinals differ per
                        // process under per-rank HIP_VISIBLE_DEVICES, bus ids do not
    int32_t role;       // R_SEND | R_RECV: a sender must hear a receiver, and vice versa
    int32_t pid;        // the writer's process (diagnostics: an echo carries our own pid)
    uint64_t nonce;     // remote_edge_options::nonce: both ends belong to one job
};
enum role_code : int32_t { R_SEND = 0x53454e44, R_RECV = 0x52454356 };
// p2p: the receiver's landing slots, sent after its hello; the sender answers with a u32
// status (0 = mapped)
struct p2p_offer {
    uint8_t handle[NSH_IPC_HANDLE_BYTES];
    uint32_t slots;
    uint32_t pad;
    uint64_t slot_bytes;
};
int32_t transport_code(const std::string& s)
{
    if (s == "auto") return T_AUTO;
    if (s == "rccl") return T_RCCL;
    if (s == "socket") return T_SOCKET;
    if (s == "p2p") return T_P2P;
    if (s == "deferred_test") return T_DEFERRED_TEST;
    throw std::invalid_argument("remote edge: unknown transport '" + s + "'");
}
using clk = std::chrono::steady_clock;
double since(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

// Test hooks are environment-gated; each one says so on stderr once per process when it acts.
void test_hook_notice(const char* var, const char* value)
{
    static std::mutex m;
    static std::set<std::string> seen;
    std::lock_guard<std::mutex> g(m);
    if (seen.insert(var).second) std::fprintf(stderr, "newsched remote edge: test hook %s=%s active\n", var, value);
}

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
    // close with a reset instead of FIN (no TIME_WAIT): for refused peers
    void reset_on_close()
    {
        linger l{ 1, 0 };
        setsockopt(_fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
    }
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

std::atomic<uint64_t> g_self_connects{ 0 };
std::atomic<uint64_t> g_peers_refused{ 0 };

// port 0: the kernel picks a free one; *bound receives the port actually bound
int listen_on(const std::string& host, int port, int* bound)
{
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw std::runtime_error("remote edge: socket");
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a = resolve(host, port);
    if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 8) != 0) {
        const int e = errno;
        ::close(fd);
        throw std::runtime_error("remote edge: cannot listen on " + host + ":" + std::to_string(port) + ": " +
                                 std::strerror(e));
    }
    sockaddr_in got{};
    socklen_t len = sizeof(got);
    if (::getsockname(fd, reinterpret_cast<sockaddr*>(&got), &len) != 0) {
        ::close(fd);
        throw std::runtime_error("remote edge: getsockname");
    }
    *bound = ntohs(got.sin_port);
    return fd;
}

std::shared_ptr<channel> accept_one(int lfd, double timeout_s, const std::atomic<bool>& cancel)
{
    const auto t0 = clk::now();
    for (;;) {
        pollfd pfd{ lfd, POLLIN, 0 };
        if (::poll(&pfd, 1, 100) > 0) break;
        if (cancel.load()) throw std::runtime_error("remote edge: cancelled");
        if (since(t0) > timeout_s) throw std::runtime_error("remote edge: no peer connected within the timeout");
    }
    const int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) throw std::runtime_error(std::string("remote edge: accept: ") + std::strerror(errno));
    return std::make_shared<channel>(fd);
}

// one hello from `ch` within timeout_s; false if none came (closed, timed out, truncated)
bool recv_hello(channel& ch, hello& h, double timeout_s, const std::atomic<bool>& cancel)
{
    const auto t0 = clk::now();
    while (!ch.readable(100)) {
        if (cancel.load() || since(t0) > timeout_s) return false;
    }
    try {
        return ch.recv_bytes(&h, sizeof(h));
    } catch (const std::exception&) {
        return false;
    }
}

// A socket whose local and peer addresses are equal is connected to itself: connect() to a
// port nobody listens on, from an ephemeral source port that happens to equal it, completes by
// TCP simultaneous open (GPUTEST_r04, rank 4 of the 8-rank C5 rehearsal).
bool connected_to_itself(int fd)
{
    sockaddr_in a{}, b{};
    socklen_t la = sizeof(a), lb = sizeof(b);
    if (::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &la) != 0 ||
        ::getpeername(fd, reinterpret_cast<sockaddr*>(&b), &lb) != 0)
        return false;
    return a.sin_addr.s_addr == b.sin_addr.s_addr && a.sin_port == b.sin_port;
}

// close without TIME_WAIT (RST): the port is free again at once for its rightful listener
void close_reset(int fd)
{
    linger l{ 1, 0 };
    setsockopt(fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
    ::close(fd);
}

// Test hook NSH_REMOTE_TEST_SELF_CONNECT: "1" = the first connect attempt binds its source to
// the destination address, which with nobody listening there yields a socket connected to
// itself (what an ephemeral source port equal to the destination does by chance); "hello" =
// the same, and the socket-level check below is skipped, so the hello's role check has to
// refuse the echo. Returns 0 (off), 1 or 2.
int self_connect_hook()
{
    const char* f = std::getenv("NSH_REMOTE_TEST_SELF_CONNECT");
    if (!f || !*f || *f == '0') return 0;
    test_hook_notice("NSH_REMOTE_TEST_SELF_CONNECT", f);
    return std::strcmp(f, "hello") == 0 ? 2 : 1;
}

// soft = true: at the timeout return nullptr instead of throwing (rendezvous mode re-reads the
// published port then: the entry may have been stale)
std::shared_ptr<channel> connect_retry(const std::string& host, int port, double timeout_s,
                                       const std::atomic<bool>& cancel, int& force_self, bool soft = false)
{
    const auto t0 = clk::now();
    const sockaddr_in a = resolve(host, port);
    for (;;) {
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) throw std::runtime_error("remote edge: socket");
        const int hook = force_self;
        if (hook) { // a bind failure means someone listens there: connect normally
            force_self = 0;
            int one = 1;
            setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            (void)::bind(fd, reinterpret_cast<const sockaddr*>(&a), sizeof(a));
        }
        if (::connect(fd, reinterpret_cast<const sockaddr*>(&a), sizeof(a)) == 0) {
            if (hook == 2 || !connected_to_itself(fd)) return std::make_shared<channel>(fd);
            g_self_connects.fetch_add(1);
            std::fprintf(stderr, "newsched remote edge: rejected a socket connected to itself (%s:%d); retrying\n",
                         host.c_str(), port);
            close_reset(fd);
        } else {
            ::close(fd);
        }
        if (cancel.load()) throw std::runtime_error("remote edge: cancelled");
        if (since(t0) > timeout_s) {
            if (soft) return nullptr;
            throw std::runtime_error("remote edge: cannot connect to " + host + ":" + std::to_string(port));
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

// ---- rendezvous files: <dir>/crossing<i> = "<port> <nonce>" ----------------------------
std::string rdv_path(const std::string& dir, int crossing) { return dir + "/crossing" + std::to_string(crossing); }

void rdv_publish(const std::string& dir, int crossing, int port, uint64_t nonce)
{
    const std::string p = rdv_path(dir, crossing);
    const std::string tmp = p + ".tmp." + std::to_string((long)::getpid());
    FILE* f = std::fopen(tmp.c_str(), "w");
    if (!f) throw std::runtime_error("remote edge: cannot write " + tmp + ": " + std::strerror(errno));
    std::fprintf(f, "%d %llu\n", port, (unsigned long long)nonce);
    const bool ok = std::fclose(f) == 0 && std::rename(tmp.c_str(), p.c_str()) == 0; // atomic publish
    if (!ok) throw std::runtime_error("remote edge: cannot publish " + p + ": " + std::strerror(errno));
}

// the port the receiver of `crossing` published for this job (waits for it; a file left by
// another job -- another nonce -- is waited past, it is replaced when this job's receiver
// publishes)
int rdv_lookup(const std::string& dir, int crossing, uint64_t nonce, double timeout_s, const std::atomic<bool>& cancel)
{
    const std::string p = rdv_path(dir, crossing);
    const auto t0 = clk::now();
    std::string seen;
    for (;;) {
        if (FILE* f = std::fopen(p.c_str(), "r")) {
            int port = 0;
            unsigned long long n = 0;
            const int k = std::fscanf(f, "%d %llu", &port, &n);
            std::fclose(f);
            if (k == 2 && port > 0 && port < 65536) {
                if ((uint64_t)n == nonce) return port;
                seen = " (" + p + " holds nonce " + std::to_string(n) + ", this job's is " + std::to_string(nonce) + ")";
            }
        }
        if (cancel.load()) throw std::runtime_error("remote edge: cancelled");
        if (since(t0) > timeout_s)
            throw std::runtime_error("remote edge: no receiver published crossing " + std::to_string(crossing) + " in " +
                                     dir + " within the timeout" + seen);
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

// "" if `peer` is the other end this side needs (role `want`, this job's nonce), else why not
std::string refuse_reason(const hello& peer, int32_t want, uint64_t nonce)
{
    if (peer.magic != M_HELLO) return "not a newsched remote-edge hello (magic)";
    if (peer.role != want) {
        if (peer.role == (want == R_SEND ? R_RECV : R_SEND) && peer.pid == (int32_t)::getpid() && want == R_RECV)
            return "the peer is this process's own sender (a socket connected to itself echoed our hello)";
        return std::string("the peer is a ") + (peer.role == R_SEND ? "sender" : peer.role == R_RECV ? "receiver" : "stranger") +
               " (pid " + std::to_string(peer.pid) + "), expected a " + (want == R_SEND ? "sender" : "receiver");
    }
    if (peer.nonce != nonce)
        return "the peer (pid " + std::to_string(peer.pid) + ") belongs to another job (nonce " + std::to_string(peer.nonce) +
               ", this job's is " + std::to_string(nonce) + ")";
    return "";
}
} // namespace

uint64_t self_connects_rejected() { return g_self_connects.load(); }
uint64_t peers_refused() { return g_peers_refused.load(); }

// ---- data transports -------------------------------------------------------------------
//
// Edge ordering (the one rule every transport follows, applied in domain_adapter_remote::pump):
// a DATA message's payload is the sender's ring span [p, p + bytes). send() either
//   * returns release::now: nothing reads the span after the next write into it. Either the
//     payload was consumed before send() returned (socket), or its read was enqueued on the
//     calling thread's stream (rccl, p2p): the upstream kernel that writes the span next is
//     launched on the same partition stream, after the read; a writer on another stream waits
//     for the event hip_buffer::post_read records there. The span is released at once, with no
//     host wait -- the early release of the RCCL path;
//   * or returns release::deferred: the payload is read later on another thread (the
//     host-memory test transport below, where no stream orders the writer); `done` runs on that
//     thread, in send order, once the read is complete, and only then is the span released.
// The DATA header itself may go out later than send() returns (p2p: when the copy has landed);
// send_control() keeps DONE / CLOSE behind every DATA message handed over before it.
class transport
{
public:
    enum class release { now, deferred };
    virtual ~transport() = default;
    virtual const char* kind() const = 0;
    virtual release send(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, const void* p, size_t bytes,
                         std::function<void()> done) = 0;
    virtual void send_control(channel& ch, uint32_t type) { ch.send_msg(type); }
    virtual void flush() {} // every message handed over so far is on the wire
    // sender: a reverse message owned by the transport (M_SLOT_FREE); false if not its own
    virtual bool on_reverse(const msg&) { return false; }
    // receiver: the payload of one DATA message into p (device or host, as the ring)
    virtual void recv(channel& ch, void* p, size_t bytes) = 0;
};

namespace {
// DATA header, then [u32 blob length][blob] when it has tags, then the payload
template <typename F>
void write_data(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, F&& payload)
{
    ch.send_msg_with(
        M_DATA, n,
        [&] {
            if (ntags) {
                const uint32_t len = (uint32_t)blob.size();
                ch.send_bytes(&len, sizeof(len));
                ch.send_bytes(blob.data(), blob.size());
            }
            payload();
        },
        ntags);
}

// FIFO of jobs run in order on one thread (deferred message sends); the first failure is kept
// and rethrown to the producer.
class outbox
{
public:
    outbox() : _thr([this] { loop(); }) {}
    ~outbox()
    {
        {
            std::lock_guard<std::mutex> g(_m);
            _stop = true;
        }
        _cv.notify_all();
        _thr.join();
    }
    void push(std::function<void()> job)
    {
        rethrow();
        {
            std::lock_guard<std::mutex> g(_m);
            _q.push_back(std::move(job));
        }
        _cv.notify_all();
    }
    void flush()
    {
        std::unique_lock<std::mutex> l(_m);
        _idle_cv.wait(l, [this] { return (_q.empty() && !_busy) || _err; });
        l.unlock();
        rethrow();
    }
    // the first failed job's exception, if any (a failed job skips every later one)
    void rethrow()
    {
        std::lock_guard<std::mutex> g(_m);
        if (_err) std::rethrow_exception(_err);
    }

private:
    void loop()
    {
        std::unique_lock<std::mutex> l(_m);
        for (;;) {
            _cv.wait(l, [this] { return _stop || !_q.empty(); });
            if (_q.empty()) return; // stop requested and drained
            auto job = std::move(_q.front());
            _q.pop_front();
            _busy = true;
            l.unlock();
            std::exception_ptr e;
            try {
                if (!_err) job();
            } catch (...) {
                e = std::current_exception();
            }
            l.lock();
            _busy = false;
            if (e && !_err) _err = e;
            _idle_cv.notify_all();
        }
    }
    std::mutex _m;
    std::condition_variable _cv, _idle_cv;
    std::deque<std::function<void()>> _q;
    bool _busy = false, _stop = false;
    std::exception_ptr _err;
    std::thread _thr;
};
} // namespace

// Bytes over the control socket. Device memory is staged through a pinned bounce buffer
// (one synchronous D2H/H2D per message): the path for host rings, and the fallback for
// device rings when neither RCCL nor the IPC mapping is available.
class socket_transport : public transport
{
public:
    explicit socket_transport(bool device) : _device(device) {}
    ~socket_transport() override
    {
        if (_bounce) nsh_host_free(_bounce);
    }
    const char* kind() const override { return _device ? "socket(staged)" : "socket"; }
    release send(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, const void* p, size_t bytes,
                 std::function<void()>) override
    {
        if (!_device) {
            write_data(ch, n, ntags, blob, [&] { ch.send_bytes(p, bytes); });
            return release::now;
        }
        ensure(bytes);
        void* s = hip::current_stream();
        hip::check(nsh_memcpy_async(_bounce, p, bytes, NSH_D2H, s), "remote edge: stage D2H");
        hip::check(nsh_stream_sync(s), "remote edge: stage sync");
        write_data(ch, n, ntags, blob, [&] { ch.send_bytes(_bounce, bytes); });
        return release::now;
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

// Test transport for host rings (transport "deferred_test"; CPU tests only): the payload is
// read from the ring span on a worker thread after a delay, as an asynchronous engine would,
// and the span is released only when that read is done (release::deferred). A checksum taken
// when send() is called is compared with the bytes the delayed read sees; any difference means
// the ring was overwritten before the transfer read it, and is counted
// (deferred_test_violations()). NSH_REMOTE_TEST_EARLY_RELEASE=1 makes it claim release::now
// instead: the negative control, which must produce violations.
class deferred_test_transport : public transport
{
public:
    deferred_test_transport()
    {
        const char* d = std::getenv("NSH_REMOTE_TEST_DELAY_US");
        _delay_us = d ? std::atoi(d) : 2000;
        const char* e = std::getenv("NSH_REMOTE_TEST_EARLY_RELEASE");
        _early = e && *e == '1';
        if (_early) test_hook_notice("NSH_REMOTE_TEST_EARLY_RELEASE", "1 (negative control: unsafe release)");
    }
    ~deferred_test_transport() override
    {
        try {
            _box.flush();
        } catch (...) {
        }
    }
    const char* kind() const override { return _early ? "deferred_test(early)" : "deferred_test"; }
    release send(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, const void* p, size_t bytes,
                 std::function<void()> done) override
    {
        const uint64_t sum0 = fnv(p, bytes);
        _box.push([this, &ch, n, ntags, blob, p, bytes, sum0, done = std::move(done)] {
            std::this_thread::sleep_for(std::chrono::microseconds(_delay_us));
            std::string copy(static_cast<const char*>(p), bytes); // the asynchronous read
            if (fnv(copy.data(), bytes) != sum0) g_violations.fetch_add(1);
            write_data(ch, n, ntags, blob, [&] { ch.send_bytes(copy.data(), bytes); });
            if (!_early) done();
        });
        return _early ? release::now : release::deferred;
    }
    void send_control(channel& ch, uint32_t type) override
    {
        _box.push([&ch, type] { ch.send_msg(type); });
    }
    void flush() override { _box.flush(); }
    void recv(channel& ch, void* p, size_t bytes) override
    {
        if (!ch.recv_bytes(p, bytes)) throw std::runtime_error("remote edge: peer closed");
    }
    static std::atomic<uint64_t> g_violations;

private:
    static uint64_t fnv(const void* p, size_t n)
    {
        uint64_t h = 1469598103934665603ull;
        auto* c = static_cast<const uint8_t*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
        return h;
    }
    int _delay_us;
    bool _early;
    outbox _box;
};
std::atomic<uint64_t> deferred_test_transport::g_violations{ 0 };
uint64_t deferred_test_violations() { return deferred_test_transport::g_violations.load(); }

// Device rings of two processes through an IPC-mapped landing area on the receiver's GPU:
// K slots of one message each. Sender: a stream-ordered copy from its ring span into a free
// slot (nsh_memcpy_async on the partition stream; same GPU: local D2D, two GPUs: a peer write
// over xGMI), an event behind it, release::now (the copy is stream-ordered before the next
// write into the span); the DATA header (with the slot number) goes out from the outbox
// thread once that event has completed, so the receiver never reads a slot before it landed.
// Receiver: one local D2D copy from the slot into its ring on its own stream, then
// M_SLOT_FREE(slot) once that copy is done. A sender with no free slot reads reverse messages
// until one comes back -- and fails instead of waiting forever when the outbox has failed (its
// DATA headers are then skipped, so no slot would ever be freed), the adapter is closing, or
// the receiver closed the channel (read_reverse throws); a merely backpressured receiver is
// waited for, unless remote_edge_options::stall_timeout_s sets a limit.
class p2p_transport : public transport
{
public:
    static constexpr uint32_t kSlots = 4;

    // receiver side: allocate and export the slots (throws if IPC export is unavailable)
    p2p_transport(int device, size_t slot_bytes, p2p_offer& offer) : _sender(false), _device(device), _slot_bytes(slot_bytes)
    {
        hip::check(nsh_malloc(device, slot_bytes * kSlots, &_local), "remote edge: p2p slots");
        if (nsh_ipc_mem_export(_local, offer.handle) != 0) {
            const std::string e = nsh_last_error();
            nsh_free(_local);
            _local = nullptr;
            throw std::runtime_error("remote edge: p2p export: " + e);
        }
        offer.slots = kSlots;
        offer.slot_bytes = slot_bytes;
    }
    // sender side: map the receiver's slots; read_reverse(block) reads and dispatches one
    // reverse message (false when none arrived)
    p2p_transport(int device, const p2p_offer& offer, std::function<bool()> read_reverse,
                  const std::atomic<bool>* closing, double timeout_s)
        : _sender(true), _device(device), _slot_bytes(offer.slot_bytes), _read_reverse(std::move(read_reverse)),
          _closing(closing), _timeout_s(timeout_s)
    {
        if (const char* f = std::getenv("NSH_REMOTE_TEST_FAIL_OUTBOX"); f && *f) { // test hook (see send)
            _fail_after = std::atoi(f);
            test_hook_notice("NSH_REMOTE_TEST_FAIL_OUTBOX", f);
        }
        if (offer.slots == 0 || offer.slots > 64) throw std::runtime_error("remote edge: p2p offer");
        hip::check(nsh_ipc_mem_open(device, offer.handle, &_remote), "remote edge: p2p map");
        _events.resize(offer.slots, nullptr);
        for (auto& e : _events) hip::check(nsh_event_create(&e), "remote edge: p2p event");
        for (uint32_t s = 0; s < offer.slots; ++s) _free.push_back(s);
        _box = std::make_unique<outbox>();
    }
    ~p2p_transport() override
    {
        if (_box) {
            try {
                _box->flush();
            } catch (...) {
            }
            _box.reset();
        }
        for (void* e : _events)
            if (e) nsh_event_destroy(e);
        if (_remote) nsh_ipc_mem_close(_remote);
        if (_local) nsh_free(_local);
    }
    const char* kind() const override { return "p2p"; }

    release send(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, const void* p, size_t bytes,
                 std::function<void()>) override
    {
        if (bytes > _slot_bytes) throw std::runtime_error("remote edge: p2p message larger than a slot");
        uint32_t slot;
        const auto t0 = clk::now();
        for (;;) {
            {
                std::lock_guard<std::mutex> g(_m);
                if (!_free.empty()) {
                    slot = _free.front();
                    _free.pop_front();
                    break;
                }
            }
            _box->rethrow(); // a failed DATA job: the receiver will never free a slot
            if (_closing && _closing->load()) throw std::runtime_error("remote edge: p2p send while closing");
            // a backpressured receiver (slow downstream) frees slots late, not never: only an
            // explicit stall limit ends the wait (remote_edge_options::stall_timeout_s)
            if (_timeout_s > 0 && since(t0) > _timeout_s)
                throw std::runtime_error("remote edge: p2p: no landing slot freed within stall_timeout_s");
            _read_reverse(); // blocks briefly for a reverse message (M_SLOT_FREE)
        }
        void* s = hip::current_stream();
        hip::check(nsh_memcpy_async(static_cast<char*>(_remote) + (size_t)slot * _slot_bytes, p, bytes, NSH_DEFAULT, s),
                   "remote edge: p2p copy");
        void* ev = _events[slot];
        hip::check(nsh_event_record(ev, s), "remote edge: p2p event");
        const bool fail = _fail_after >= 0 && _sent++ >= _fail_after; // test hook: this job fails
        _box->push([&ch, n, ntags, blob, ev, slot, fail] {
            if (fail) throw std::runtime_error("remote edge: p2p DATA job failed (NSH_REMOTE_TEST_FAIL_OUTBOX)");
            hip::check(nsh_event_sync(ev), "remote edge: p2p copy wait");
            write_data(ch, n, ntags, blob, [&] { ch.send_bytes(&slot, sizeof(slot)); });
        });
        return release::now;
    }
    void send_control(channel& ch, uint32_t type) override
    {
        _box->push([&ch, type] { ch.send_msg(type); });
    }
    void flush() override
    {
        if (_box) _box->flush();
    }
    bool on_reverse(const msg& m) override
    {
        if (m.type != M_SLOT_FREE) return false;
        std::lock_guard<std::mutex> g(_m);
        _free.push_back((uint32_t)m.n);
        return true;
    }
    void recv(channel& ch, void* p, size_t bytes) override
    {
        uint32_t slot = 0;
        if (!ch.recv_bytes(&slot, sizeof(slot))) throw std::runtime_error("remote edge: peer closed");
        if (slot >= kSlots || bytes > _slot_bytes) throw std::runtime_error("remote edge: bad p2p slot");
        void* s = hip::current_stream();
        hip::check(nsh_memcpy_async(p, static_cast<char*>(_local) + (size_t)slot * _slot_bytes, bytes, NSH_D2D, s),
                   "remote edge: p2p slot copy");
        hip::check(nsh_stream_sync(s), "remote edge: p2p slot copy wait");
        ch.send_msg(M_SLOT_FREE, slot);
    }

private:
    bool _sender;
    int _device;
    size_t _slot_bytes;
    std::function<bool()> _read_reverse;
    const std::atomic<bool>* _closing = nullptr;
    double _timeout_s = 0; // stall limit, 0 = none
    int _fail_after = -1; // test hook: DATA jobs from this one on fail
    int _sent = 0;
    void* _local = nullptr;  // receiver: the slots
    void* _remote = nullptr; // sender: the receiver's slots, mapped
    std::vector<void*> _events;
    std::mutex _m;
    std::deque<uint32_t> _free;
    std::unique_ptr<outbox> _box;
};

std::mutex g_rccl_path_m;
std::string g_rccl_path;

// RCCL point-to-point on the partition streams (device rings on different GPUs). librccl
// is loaded on first use so that host-only builds and tests do not need it, deliberately: the
// copy this process has already loaded if there is one (under torch that is torch's bundled
// librccl, built against the HIP runtime torch loaded -- libamdhip64.so.7 has one SONAME, so that
// is the runtime this library runs on too), else /opt/rocm's; the file actually bound is recorded
// (dladdr of ncclSend, domain_adapter_remote::rccl_library(), bench's c5_pipeline). Asynchronous
// communicator errors (ncclCommGetAsyncError) are checked before every call and at DONE / CLOSE,
// so a failed transfer is an error of fg->run(), not a hang. Test hook:
// NSH_RCCL_LIB names another library with the same five entry points (the tests load
// build/tests/libfake_rccl.so, tests/cpp/fake_rccl.c: payloads over a Unix socket, read and
// landed in stream order on device rings), and with NSH_REMOTE_TEST_RCCL=1 the receiver accepts
// "rccl" for any pair of rings, so this transport's protocol (id exchange, communicator per
// crossing, DATA header then the payload's send / recv on the partition / adapter streams,
// release at once, discarded messages still received, teardown) runs in the 2-process tests on
// the CPU (host rings) and on one GPU (device rings); the real library needs two GPUs.
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
        int (*async_error)(void*, int*) = nullptr; // ncclCommGetAsyncError (optional)
        int (*group_start)() = nullptr;            // ncclGroupStart / ncclGroupEnd (optional: the
        int (*group_end)() = nullptr;              // crossings never group; rccl_self_test does)
        std::string path;                          // the file ncclSend came from
    };
public:
    static api& lib()
    {
        static api a;
        static std::once_flag once;
        std::call_once(once, [] {
            if (const char* t = std::getenv("NSH_RCCL_LIB"); t && *t) {
                test_hook_notice("NSH_RCCL_LIB", t);
                a.h = dlopen(t, RTLD_NOW | RTLD_LOCAL); // test double (see above); no fallback
            } else {
                a.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD); // already in the process (torch's)
                if (!a.h) a.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
                if (!a.h) a.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            }
            if (!a.h) return;
            a.get_unique_id = (int (*)(void*))dlsym(a.h, "ncclGetUniqueId");
            a.comm_destroy = (int (*)(void*))dlsym(a.h, "ncclCommDestroy");
            a.err_str = (const char* (*)(int))dlsym(a.h, "ncclGetErrorString");
            a.send = (int (*)(const void*, size_t, int, int, void*, void*))dlsym(a.h, "ncclSend");
            a.recv = (int (*)(void*, size_t, int, int, void*, void*))dlsym(a.h, "ncclRecv");
            a.comm_init_rank = dlsym(a.h, "ncclCommInitRank");
            a.async_error = (int (*)(void*, int*))dlsym(a.h, "ncclCommGetAsyncError");
            a.group_start = (int (*)())dlsym(a.h, "ncclGroupStart");
            a.group_end = (int (*)())dlsym(a.h, "ncclGroupEnd");
            Dl_info di{};
            if (a.send && dladdr((void*)a.send, &di) && di.dli_fname) a.path = di.dli_fname;
            std::lock_guard<std::mutex> g(g_rccl_path_m);
            g_rccl_path = a.path;
        });
        if (!a.h || !a.get_unique_id || !a.send || !a.recv || !a.comm_destroy || !a.comm_init_rank)
            throw std::runtime_error("remote edge: librccl.so.1 not loadable");
        return a;
    }

private:
    void ck(int r, const char* what)
    {
        if (r != 0)
            throw std::runtime_error(std::string("remote edge: ") + what + ": " +
                                     (lib().err_str ? lib().err_str(r) : std::to_string(r)));
    }
    // an asynchronous failure of an earlier send / receive (ncclInProgress = 7 is not one)
    void check_async()
    {
        int e = 0;
        if (_comm && lib().async_error && lib().async_error(_comm, &e) == 0 && e != 0 && e != 7)
            ck(e, "asynchronous communicator error");
    }

public:
    struct uid { // ncclUniqueId: 128 bytes, passed by value
        char b[128];
    };
    using init_fn = int (*)(void**, int, uid, int);

    rccl_transport(channel& ch, bool sender, int device, bool dev_ring) : _sender(sender), _dev(dev_ring), _device(device)
    {
        auto& L = lib();
        if (_dev) hip::check(nsh_set_device(device), "remote edge: set device");
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
    release send(channel& ch, uint64_t n, uint32_t ntags, const std::string& blob, const void* p, size_t bytes,
                 std::function<void()>) override
    {
        check_async();
        check_span(p, "ncclSend");
        // header first: the receiver posts the matching ncclRecv when it reads it
        write_data(ch, n, ntags, blob, [] {});
        ck(lib().send(p, bytes, /*ncclInt8*/ 0, /*peer*/ 1, _comm, stream()), "ncclSend");
        return release::now;
    }
    void send_control(channel& ch, uint32_t type) override
    {
        // a run whose transfers failed must end in an error, not a DONE: at the end of a run the
        // sends are drained first (the partition stream: the flush that ends the run waits for it
        // anyway), so an asynchronous failure of any of them is seen here
        if (type == M_DONE && stream()) hip::check(nsh_stream_sync(stream()), "remote edge: rccl drain");
        check_async();
        ch.send_msg(type);
    }
    void recv(channel&, void* p, size_t bytes) override
    {
        check_async();
        check_span(p, "ncclRecv");
        ck(lib().recv(p, bytes, /*ncclInt8*/ 0, /*peer*/ 0, _comm, stream()), "ncclRecv");
    }

private:
    void* stream() const { return _dev ? hip::current_stream() : nullptr; }
    // a device-ring span handed to librccl must be device memory of this edge's GPU (VMM ring
    // mappings included; tests/test_rccl_real.py): anything else is this edge's error, not a
    // fault inside an RCCL kernel
    void check_span(const void* p, const char* what) const
    {
        if (!_dev || _device < 0) return;
        int d = -1;
        hip::check(nsh_pointer_device(p, &d), "remote edge: pointer attributes");
        if (d != _device)
            throw std::runtime_error(std::string("remote edge: ") + what + ": span is not device memory of GPU " +
                                     std::to_string(_device) + " (found " + std::to_string(d) + ")");
    }
    bool _sender;
    bool _dev; // device ring (always, but for the host-ring test double)
    int _device;
    void* _comm = nullptr;
};

} // namespace remote

std::string domain_adapter_remote::rccl_library()
{
    std::lock_guard<std::mutex> g(remote::g_rccl_path_m);
    return remote::g_rccl_path;
}

void domain_adapter_remote::rccl_self_test(int device, const void* src, void* dst, size_t bytes, void* stream, int peer)
{
    auto& L = remote::rccl_transport::lib(); // the crossings' own table: same dlopen order, same symbols
    auto ck = [&L](int r, const char* what) {
        if (r != 0)
            throw std::runtime_error(std::string("rccl_self_test: ") + what + ": " +
                                     (L.err_str ? L.err_str(r) : std::to_string(r)) + " (" + std::to_string(r) + ")");
    };
    if (!L.group_start || !L.group_end) throw std::runtime_error("rccl_self_test: ncclGroupStart/End not exported");
    // the buffers go to RCCL kernels: anything but device memory of this GPU is refused here,
    // before any RCCL call, instead of faulting inside one
    for (const void* p : { src, (const void*)dst }) {
        int d = -1;
        hip::check(nsh_pointer_device(p, &d), "rccl_self_test: pointer attributes");
        if (d != device)
            throw std::invalid_argument("rccl_self_test: buffer " + std::to_string((uintptr_t)p) +
                                        " is not device memory of GPU " + std::to_string(device) + " (found " +
                                        std::to_string(d) + ")");
    }
    hip::check(nsh_set_device(device), "rccl_self_test: set device");
    remote::rccl_transport::uid id{};
    ck(L.get_unique_id(&id), "ncclGetUniqueId");
    void* comm = nullptr;
    ck(reinterpret_cast<remote::rccl_transport::init_fn>(L.comm_init_rank)(&comm, 1, id, 0), "ncclCommInitRank(nranks=1)");
    std::string failure;
    try {
        ck(L.group_start(), "ncclGroupStart");
        const int rs = L.send(src, bytes, /*ncclInt8*/ 0, peer, comm, stream);
        const int rr = L.recv(dst, bytes, /*ncclInt8*/ 0, peer, comm, stream);
        const int re = L.group_end(); // always closed, whatever the two calls returned
        ck(rs, "ncclSend");
        ck(rr, "ncclRecv");
        ck(re, "ncclGroupEnd");
        hip::check(nsh_stream_sync(stream), "rccl_self_test: stream sync");
        int ae = 0;
        if (L.async_error) {
            ck(L.async_error(comm, &ae), "ncclCommGetAsyncError");
            ck(ae, "asynchronous communicator error");
        }
    } catch (const std::exception& e) {
        failure = e.what();
    }
    L.comm_destroy(comm);
    if (!failure.empty()) throw std::runtime_error(failure);
}

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
} // namespace

domain_adapter_remote::domain_adapter_remote(remote_role role, int crossing, const remote_edge_options& opt)
    : domain_adapter(buffer_location_t::LOCAL, role == remote_role::SEND ? "da_remote_send" : "da_remote_recv"),
      _role(role), _crossing(crossing), _opt(opt)
{
}

domain_adapter_remote::sptr domain_adapter_remote::make(remote_role role, port_sptr other_port, int crossing,
                                                        const remote_edge_options& opt)
{
    remote::transport_code(opt.transport); // unknown names fail here, not on the setup thread
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
        // reaches this crossing, whatever order either process initialises its edges in.
        // With a rendezvous directory the kernel picks the port (bound before anyone can
        // connect to it) and the sender learns it from the published file.
        const bool rdv = !opt.rendezvous_dir.empty();
        p->_lfd = remote::listen_on(opt.host, rdv ? 0 : opt.base_port + crossing, &p->_port);
        if (rdv) remote::rdv_publish(opt.rendezvous_dir, crossing, p->_port, opt.nonce);
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
                _tr->send_control(*_ch, remote::M_CLOSE); // behind every DATA / DONE still queued
                _tr->flush();
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
    if (_lfd >= 0) ::close(_lfd);
    if (_role == remote_role::RECV && !_opt.rendezvous_dir.empty()) {
        // withdraw this receiver's entry, unless another receiver has replaced it since
        const std::string p = remote::rdv_path(_opt.rendezvous_dir, _crossing);
        if (FILE* f = std::fopen(p.c_str(), "r")) {
            int port = 0;
            const bool mine = std::fscanf(f, "%d", &port) == 1 && port == _port;
            std::fclose(f);
            if (mine) ::unlink(p.c_str());
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
        mine.want = transport_code(_opt.transport);
        mine.role = _role == remote_role::SEND ? R_SEND : R_RECV;
        mine.pid = (int32_t)::getpid();
        mine.nonce = _opt.nonce;
        if (dev_side && _device >= 0) hip::check(nsh_device_pci_id(_device, mine.pci, (int)sizeof(mine.pci)), "remote edge: pci id");
        const std::string where = "remote edge: crossing " + std::to_string(_crossing);
        hello peer{};
        const auto t0 = clk::now();
        std::string last_refusal;
        // a peer that is not this crossing's other end: counted, said on stderr, dropped
        auto refused = [&](const std::string& why) {
            g_peers_refused.fetch_add(1);
            last_refusal = why;
            std::fprintf(stderr, "newsched %s: refused a peer: %s; retrying\n", where.c_str(), why.c_str());
        };
        auto out_of_time = [&] {
            return std::runtime_error(where + ": no valid " + (_role == remote_role::SEND ? "receiver" : "sender") +
                                      " within " + std::to_string((int)_opt.timeout_s) + " s" +
                                      (last_refusal.empty() ? "" : " (last peer refused: " + last_refusal + ")"));
        };
        if (_role == remote_role::SEND) {
            int force_self = self_connect_hook();
            for (;;) { // rendezvous, connect, hello; a wrong peer is dropped and the rendezvous retried
                const double left = _opt.timeout_s - since(t0);
                if (left <= 0) throw out_of_time();
                const bool rdv = !_opt.rendezvous_dir.empty();
                const int port = rdv ? rdv_lookup(_opt.rendezvous_dir, _crossing, _opt.nonce, left, _closing)
                                     : _opt.base_port + _crossing;
                // rendezvous: a published port nobody listens on may be a stale entry with this job's
                // nonce (a receiver that was re-created, or died before removing it): connect for a
                // short slice, then read the entry again -- a fresh receiver has republished it
                auto ch = connect_retry(_opt.host, port, rdv ? std::min(left, 1.0) : left, _closing, force_self, rdv);
                if (!ch) {
                    refused("nothing listens on published port " + std::to_string(port) + "; reading the entry again");
                    continue;
                }
                ch->send_bytes(&mine, sizeof(mine));
                if (!recv_hello(*ch, peer, _opt.timeout_s - since(t0), _closing)) {
                    if (_closing.load()) throw std::runtime_error("remote edge: cancelled");
                    refused("no hello from " + _opt.host + ":" + std::to_string(port));
                    continue;
                }
                const std::string why = refuse_reason(peer, R_RECV, _opt.nonce);
                if (why.empty()) {
                    _ch = std::move(ch);
                    break;
                }
                refused(why);
                ch->reset_on_close();
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
            // the right job and role: anything else that differs is a configuration error
            if (peer.crossing != _crossing || peer.item_size != _isz)
                throw std::runtime_error(where + ": handshake mismatch (peer crossing " + std::to_string(peer.crossing) +
                                         ", item size " + std::to_string(peer.item_size) + " vs " + std::to_string(_isz) + ")");
            _max_chunk = (int)peer.max_chunk;
            int32_t chosen = peer.chosen;
            if (chosen == T_P2P) {
                p2p_offer offer{};
                if (!_ch->recv_bytes(&offer, sizeof(offer))) throw std::runtime_error("remote edge: peer closed in p2p setup");
                uint32_t status = 0;
                std::string why;
                try {
                    _tr = std::make_shared<p2p_transport>(_device, offer, [this] { return read_reverse(100); }, &_closing,
                                                          _opt.stall_timeout_s);
                } catch (const std::exception& e) {
                    status = 1;
                    why = e.what();
                }
                _ch->send_bytes(&status, sizeof(status));
                if (status != 0) {
                    if (mine.want == T_P2P) throw std::runtime_error(why);
                    chosen = T_SOCKET; // auto: the receiver falls back with us
                }
            }
            if (chosen == T_RCCL)
                _tr = std::make_shared<rccl_transport>(*_ch, true, _device, dev_side);
            else if (chosen == T_DEFERRED_TEST)
                _tr = std::make_shared<deferred_test_transport>();
            else if (chosen == T_SOCKET)
                _tr = std::make_shared<socket_transport>(dev_side);
            else if (chosen != T_P2P)
                throw std::runtime_error(where + ": the receiver answered no transport (code " + std::to_string(chosen) + ")");
        } else {
            for (;;) { // accept until this crossing's sender says hello
                const double left = _opt.timeout_s - since(t0);
                if (left <= 0) throw out_of_time();
                auto ch = accept_one(_lfd, left, _closing);
                // a real sender says hello as soon as it connects: a client silent for 2 s is dropped,
                // so the accept loop reaches the next queued connection (the real sender waits in
                // the backlog for our hello meanwhile)
                if (!recv_hello(*ch, peer, std::min(_opt.timeout_s - since(t0), 2.0), _closing)) {
                    if (_closing.load()) throw std::runtime_error("remote edge: cancelled");
                    refused("a client connected and sent no hello within 2 s");
                    ch->reset_on_close();
                    continue;
                }
                const std::string why = refuse_reason(peer, R_SEND, _opt.nonce);
                if (why.empty()) {
                    _ch = std::move(ch);
                    break;
                }
                refused(why);
                ch->reset_on_close();
            }
            if (peer.crossing != _crossing || peer.item_size != _isz)
                throw std::runtime_error(where + ": handshake mismatch (peer crossing " + std::to_string(peer.crossing) +
                                         ", item size " + std::to_string(peer.item_size) + " vs " + std::to_string(_isz) + ")");
            // messages must fit the empty ring in one contiguous span
            buffer_info_t wi{};
            _buffer->write_info(wi);
            mine.max_chunk = wi.n_items;
            peer.pci[sizeof(peer.pci) - 1] = 0;
            // transport: rccl needs device rings on two GPUs (told apart by PCI bus id), p2p
            // device rings on one or two GPUs, deferred_test host rings; auto = rccl across
            // GPUs, p2p on one GPU, socket otherwise
            const bool both_dev = dev_side && peer.is_device && mine.pci[0] && peer.pci[0];
            const bool two_gpus = both_dev && std::strncmp(peer.pci, mine.pci, sizeof(mine.pci)) != 0;
            const int32_t want = peer.want ? peer.want : mine.want;
            // test hook: with the RCCL test double loaded (NSH_RCCL_LIB), NSH_REMOTE_TEST_RCCL=1 accepts rccl
            // without two PCI bus ids; the real library is never handed host rings or one GPU twice
            const char* tr = std::getenv("NSH_REMOTE_TEST_RCCL");
            const char* tl = std::getenv("NSH_RCCL_LIB");
            const bool rccl_test = tr && *tr == '1' && tl && *tl && dev_side == (peer.is_device != 0);
            if (tr && *tr == '1') test_hook_notice("NSH_REMOTE_TEST_RCCL", rccl_test ? "1 (accepted)" : "1 (ignored: NSH_RCCL_LIB unset)");
            if (want == T_RCCL && !two_gpus && !rccl_test)
                throw std::runtime_error("remote edge: rccl transport needs device rings on two different GPUs");
            if (want == T_P2P && !both_dev) throw std::runtime_error("remote edge: p2p transport needs device rings");
            if (want == T_DEFERRED_TEST && (dev_side || peer.is_device))
                throw std::runtime_error("remote edge: deferred_test transport needs host rings");
            mine.chosen = want != T_AUTO ? want : two_gpus ? T_RCCL : both_dev ? T_P2P : T_SOCKET;
            p2p_offer offer{};
            std::shared_ptr<p2p_transport> p2p;
            if (mine.chosen == T_P2P) {
                try {
                    p2p = std::make_shared<p2p_transport>(_device, (size_t)mine.max_chunk * _isz, offer);
                } catch (const std::exception&) {
                    if (want == T_P2P) throw;
                    mine.chosen = T_SOCKET; // auto: IPC export unavailable
                }
            }
            _ch->send_bytes(&mine, sizeof(mine));
            _max_chunk = (int)mine.max_chunk;
            if (mine.chosen == T_P2P) {
                _ch->send_bytes(&offer, sizeof(offer));
                uint32_t status = 1;
                if (!_ch->recv_bytes(&status, sizeof(status))) throw std::runtime_error("remote edge: peer closed in p2p setup");
                if (status == 0) {
                    _tr = p2p;
                } else {
                    if (want == T_P2P) throw std::runtime_error("remote edge: the sender could not map the p2p slots");
                    mine.chosen = T_SOCKET;
                }
            }
            if (mine.chosen == T_RCCL)
                _tr = std::make_shared<rccl_transport>(*_ch, false, _device, dev_side);
            else if (mine.chosen == T_DEFERRED_TEST)
                _tr = std::make_shared<deferred_test_transport>();
            else if (mine.chosen == T_SOCKET)
                _tr = std::make_shared<socket_transport>(dev_side);
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
        // is discarded if this run's reader has already finished. The ring is written under
        // _ring_m, which reset_flags takes to drop a finished run's unread items: a message
        // of the old run is either in the ring before that drop or goes to the discard area.
        const uint64_t data_run = _remote_done.load() + 1;
        bool placed = false;
        for (;;) {
            if (_runs.load() >= data_run) {
                std::lock_guard<std::mutex> w(_ring_m);
                if (_reader_finished.load() >= data_run) break; // discard below
                buffer_info_t wi{};
                if (_buffer->write_info(wi) && wi.n_items >= n) {
                    _tr->recv(*_ch, wi.ptr, bytes);
                    const uint64_t w0 = _buffer->total_written(); // the items' absolute offsets start here
                    for (auto& t : tags) {
                        t.offset += w0;
                        _buffer->add_tag(std::move(t));
                    }
                    _buffer->post_write(n);
                    placed = true;
                    break;
                }
            }
            std::unique_lock<std::mutex> l(_m);
            _cv.wait_for(l, std::chrono::milliseconds(1));
            if (_closing.load()) return;
        }
        if (placed) {
            _moved.fetch_add((uint64_t)n);
            notify_downstream();
            continue;
        }
        // reader finished: the bytes still have to be received
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
    }
}

// Forward everything readable in the local ring, one DATA message per contiguous span of at
// most _max_chunk items, and release each span by the edge ordering rule
// (remote::transport, above): at once when the transport's read of it is ordered before any
// later write (socket: consumed; rccl / p2p: enqueued on this partition stream), else when the
// transport reports the read done (release_span on its thread). Items handed to the transport
// but not yet released are skipped (_inflight).
void domain_adapter_remote::pump()
{
    if (_thr.joinable()) _thr.join(); // setup finished (first use)
    check_failed();
    try {
        pump_locked();
    } catch (...) { // a failed transfer fails the edge: no later call retries it
        _err = std::current_exception();
        _failed.store(true);
        throw;
    }
}

void domain_adapter_remote::pump_locked()
{
    std::lock_guard<std::mutex> g(_pump_m);
    for (;;) {
        buffer_info_t ri{};
        if (!_buffer->read_info(ri)) break;
        const int64_t avail = (int64_t)ri.n_items - (int64_t)_inflight;
        if (avail <= 0) break;
        const int m = (int)std::min<int64_t>(avail, _max_chunk);
        // the tags of these m items travel in the same message (offsets relative to its first item)
        const uint64_t r0 = _buffer->total_read() + _inflight;
        const auto tags = _buffer->tags_in_window(_inflight, _inflight + (uint64_t)m);
        std::string blob;
        for (auto& t : tags) {
            remote::put_raw(blob, (uint64_t)(t.offset - r0));
            remote::put_pmt(blob, t.key);
            remote::put_pmt(blob, t.value);
            remote::put_pmt(blob, t.srcid);
        }
        const void* p = static_cast<const char*>(ri.ptr) + _inflight * _isz;
        const auto how = _tr->send(*_ch, (uint64_t)m, (uint32_t)tags.size(), blob, p, (size_t)m * _isz,
                                   [this, m] { release_span(m, true); });
        if (how == remote::transport::release::now)
            release_span(m, false);
        else
            _inflight += (uint64_t)m;
        _moved.fetch_add((uint64_t)m);
    }
}

// The oldest m forwarded items leave the ring: their tags went with them. `deferred`: called on
// the transport's thread once its read completed (wakes the upstream block, which may be
// waiting for space); else on the partition thread inside pump().
void domain_adapter_remote::release_span(int m, bool deferred)
{
    std::unique_lock<std::mutex> g(_pump_m, std::defer_lock);
    if (deferred) g.lock();
    _buffer->prune_tags(m);
    _buffer->post_read(m);
    if (!deferred) return;
    _inflight -= (uint64_t)m;
    g.unlock();
    try {
        for (auto& p : all_ports())
            p->notify_connected_ports(std::make_shared<scheduler_action>(scheduler_action_t::NOTIFY_OUTPUT, id()));
    } catch (const std::exception&) {
    }
}

// SEND: handle one reverse message if one arrives within timeout_ms (READER_DONE, or a message
// the transport owns, e.g. p2p's M_SLOT_FREE). Returns whether one was handled.
bool domain_adapter_remote::read_reverse(int timeout_ms)
{
    std::lock_guard<std::mutex> g(_rev_m);
    if (!_ch->readable(timeout_ms)) return false;
    remote::msg m{};
    if (!_ch->recv_msg(m)) throw std::runtime_error("remote edge: receiver closed");
    if (m.type == remote::M_READER_DONE)
        _remote_done.fetch_add(1);
    else if (!_tr || !_tr->on_reverse(m))
        throw std::runtime_error("remote edge: unexpected reverse message");
    return true;
}

void domain_adapter_remote::poll_reverse()
{
    // called on the sender's partition thread (reader_done)
    if (!_ready.load()) return;
    try {
        while (read_reverse(0)) {
        }
    } catch (const std::exception&) {
        // receiver gone: its READER_DONE / DONE bookkeeping no longer matters
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
    if (_role == remote_role::SEND && !_failed.load()) { // a failed edge has nothing left to send
        pump();
        _tr->send_control(*_ch, remote::M_DONE); // behind this run's DATA messages
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
// A new run (prepare_run, every thread of the last run finished). The previous run's unread
// items and their tags are dropped here, before _runs moves on: a RECV ring may hold the
// remainder a decimator left below one output, and the receive thread starts writing the next
// run's data into the ring as soon as _runs is bumped (the remote counterpart of
// buffer::discard_unread, which prepare_run calls after reset_flags). A SEND side first lets
// its transport finish the last run's messages (deferred releases included).
void domain_adapter_remote::reset_flags()
{
    if (_role == remote_role::SEND && _ready.load() && _tr) _tr->flush(); // _ready first: _tr is set before it
    std::lock_guard<std::mutex> w(_ring_m);
    if (_buffer) {
        _buffer->reset_flags();
        _buffer->discard_unread();
    }
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
