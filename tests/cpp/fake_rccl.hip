// Test double of the RCCL entry points gr::domain_adapter_remote's "rccl" transport calls
// (newsched_amd/runtime/lib/domain_adapter_remote.cpp, rccl_transport), for multi-process tests of
// that transport without two GPUs (tests/test_remote_edge.py, tests/test_bench.py; loaded through
// NSH_RCCL_LIB with NSH_REMOTE_TEST_RCCL=1). Not RCCL: two ranks, one Unix-domain stream socket per
// communicator (abstract namespace, named by the unique id), one direction per communicator (rank
// 0 sends, rank 1 receives -- how the transport uses it).
//
// Rendezvous, as RCCL's point-to-point kernels behave on device rings (stream != NULL):
//   ncclSend  enqueues on the caller's stream a gate kernel that holds the stream until the peer's
//             matching receive has been reached on the PEER's stream, then the payload's D2H read
//             into pinned staging; returns at once. A worker thread takes the sends in call order:
//             waits for the peer's READY(seq), opens the gate, waits for the read and sends the
//             bytes. So the sender's partition stream stalls inside ncclSend while the receiver
//             has not posted (or its stream has not reached) the receive -- a full receiving ring
//             or a slow sink holds the sender's stream, as with RCCL.
//   ncclRecv  enqueues on the caller's stream a gate kernel that first marks "reached" (a system-
//             scope store to host memory) and then holds the stream until the payload has landed
//             in pinned staging, then the H2D into the ring; returns at once (asynchronous, as
//             RCCL's). A worker thread takes the receives in call order: waits until the stream
//             has reached the gate, sends READY(seq), receives the bytes, opens the gate.
// Host rings (stream NULL, CPU tests): no stream to order against, so both calls complete before
// they return -- ncclSend waits for READY(seq) and sends, ncclRecv sends READY and receives: the
// calling thread is what the rendezvous holds.
//
// Every wait is bounded (FAKE_RCCL_TIMEOUT_S, default 60 s; the gate kernel by the device's
// real-time counter): a rendezvous that never completes fails the communicator ("rendezvous timed
// out", ncclCommGetAsyncError and every later call report it) instead of hanging the GPU, and the
// gates are opened so every stream drains. FAKE_RCCL_MISORDER=1 is the negative control: the
// receiver posts READY only after its payload arrived, which a rendezvous can never satisfy, so
// the first message times out (with the pre-round-4 double, which never blocked the sender, the
// same mis-order passed). fake_rccl_stats() reports how long sends waited for their receive.
//
// Pinned staging and flags are pooled per communicator and freed only at ncclCommDestroy:
// hipHostFree synchronises the device, which would wait on a gate this very thread has to open.
#include <hip/hip_runtime.h>

#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace {

struct ncclUniqueId {
    char internal[128];
};

enum { OK = 0, E_SYS = 2, E_ARG = 4, E_TIMEOUT = 5 };

double timeout_s()
{
    const char* v = std::getenv("FAKE_RCCL_TIMEOUT_S");
    const double t = v ? std::atof(v) : 60.0;
    return t > 0 ? t : 60.0;
}
bool misorder()
{
    const char* v = std::getenv("FAKE_RCCL_MISORDER");
    return v && *v == '1';
}
using clk = std::chrono::steady_clock;
double since(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

// The gate: lane 0 marks `reached` (receives), then waits for `gate`; gives up after `ticks` of the
// 100 MHz real-time counter and records that in `status` (every wave exits: nothing outlives it).
__global__ void k_gate(unsigned* reached, unsigned* gate, unsigned* status, unsigned long long ticks)
{
    if (threadIdx.x != 0) return;
    if (reached) __hip_atomic_store(reached, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(32);
    }
}

std::atomic<uint64_t> g_sends{ 0 }, g_waited{ 0 }, g_max_wait_us{ 0 };
void note_wait(double s)
{
    const uint64_t us = (uint64_t)(s * 1e6);
    g_sends.fetch_add(1);
    if (us > 200) g_waited.fetch_add(1);
    uint64_t m = g_max_wait_us.load();
    while (us > m && !g_max_wait_us.compare_exchange_weak(m, us)) {
    }
}

struct op {
    uint64_t seq = 0;
    size_t n = 0;
    bool dev = false;
    unsigned* flags = nullptr; // pinned, coherent: [0] reached, [1] gate, [2] gate timed out
    char* staging = nullptr;   // pinned (device rings) / heap (host rings)
    size_t cap = 0;
    hipEvent_t ev = nullptr;   // behind the stream's copy
    clk::time_point posted;
};

struct fcomm {
    int fd = -1;
    int rank = 0;
    int dir = 0; // 1 send, 2 recv (fixed by the first call)
    std::mutex m;
    std::condition_variable cv;
    std::deque<op*> q;
    std::vector<op*> pool;    // finished ops, their pinned memory reusable
    std::vector<op*> retired; // device receives whose H2D may still be running
    std::thread worker;
    bool stop = false;
    std::atomic<int> err{ OK };
    uint64_t next_seq = 0;
    double tmo = 60.0;

    void fail(int code, const char* what, uint64_t seq)
    {
        int expect = OK;
        if (err.compare_exchange_strong(expect, code))
            std::fprintf(stderr, "fake rccl: rank %d: %s (message %llu)\n", rank, what, (unsigned long long)seq);
    }
};

void open_gate(op* o) { __atomic_store_n(&o->flags[1], 1u, __ATOMIC_SEQ_CST); } // host side

// a pooled op with room for n bytes (pinned memory for device rings)
op* take_op(fcomm* c, size_t n, bool dev)
{
    op* o = nullptr;
    {
        std::lock_guard<std::mutex> g(c->m);
        for (size_t i = 0; i < c->pool.size(); ++i)
            if (c->pool[i]->dev == dev && c->pool[i]->cap >= n) {
                o = c->pool[i];
                c->pool.erase(c->pool.begin() + (long)i);
                break;
            }
    }
    if (!o) {
        o = new op();
        o->dev = dev;
        o->cap = n ? n : 1;
        if (dev) {
            if (hipHostMalloc((void**)&o->flags, 64, hipHostMallocCoherent) != hipSuccess ||
                hipHostMalloc((void**)&o->staging, o->cap, 0) != hipSuccess ||
                hipEventCreateWithFlags(&o->ev, hipEventDisableTiming) != hipSuccess) {
                delete o; // (the partial allocation is leaked: a test double out of pinned memory)
                return nullptr;
            }
        } else {
            o->staging = (char*)std::malloc(o->cap);
            if (!o->staging) {
                delete o;
                return nullptr;
            }
        }
    }
    o->n = n;
    if (o->flags) {
        o->flags[0] = o->flags[1] = o->flags[2] = 0u;
        std::atomic_thread_fence(std::memory_order_seq_cst);
    }
    return o;
}
void give_back(fcomm* c, op* o)
{
    std::lock_guard<std::mutex> g(c->m);
    c->pool.push_back(o);
}

// bounded socket I/O; false on timeout or error
bool send_all(int fd, const void* p, size_t n, double tmo)
{
    auto* b = static_cast<const char*>(p);
    const auto t0 = clk::now();
    while (n) {
        pollfd pfd{ fd, POLLOUT, 0 };
        if (::poll(&pfd, 1, 100) <= 0) {
            if (since(t0) > tmo) return false;
            continue;
        }
        const ssize_t w = ::send(fd, b, n, MSG_NOSIGNAL | MSG_DONTWAIT);
        if (w > 0) {
            b += w;
            n -= (size_t)w;
        } else if (w < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) {
            continue;
        } else {
            return false;
        }
    }
    return true;
}
bool recv_all(int fd, void* p, size_t n, double tmo)
{
    auto* b = static_cast<char*>(p);
    const auto t0 = clk::now();
    while (n) {
        pollfd pfd{ fd, POLLIN, 0 };
        if (::poll(&pfd, 1, 100) <= 0) {
            if (since(t0) > tmo) return false;
            continue;
        }
        const ssize_t r = ::recv(fd, b, n, MSG_DONTWAIT);
        if (r > 0) {
            b += r;
            n -= (size_t)r;
        } else if (r < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) {
            continue;
        } else {
            return false; // peer closed or error
        }
    }
    return true;
}

// Sender worker: per send, READY(seq) from the peer, then the gate, the staged read, the bytes.
void send_one(fcomm* c, op* o)
{
    if (c->err.load() == OK) {
        uint64_t ready = ~0ull;
        if (!recv_all(c->fd, &ready, sizeof(ready), c->tmo))
            c->fail(E_TIMEOUT, "rendezvous timed out: the peer never posted the matching receive", o->seq);
        else if (ready != o->seq)
            c->fail(E_SYS, "rendezvous out of order", o->seq);
        else
            note_wait(since(o->posted));
    }
    if (o->dev) {
        open_gate(o); // on failure too: the stream must drain
        if (hipEventSynchronize(o->ev) != hipSuccess) c->fail(E_SYS, "staged read failed", o->seq);
        if (o->flags[2]) c->fail(E_TIMEOUT, "rendezvous timed out on the device gate", o->seq);
    }
    if (c->err.load() == OK && !send_all(c->fd, o->staging, o->n, c->tmo)) c->fail(E_SYS, "payload send failed", o->seq);
    give_back(c, o);
}

// Receiver worker (device rings): wait until the stream reached the receive, READY, the bytes, gate.
void reap(fcomm* c, bool wait);
void recv_one(fcomm* c, op* o)
{
    reap(c, false);
    if (c->err.load() == OK) {
        const auto t0 = clk::now();
        while (__atomic_load_n(&o->flags[0], __ATOMIC_ACQUIRE) == 0u) {
            if (since(t0) > c->tmo) {
                c->fail(E_TIMEOUT, "rendezvous timed out: the receiving stream never reached the receive", o->seq);
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    const bool mis = misorder();
    if (c->err.load() == OK && !mis && !send_all(c->fd, &o->seq, sizeof(o->seq), c->tmo))
        c->fail(E_SYS, "READY send failed", o->seq);
    if (c->err.load() == OK && !recv_all(c->fd, o->staging, o->n, c->tmo))
        c->fail(E_TIMEOUT, "rendezvous timed out: the payload never arrived", o->seq);
    if (c->err.load() == OK && mis) (void)send_all(c->fd, &o->seq, sizeof(o->seq), c->tmo); // too late
    open_gate(o);
    std::lock_guard<std::mutex> g(c->m);
    c->retired.push_back(o);
}

// receives whose H2D has completed go back to the pool
void reap(fcomm* c, bool wait)
{
    std::vector<op*> done, keep;
    {
        std::lock_guard<std::mutex> g(c->m);
        for (op* o : c->retired) {
            const hipError_t q = wait ? hipEventSynchronize(o->ev) : hipEventQuery(o->ev);
            (q == hipErrorNotReady ? keep : done).push_back(o);
        }
        c->retired.swap(keep);
        for (op* o : done) c->pool.push_back(o);
    }
}

void worker_main(fcomm* c)
{
    for (;;) {
        op* o = nullptr;
        {
            std::unique_lock<std::mutex> l(c->m);
            c->cv.wait_for(l, std::chrono::milliseconds(5), [c] { return c->stop || !c->q.empty(); });
            if (!c->q.empty()) {
                o = c->q.front();
                c->q.pop_front();
            } else if (c->stop) {
                return;
            }
        }
        if (!o) {
            if (c->dir == 2) reap(c, false);
            continue;
        }
        if (c->dir == 1)
            send_one(c, o);
        else
            recv_one(c, o);
    }
}

void sock_name(const ncclUniqueId* id, sockaddr_un* a, socklen_t* len)
{
    std::memset(a, 0, sizeof(*a));
    a->sun_family = AF_UNIX;
    const size_t n = strnlen(id->internal, sizeof(a->sun_path) - 2);
    std::memcpy(a->sun_path + 1, id->internal, n); // abstract: leading NUL, no file
    *len = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + n);
}

int set_dir(fcomm* c, int dir)
{
    if (c->dir == 0) c->dir = dir;
    return c->dir == dir ? OK : E_ARG;
}

void enqueue(fcomm* c, op* o)
{
    std::lock_guard<std::mutex> g(c->m);
    c->q.push_back(o);
    c->cv.notify_all();
}

} // namespace

extern "C" {

int ncclGetUniqueId(ncclUniqueId* id)
{
    static std::atomic<int> counter{ 0 };
    const auto ns = std::chrono::steady_clock::now().time_since_epoch().count();
    std::memset(id, 0, sizeof(*id));
    std::snprintf(id->internal, sizeof(id->internal), "nsh_fake_rccl_%d_%lld_%d", (int)getpid(), (long long)ns,
                  counter.fetch_add(1));
    return OK;
}

int ncclCommInitRank(void** comm, int nranks, ncclUniqueId id, int rank)
{
    if (!comm || nranks != 2 || rank < 0 || rank > 1) return E_ARG;
    sockaddr_un a;
    socklen_t len;
    sock_name(&id, &a, &len);
    const double tmo = timeout_s();
    int fd = -1;
    if (rank == 0) {
        const int l = ::socket(AF_UNIX, SOCK_STREAM, 0);
        if (l < 0) return E_SYS;
        if (::bind(l, (sockaddr*)&a, len) != 0 || ::listen(l, 1) != 0) {
            ::close(l);
            return E_SYS;
        }
        pollfd pfd{ l, POLLIN, 0 };
        if (::poll(&pfd, 1, (int)(tmo * 1000)) > 0) fd = ::accept(l, nullptr, nullptr);
        ::close(l);
    } else {
        const auto t0 = clk::now();
        while (since(t0) < tmo) {
            fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
            if (fd < 0) return E_SYS;
            if (::connect(fd, (sockaddr*)&a, len) == 0) break;
            ::close(fd);
            fd = -1;
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
    }
    if (fd < 0) return E_SYS;
    auto* c = new fcomm();
    c->fd = fd;
    c->rank = rank;
    c->tmo = tmo;
    c->worker = std::thread(worker_main, c);
    *comm = c;
    return OK;
}

int ncclSend(const void* buf, size_t count, int datatype, int peer, void* comm, void* stream)
{
    auto* c = static_cast<fcomm*>(comm);
    if (!c || datatype != 0 || peer != 1 - c->rank || (!buf && count) || set_dir(c, 1) != OK) return E_ARG;
    if (const int e = c->err.load()) return e;
    if (!stream) { // host ring: synchronous rendezvous
        const uint64_t seq = c->next_seq++;
        const auto t0 = clk::now();
        uint64_t ready = ~0ull;
        if (!recv_all(c->fd, &ready, sizeof(ready), c->tmo)) {
            c->fail(E_TIMEOUT, "rendezvous timed out: the peer never posted the matching receive", seq);
            return c->err.load();
        }
        if (ready != seq) {
            c->fail(E_SYS, "rendezvous out of order", seq);
            return c->err.load();
        }
        note_wait(since(t0));
        if (!send_all(c->fd, buf, count, c->tmo)) {
            c->fail(E_SYS, "payload send failed", seq);
            return c->err.load();
        }
        return OK;
    }
    op* o = take_op(c, count, true);
    if (!o) return E_SYS;
    o->seq = c->next_seq++;
    o->posted = clk::now();
    {
        const auto s = static_cast<hipStream_t>(stream);
        const unsigned long long ticks = (unsigned long long)(c->tmo * 1e8); // s_memrealtime: 100 MHz
        hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, (unsigned*)nullptr, &o->flags[1], &o->flags[2], ticks);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(o->staging, buf, count, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(o->ev, s) != hipSuccess) {
            open_gate(o);
            return E_SYS;
        }
    }
    enqueue(c, o);
    return OK;
}

int ncclRecv(void* buf, size_t count, int datatype, int peer, void* comm, void* stream)
{
    auto* c = static_cast<fcomm*>(comm);
    if (!c || datatype != 0 || peer != 1 - c->rank || (!buf && count) || set_dir(c, 2) != OK) return E_ARG;
    if (const int e = c->err.load()) return e;
    const uint64_t seq = c->next_seq++;
    if (!stream) { // host ring: synchronous
        if (!misorder() && !send_all(c->fd, &seq, sizeof(seq), c->tmo)) {
            c->fail(E_SYS, "READY send failed", seq);
            return c->err.load();
        }
        if (!recv_all(c->fd, buf, count, c->tmo)) {
            c->fail(E_TIMEOUT, "rendezvous timed out: the payload never arrived", seq);
            return c->err.load();
        }
        if (misorder()) (void)send_all(c->fd, &seq, sizeof(seq), c->tmo);
        return OK;
    }
    op* o = take_op(c, count, true);
    if (!o) return E_SYS;
    o->seq = seq;
    o->posted = clk::now();
    const auto s = static_cast<hipStream_t>(stream);
    const unsigned long long ticks = (unsigned long long)(c->tmo * 1e8);
    hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, s, &o->flags[0], &o->flags[1], &o->flags[2], ticks);
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(buf, o->staging, count, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipEventRecord(o->ev, s) != hipSuccess) {
        open_gate(o);
        return E_SYS;
    }
    enqueue(c, o);
    return OK;
}

int ncclCommGetAsyncError(void* comm, int* async_error)
{
    auto* c = static_cast<fcomm*>(comm);
    if (!c || !async_error) return E_ARG;
    *async_error = c->err.load();
    return OK;
}

int ncclCommDestroy(void* comm)
{
    auto* c = static_cast<fcomm*>(comm);
    if (!c) return OK;
    {
        std::lock_guard<std::mutex> g(c->m);
        c->stop = true;
        c->cv.notify_all();
    }
    c->worker.join(); // finishes the queued messages (each bounded)
    reap(c, true);
    ::close(c->fd);
    for (op* o : c->pool) {
        if (o->dev) {
            (void)hipEventDestroy(o->ev);
            (void)hipHostFree(o->flags);
            (void)hipHostFree(o->staging);
        } else {
            std::free(o->staging);
        }
        delete o;
    }
    delete c;
    return OK;
}

const char* ncclGetErrorString(int r)
{
    switch (r) {
    case OK: return "fake rccl: ok";
    case E_ARG: return "fake rccl: invalid argument";
    case E_TIMEOUT: return "fake rccl: rendezvous timed out";
    default: return "fake rccl: system error (peer gone?)";
    }
}

// test probe: sends completed, sends that waited > 200 us for their receive, the longest wait
void fake_rccl_stats(unsigned long long* sends, unsigned long long* waited, unsigned long long* max_wait_us)
{
    if (sends) *sends = g_sends.load();
    if (waited) *waited = g_waited.load();
    if (max_wait_us) *max_wait_us = g_max_wait_us.load();
}

} // extern "C"
