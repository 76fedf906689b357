// Cross-process domain adapters: one flowgraph partitioned over several processes (one
// per GPU), with every edge between domains of different processes carried by a
// point-to-point channel.
//
// The reference partitions a flowgraph only within one process
// (runtime/lib/graph_utils.cpp:11-205 + domain_adapter_direct.hpp:10-258; its
// domain_adapter.hpp:13-97 already names LOCAL/REMOTE buffer locations and a request
// protocol for the purpose). Here each process builds the SAME flowgraph and the SAME
// domain_conf list (SPMD), marks the domains that live elsewhere with remote_domain, and
// calls flowgraph::partition: graph_utils then instantiates only the local half of every
// crossing edge whose other end is remote:
//
//   process A:  blk_a -> [da_remote SEND] ~~~~ control: TCP (counts, done flags)
//   process B:                        ~~~~~> [da_remote RECV] -> blk_b
//                                     data:  rccl   ncclSend/ncclRecv on the partition streams
//                                                   (device rings on different GPUs)
//                                            p2p    stream-ordered copy into IPC-mapped landing
//                                                   slots on the receiver's GPU (device rings,
//                                                   same GPU or two GPUs)
//                                            socket the TCP socket (host rings; device rings
//                                                   staged through pinned memory)
//
// Rendezvous (how a sender finds its receiver). With `rendezvous_dir` set (the normal case):
// the receiver binds an ephemeral port chosen by the kernel when its adapter is made
// (partition time), then publishes "<port> <nonce>" in <rendezvous_dir>/crossing<i>
// (write + rename, atomic); the sender waits for that file and only then connects, so it
// never connects to a port nobody listens on. Without it, crossing i uses the fixed port
// base_port + i (pick one outside ip_local_port_range). Either way the connection is
// checked before use: a socket connected to itself (TCP simultaneous open when the sender's
// source port equals the destination port and no listener exists yet) is rejected and the
// connect retried; the hellos carry the role (SEND / RECV), the job's nonce and the pid, and a
// peer with the wrong role or nonce (an echo, another job's listener, a stray client) is
// dropped and the rendezvous retried until timeout_s. (GPUTEST_r04: an 8-rank C5 run on
// derived ephemeral ports paired a sender with itself)
// Sender: every post_write of the upstream block is forwarded immediately (chunks of at
// most the receiver's free ring space). The span is released by one rule for every
// transport (remote::transport in the .cpp): at once when the transport's read of it is
// stream-ordered after the producing kernel and before the next one (rccl, p2p) or already
// done (socket); when the transport reports the read complete otherwise (the host-ring test
// transport "deferred_test"). Receiver: a thread per adapter places each message into its
// ring, then post_write + NOTIFY_INPUT wake the downstream block. Per-run DONE / READER_DONE
// messages make drain-based termination and restarted flowgraphs work across processes.
#pragma once
#include <gnuradio/domain_adapter.hpp>
#include <gnuradio/scheduler.hpp>

#include <atomic>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace gr {

namespace remote {
class channel;   // TCP control (and host data) socket
class transport; // data path: "rccl" | "p2p" | "socket" | "deferred_test"
// deferred_test transport: messages whose ring span changed between send() and the transport's
// delayed read of it (the ring was overwritten before the transfer read it); process-wide
uint64_t deferred_test_violations();
// connections rejected because they were connected to themselves (process-wide)
uint64_t self_connects_rejected();
// hello exchanges refused because the peer had the wrong role / nonce (process-wide)
uint64_t peers_refused();
} // namespace remote

// Placeholder scheduler for a domain that another process runs. Never initialised or
// started here; `rank` is informational (the process that owns the domain).
class remote_domain : public scheduler
{
public:
    using sptr = std::shared_ptr<remote_domain>;
    static sptr make(int rank, const std::string& name = "remote") { return std::make_shared<remote_domain>(rank, name); }
    remote_domain(int rank, const std::string& name) : scheduler(name), _rank(rank) {}
    int rank() const { return _rank; }
    void initialize(flat_graph_sptr, flowgraph_monitor_sptr, neighbor_interface_map) override {}
    void push_message(scheduler_message_sptr) override {}
    void start() override {}
    void stop() override {}
    void wait() override {}

private:
    int _rank;
};

enum class remote_role { SEND, RECV };

struct remote_edge_options {
    std::string host = "127.0.0.1"; // address of the receiving process
    // a directory every process of the job can see (one node): receivers publish the port they
    // were given there; "" = the fixed ports below
    std::string rendezvous_dir;
    int base_port = 29650;          // without rendezvous_dir: crossing i listens on base_port + i
    uint64_t nonce = 0;             // job id, the same in every process of one flowgraph
    // "auto" (rccl across GPUs, p2p for two processes on one GPU, socket for host rings) |
    // "rccl" | "p2p" | "socket" | "deferred_test" (host rings; CPU tests of the release rule)
    std::string transport = "auto";
    int device = -1;                // GPU of this process (-1: the current thread's device)
    double timeout_s = 120.0;       // connect / accept / handshake limit
    // p2p: how long a sender waits for a free landing slot while the receiver is alive but
    // backpressured (its downstream slow or paused); 0 = as long as the channel is healthy
    double stall_timeout_s = 0;
};

class domain_adapter_remote : public domain_adapter
{
public:
    using sptr = std::shared_ptr<domain_adapter_remote>;
    // other_port: the local block port this adapter faces (SEND faces an output port).
    static sptr make(remote_role role, port_sptr other_port, int crossing, const remote_edge_options& opt);
    ~domain_adapter_remote() override;

    // buffer interface: RECV serves the downstream block's reads, SEND the upstream
    // block's writes; both forward to the LOCAL ring created by the buffer manager.
    void* read_ptr() override;
    void* write_ptr() override;
    bool read_info(buffer_info_t& info) override;
    bool write_info(buffer_info_t& info) override;
    void post_read(int n) override;
    void post_write(int n) override;
    void copy_items(buffer_sptr from, int n) override;
    void set_writer_done() override;
    void set_reader_done() override;
    bool writer_done() const override;
    bool reader_done() const override;
    void reset_flags() override;
    // Tags live on the LOCAL ring; the tags of each DATA message's items travel with it (their
    // offsets relative to the message's first item) and land on the receiving ring at the
    // same items, so absolute offsets survive the process boundary.
    gr::buffer* tag_target() override { return _buffer ? _buffer.get() : this; }

    void buffer_ready() override; // connect, handshake, start the receive thread

    remote_role role() const { return _role; }
    int crossing() const { return _crossing; }
    std::string transport_kind() const;
    uint64_t items_moved() const { return _moved.load(); }
    // The librccl file the rccl transport bound in this process (dladdr of ncclSend; "" before
    // the first rccl crossing): an already-loaded copy (torch's) if any, else /opt/rocm's.
    static std::string rccl_library();
    // The rccl transport's library binding exercised in ONE process (no peer, no second GPU):
    // through the same dlopen / dlsym table as the crossings, a 1-rank communicator on `device`
    // (ncclGetUniqueId, ncclCommInitRank), a grouped ncclSend + ncclRecv of `bytes` from src to
    // dst to `peer` (0 = self) on `stream`, the stream drained, ncclCommGetAsyncError, destroy.
    // src / dst must be device memory of `device` (checked before any RCCL call). Every failure,
    // RCCL's own codes included, throws with RCCL's error text.
    static void rccl_self_test(int device, const void* src, void* dst, size_t bytes, void* stream, int peer = 0);

private:
    domain_adapter_remote(remote_role role, int crossing, const remote_edge_options& opt);
    void pump();           // SEND: forward everything readable in the local ring
    void pump_locked();    // SEND: pump's loop (under _pump_m)
    void release_span(int m, bool deferred); // SEND: the edge's release rule (see pump)
    bool read_reverse(int timeout_ms);       // SEND: one reverse message, if any
    void poll_reverse();   // SEND: consume reverse messages (READER_DONE, transport credits)
    void recv_loop();      // RECV thread body
    void check_failed() const;
    void notify_downstream();
    bool local_is_device_side() const; // the side of the ring this adapter touches

    remote_role _role;
    int _crossing;
    remote_edge_options _opt;
    std::shared_ptr<remote::channel> _ch;
    std::shared_ptr<remote::transport> _tr;
    int _max_chunk = 0; // items per message (receiver's empty-ring writable count)
    size_t _isz = 0;
    int _device = -1;

    std::atomic<uint64_t> _runs{ 0 };          // local runs started (reset_flags calls)
    std::atomic<uint64_t> _remote_done{ 0 };   // DONE (RECV) / READER_DONE (SEND) messages
    std::atomic<uint64_t> _moved{ 0 };
    std::atomic<uint64_t> _reader_finished{ 0 }; // RECV: runs whose local reader finished
    std::atomic<bool> _ready{ false };            // setup complete (_ch, _tr valid)
    std::atomic<bool> _closing{ false };
    std::atomic<bool> _thread_done{ false };      // RECV thread finished
    std::thread _thr;
    std::mutex _m;
    std::condition_variable _cv; // RECV: space freed by the downstream block
    std::exception_ptr _err;
    std::atomic<bool> _failed{ false };
    std::mutex _pump_m;      // SEND: pump vs. deferred releases
    std::mutex _rev_m;       // SEND: reverse-message reads
    std::mutex _ring_m;      // RECV: ring writes vs. reset_flags' discard
    uint64_t _inflight = 0;  // SEND: items handed to the transport, not yet released
    int _lfd = -1;           // RECV: listening socket (bound at make)
    int _port = 0;           // RECV: its port
    void* _stream = nullptr; // RECV thread's stream (device rings)
    void* _scratch = nullptr; // RECV: discard area after the reader finished
    size_t _scratch_bytes = 0;
};

class domain_adapter_remote_conf : public domain_adapter_conf
{
public:
    using sptr = std::shared_ptr<domain_adapter_remote_conf>;
    static sptr make(const remote_edge_options& opt = remote_edge_options())
    {
        return std::make_shared<domain_adapter_remote_conf>(opt);
    }
    explicit domain_adapter_remote_conf(const remote_edge_options& opt)
        : domain_adapter_conf(buffer_preference_t::DOWNSTREAM), _opt(opt)
    {
    }
    domain_adapter_sptr make_remote_adapter(port_sptr local_port, bool local_is_upstream, int crossing,
                                            const std::string& name) override;
    const remote_edge_options& options() const { return _opt; }
    // The adapters this conf instantiated in this process (partition order), e.g. to
    // report the transport each crossing negotiated.
    std::vector<std::shared_ptr<domain_adapter_remote>> adapters() const
    {
        std::vector<std::shared_ptr<domain_adapter_remote>> v;
        for (auto& w : _made)
            if (auto a = w.lock()) v.push_back(a);
        return v;
    }

private:
    remote_edge_options _opt;
    std::vector<std::weak_ptr<domain_adapter_remote>> _made;
};

} // namespace gr
