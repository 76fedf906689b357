// Cross-process flowgraphs (domain_adapter_remote): every case is run by TWO processes
// (tests/test_remote_edge.py starts them with QA_RANK=0/1 and a shared QA_PORT). Both
// build the same flowgraph and domain list; each runs the domains of its rank and marks
// the others remote_domain, so graph_utils::partition instantiates one half of every
// crossing per process. The reference has no multi-process partitioning (its in-process
// adapter test is disabled, schedulers/mt/test/qa_scheduler_mt.cpp:40-78); expectations
// are the single-process results (exact for copies and complex products, 1e-5 norm-wise
// for the FIR pipeline).
#include "qa.hpp"
#include "qa_ref.hpp"

#include <chrono>
#include <cstdlib>
#include <arpa/inet.h>
#include <dlfcn.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>
#include <thread>
#include <gnuradio/blocklib/blocks/annotator.hpp>
#include <gnuradio/blocklib/blocks/copy.hpp>
#include <gnuradio/blocklib/blocks/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/blocks/head.hpp>
#include <gnuradio/blocklib/blocks/null_sink.hpp>
#include <gnuradio/blocklib/blocks/null_source.hpp>
#include <gnuradio/blocklib/blocks/multiply_const.hpp>
#include <gnuradio/blocklib/blocks/vector_sink.hpp>
#include <gnuradio/blocklib/blocks/vector_source.hpp>
#include <gnuradio/blocklib/hip/copy.hpp>
#include <gnuradio/blocklib/hip/fir_filter_ccf.hpp>
#include <gnuradio/blocklib/hip/multiply_const.hpp>
#include <gnuradio/blocklib/hip/synth_source.hpp>
#include <gnuradio/domain_adapter_direct.hpp>
#include <gnuradio/domain_adapter_remote.hpp>
#include <gnuradio/flowgraph.hpp>
#include <gnuradio/hip_buffer.hpp>
#include <gnuradio/schedulers/hip/scheduler_hip.hpp>
#include <gnuradio/schedulers/mt/scheduler_mt.hpp>

using namespace gr;

static int env_int(const char* k, int d)
{
    const char* v = std::getenv(k);
    return v ? std::atoi(v) : d;
}
static int rank() { return env_int("QA_RANK", 0); }
static remote_edge_options opts()
{
    remote_edge_options o;
    // the harness gives every case a fresh rendezvous directory (QA_RDV) and a job nonce; QA_PORT
    // alone selects the fixed-port mode (the self-connect case)
    if (const char* d = std::getenv("QA_RDV")) o.rendezvous_dir = d;
    if (const char* n = std::getenv("QA_NONCE")) o.nonce = std::strtoull(n, nullptr, 10);
    o.base_port = env_int("QA_PORT", 29650);
    o.timeout_s = env_int("QA_TIMEOUT", 60);
    if (const char* t = std::getenv("QA_TRANSPORT")) o.transport = t; // default "auto"
    return o;
}
// every crossing of this process negotiated QA_EXPECT_TRANSPORT (when set)
static void expect_transport(const domain_adapter_remote_conf::sptr& da)
{
    const char* want = std::getenv("QA_EXPECT_TRANSPORT");
    for (auto& a : da->adapters()) {
        std::printf("  crossing %d (%s): transport %s\n", a->crossing(),
                    a->role() == remote_role::SEND ? "send" : "recv", a->transport_kind().c_str());
        if (want) EXPECT_TRUE(a->transport_kind() == want);
    }
}
// the scheduler for a domain owned by `owner`: real here, a placeholder elsewhere
static scheduler_sptr sched_for(int owner, scheduler_sptr real)
{
    return owner == rank() ? real : std::static_pointer_cast<scheduler>(remote_domain::make(owner));
}

// The RCCL test double's counters (tests/cpp/fake_rccl.hip), when it is the loaded transport
// library: sends completed, sends that waited > 200 us for their receive, the longest wait.
static bool fake_rccl_stats(unsigned long long& sends, unsigned long long& waited, unsigned long long& max_us)
{
    const char* lib = std::getenv("NSH_RCCL_LIB");
    if (!lib || !*lib) return false;
    void* h = dlopen(lib, RTLD_NOW | RTLD_NOLOAD); // the instance the adapter loaded
    if (!h) return false;
    auto f = (void (*)(unsigned long long*, unsigned long long*, unsigned long long*))dlsym(h, "fake_rccl_stats");
    if (f) f(&sends, &waited, &max_us);
    dlclose(h);
    return f != nullptr;
}

// A host block that copies slowly (sleeps per work() call): a slow consumer, so a receiving ring
// upstream of it fills.
class slow_copy : public blocks::copy
{
public:
    static std::shared_ptr<slow_copy> make(size_t itemsize, int sleep_us)
    {
        auto p = std::make_shared<slow_copy>(itemsize, sleep_us);
        p->add_port(untyped_port::make("input", port_direction_t::INPUT, itemsize));
        p->add_port(untyped_port::make("out", port_direction_t::OUTPUT, itemsize));
        return p;
    }
    slow_copy(size_t itemsize, int sleep_us) : blocks::copy(itemsize), _us(sleep_us) {}
    work_return_code_t work(std::vector<block_work_input>& in, std::vector<block_work_output>& out) override
    {
        std::this_thread::sleep_for(std::chrono::microseconds(_us));
        out[0].n_items = std::min(out[0].n_items, 4096);
        return blocks::copy::work(in, out);
    }

private:
    int _us;
};

// src -> *k [rank 0] ~~> copy -> sink [rank 1], run twice (restart across processes)
TEST(RemoteCpu, ChainRestart)
{
    const size_t n = 200000;
    auto x = synth(n, 7);
    const gr_complex k(0.5f, -1.25f);
    auto src = blocks::vector_source_c::make(x);
    auto mul = blocks::multiply_const_cc::make(k);
    auto cp = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, mul, 0);
    fg->connect(mul, 0, cp, 0);
    fg->connect(cp, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto da = domain_adapter_remote_conf::make(opts());
    domain_conf_vec dc{ domain_conf(s0, { src, mul }, da), domain_conf(s1, { cp, snk }, da) };
    fg->partition(dc);
    std::vector<gr_complex> ref(x);
    for (auto& v : ref) v = cmul(v, k);
    for (int run = 0; run < 3; ++run) { // vector_sink clears at each start
        fg->run();
        if (rank() == 1) {
            if (snk->data().size() != n) std::fprintf(stderr, "  run %d: %zu items\n", run, snk->data().size());
            EXPECT_TRUE(snk->data() == ref);
        }
    }
    expect_transport(da);
}

// A crossing whose setup is refused (here: "p2p" asked for host rings; on a node, "rccl" with
// both ends on one GPU) is an error of fg->run() in BOTH processes -- the receiver's refusal,
// and on the sender the closed handshake, raised when its upstream block first writes -- and
// never a process abort (the error path's wind-down used to rethrow on the scheduler thread).
static void setup_refused(const char* transport, int port_offset, const char* why)
{
    const size_t n = 50000;
    auto src = blocks::vector_source_c::make(synth(n, 3));
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += port_offset;
    o.transport = transport;
    auto conf = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, conf), domain_conf(s1, { cp1, snk }, conf) };
    fg->partition(dc);
    std::string what;
    try {
        fg->run();
    } catch (const std::exception& e) {
        what = e.what();
    }
    std::printf("  rank %d: run() raised: %s\n", rank(), what.empty() ? "(nothing)" : what.c_str());
    EXPECT_TRUE(!what.empty());
    if (rank() == 1) EXPECT_TRUE(what.find(why) != std::string::npos);
}
TEST(RemoteCpu, SetupRefusedIsAnError) { setup_refused("p2p", 100, "p2p transport needs device rings"); }
// "rccl" on host rings without the test double's hook (NSH_REMOTE_TEST_RCCL)
TEST(RemoteCpu, RcclRefusedOnHostRings)
{
    setup_refused("rccl", 110, "rccl transport needs device rings on two different GPUs");
}

// Tags across processes (reference qa_tags.cpp AcrossDomains shape, here over a process
// boundary): src -> head -> ann0 [0] ~~> copy -> ann1 -> sink [1]. ann1 must see ann0's 4 tags
// at their absolute offsets with their values and srcid, in each of two runs (the edge
// counters keep counting across runs, on both sides alike).
TEST(RemoteCpu, TagsCrossProcesses)
{
    const int N = 40000;
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), N);
    auto ann0 = blocks::annotator::make(10000, sizeof(gr_complex), 1, 1, tag_propagation_policy_t::TPP_ALL_TO_ALL);
    auto cp = blocks::copy::make(sizeof(gr_complex));
    auto ann1 = blocks::annotator::make(1u << 30, sizeof(gr_complex), 1, 1, tag_propagation_policy_t::TPP_ALL_TO_ALL);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    ann0->set_alias("ann0");
    auto fg = flowgraph::make();
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, cp, 0);
    fg->connect(cp, 0, ann1, 0);
    fg->connect(ann1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 60;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, head, ann0 }, da), domain_conf(s1, { cp, ann1, snk }, da) };
    fg->partition(dc);
    for (int run = 0; run < 2; ++run) {
        fg->run();
        if (rank() == 1) {
            auto seen = ann1->data();
            ASSERT_TRUE(seen.size() == 4u * (run + 1));
            for (size_t i = 0; i < 4; ++i) {
                const auto& t = seen[4 * run + i];
                EXPECT_EQ(t.offset, (uint64_t)(N * run + 10000 * i));
                EXPECT_TRUE(std::get<int64_t>(t.value->value()) == (int64_t)(4 * run + i));
                EXPECT_TRUE(std::get<std::string>(t.key->value()) == "seq");
                EXPECT_TRUE(t.srcid && std::get<std::string>(t.srcid->value()) == "ann0");
            }
        }
    }
    expect_transport(da);
}

// The CPU form of RemoteGpu.RestartDropsRemainder: host rings, fir_filter_ccf(h, 4) downstream
// of the crossing, n = 4k + 3, three runs; each must equal the first (bit-identical) and the
// reference.
TEST(RemoteCpu, RestartDropsRemainder)
{
    const size_t n = 100003;
    const auto h = lowpass(31, 0.1);
    auto x = synth(n, 5);
    auto src = blocks::vector_source_c::make(x);
    auto cp = blocks::copy::make(sizeof(gr_complex));
    auto fir = blocks::fir_filter_ccf::make(h, 4);
    auto snk = blocks::vector_sink_c::make(1, n / 4);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp, 0);
    fg->connect(cp, 0, fir, 0);
    fg->connect(fir, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 80;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp }, da), domain_conf(s1, { fir, snk }, da) };
    fg->partition(dc);
    const auto ref = fir_ref(x, h, 4);
    std::vector<gr_complex> first;
    for (int run = 0; run < 3; ++run) {
        fg->run();
        if (rank() == 1) {
            ASSERT_TRUE(snk->data().size() == ref.size());
            EXPECT_TRUE(close_normwise(snk->data(), ref));
            if (run == 0)
                first = snk->data();
            else
                EXPECT_TRUE(snk->data() == first);
        }
    }
    expect_transport(da);
}

// The edge's release rule with a transport whose reads complete later on another thread
// (transport "deferred_test": the payload is read from the sender's ring span after
// NSH_REMOTE_TEST_DELAY_US, and the span is released only then). Small rings (8192 items) so
// the upstream block would overwrite a released span within microseconds: the transport
// checksums each span at send() and again at its delayed read, and counts any difference.
// Expect: no violations, the data bit-exact over three runs. With
// NSH_REMOTE_TEST_EARLY_RELEASE=1 (QA_EXPECT_VIOLATIONS=1) the transport claims its read is
// done at send(): the negative control, which must show violations.
TEST(RemoteCpu, DeferredRelease)
{
    const bool early = env_int("QA_EXPECT_VIOLATIONS", 0) != 0;
    const size_t n = 120000;
    auto x = synth(n, 13);
    const gr_complex k(1.5f, -0.5f);
    std::vector<gr_complex> ref(x);
    for (auto& v : ref) v = cmul(v, k);
    {
        auto src = blocks::vector_source_c::make(x);
        auto mul = blocks::multiply_const_cc::make(k);
        auto cp = blocks::copy::make(sizeof(gr_complex));
        auto snk = blocks::vector_sink_c::make(1, n);
        auto fg = flowgraph::make();
        fg->connect(src, 0, mul, 0);
        fg->connect(mul, 0, cp, 0);
        fg->connect(cp, 0, snk, 0);
        auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
        auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
        fg->set_schedulers({ s0, s1 });
        auto o = opts();
        o.base_port += 90;
        o.transport = "deferred_test";
        auto da = domain_adapter_remote_conf::make(o);
        domain_conf_vec dc{ domain_conf(s0, { src, mul }, da), domain_conf(s1, { cp, snk }, da) };
        fg->partition(dc);
        for (int run = 0; run < (early ? 1 : 3); ++run) {
            fg->run();
            if (rank() == 1 && !early) EXPECT_TRUE(snk->data() == ref);
        }
        for (auto& a : da->adapters()) std::printf("  transport %s\n", a->transport_kind().c_str());
    } // adapters destroyed: the sender's transport has read and sent every message
    if (rank() == 0) {
        const uint64_t v = remote::deferred_test_violations();
        std::printf("  deferred_test violations: %llu\n", (unsigned long long)v);
        if (early)
            EXPECT_TRUE(v > 0);
        else
            EXPECT_EQ(v, (uint64_t)0);
    }
}

// src -> *k1 [0] ~~> *k2 [1] ~~> sink [0]: crossings in both directions between the same
// two processes (set-up order must not deadlock)
TEST(RemoteCpu, TwoCrossingsBothWays)
{
    const size_t n = 150000;
    auto x = synth(n, 99);
    const gr_complex k1(2.0f, 0.5f), k2(-0.75f, 0.25f);
    auto src = blocks::vector_source_c::make(x);
    auto m1 = blocks::multiply_const_cc::make(k1);
    auto m2 = blocks::multiply_const_cc::make(k2);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, m1, 0);
    fg->connect(m1, 0, m2, 0);
    fg->connect(m2, 0, snk, 0);
    auto a = sched_for(0, schedulers::scheduler_mt::make("a", 8192));
    auto b = sched_for(1, schedulers::scheduler_mt::make("b", 8192));
    auto c = sched_for(0, schedulers::scheduler_mt::make("c", 8192));
    fg->set_schedulers({ a, b, c });
    auto o = opts();
    o.base_port += 10;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(a, { src, m1 }, da), domain_conf(b, { m2 }, da), domain_conf(c, { snk }, da) };
    fg->partition(dc);
    fg->run();
    if (rank() == 0) {
        std::vector<gr_complex> ref(x);
        for (auto& v : ref) v = cmul(cmul(v, k1), k2);
        EXPECT_TRUE(snk->data() == ref);
    }
    expect_transport(da);
}

// endless source [0] ~~> head(n) -> sink [1]: the reader finishing first must stop the
// writer's process (READER_DONE travels upstream)
TEST(RemoteCpu, ReaderFinishesFirst)
{
    const size_t n = 100000;
    auto x = synth(4096, 3);
    auto src = blocks::vector_source_c::make(x, true);
    auto hd = blocks::head::make(sizeof(gr_complex), n);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, hd, 0);
    fg->connect(hd, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 20;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src }, da), domain_conf(s1, { hd, snk }, da) };
    fg->partition(dc);
    fg->run();
    if (rank() == 1) {
        const auto& got = snk->data();
        ASSERT_TRUE(got.size() == n);
        bool ok = true;
        for (size_t i = 0; i < n; ++i) ok = ok && got[i] == x[i % x.size()];
        EXPECT_TRUE(ok);
    }
    expect_transport(da);
}

// GPU: vector_source -[H2D]-> hip::multiply_const [rank 0, scheduler_hip] ~~> hip::copy
// [rank 1, scheduler_hip] -[D2H]-> vector_sink. Device rings on both sides (one GPU shared
// by two processes -> staged socket transport; different GPUs -> RCCL).
TEST(RemoteGpu, DeviceChainRestart)
{
    const size_t n = 1u << 20;
    auto x = synth(n, 11);
    const gr_complex k(-0.5f, 2.0f);
    auto src = blocks::vector_source_c::make(x);
    auto mul = hip::multiply_const_cc::make(k);
    auto cp = hip::copy::make(1);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, mul, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(mul, 0, cp, 0);
    fg->connect(cp, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 20));
    auto s1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 20));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 30;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, mul }, da), domain_conf(s1, { cp, snk }, da) };
    fg->partition(dc);
    std::vector<gr_complex> ref(x);
    for (auto& v : ref) v = cmul(v, k);
    for (int run = 0; run < 3; ++run) { // vector_sink clears at each start
        fg->run();
        if (rank() == 1) {
            if (snk->data().size() != n) std::fprintf(stderr, "  run %d: %zu items\n", run, snk->data().size());
            EXPECT_TRUE(snk->data() == ref);
        }
    }
    expect_transport(da);
}

// "rccl" asked for with both device rings on one GPU (the 1-GPU box): the receiver refuses it
// (RCCL cannot pair two ranks on one device) and both processes get the error from fg->run()
// -- the sender's partition thread winds down without aborting the process.
TEST(RemoteGpu, RcclRefusedOnOneGpu)
{
    const size_t n = 1u << 16;
    auto src = blocks::vector_source_c::make(synth(n, 5));
    auto mul = hip::multiply_const_cc::make(gr_complex(2.0f, 0.0f));
    auto cp = hip::copy::make(1);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, mul, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(mul, 0, cp, 0);
    fg->connect(cp, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 18));
    auto s1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 18));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 110;
    o.transport = "rccl";
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, mul }, da), domain_conf(s1, { cp, snk }, da) };
    fg->partition(dc);
    std::string what;
    try {
        fg->run();
    } catch (const std::exception& e) {
        what = e.what();
    }
    std::printf("  rank %d: run() raised: %s\n", rank(), what.empty() ? "(nothing)" : what.c_str());
    EXPECT_TRUE(!what.empty());
    if (rank() == 1) EXPECT_TRUE(what.find("two different GPUs") != std::string::npos);
}

// Tags through device rings and a process crossing: host annotator -[H2D]-> hip::copy [0]
// ~~(device rings; staged or RCCL)~~> hip::copy -[D2H]-> host annotator [1].
TEST(RemoteGpu, DeviceTags)
{
    const int N = 1 << 20;
    auto src = blocks::null_source::make(sizeof(gr_complex));
    auto head = blocks::head::make(sizeof(gr_complex), N);
    auto ann0 = blocks::annotator::make(1u << 18, sizeof(gr_complex), 1, 1, tag_propagation_policy_t::TPP_ALL_TO_ALL);
    auto c0 = hip::copy::make(1);
    auto c1 = hip::copy::make(1);
    auto ann1 = blocks::annotator::make(1u << 30, sizeof(gr_complex), 1, 1, tag_propagation_policy_t::TPP_ALL_TO_ALL);
    auto snk = blocks::null_sink::make(sizeof(gr_complex));
    auto fg = flowgraph::make();
    fg->connect(src, 0, head, 0);
    fg->connect(head, 0, ann0, 0);
    fg->connect(ann0, 0, c0, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(c0, 0, c1, 0);
    fg->connect(c1, 0, ann1, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->connect(ann1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("h0", 1u << 20));
    auto g0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 20));
    auto g1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 20));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("h1", 1u << 20));
    fg->set_schedulers({ s0, g0, g1, s1 });
    auto o = opts();
    o.base_port += 70;
    auto da = domain_adapter_remote_conf::make(o);
    auto dd = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
    // a crossing takes its downstream domain's conf: only g1's is the remote one
    domain_conf_vec dc{ domain_conf(s0, { src, head, ann0 }, dd), domain_conf(g0, { c0 }, dd),
                        domain_conf(g1, { c1 }, da), domain_conf(s1, { ann1, snk }, dd) };
    fg->partition(dc);
    fg->run();
    expect_transport(da);
    if (rank() == 1) {
        auto seen = ann1->data();
        ASSERT_TRUE(seen.size() == 4u);
        for (size_t i = 0; i < 4; ++i) {
            EXPECT_EQ(seen[i].offset, (uint64_t)((1u << 18) * i));
            EXPECT_TRUE(std::get<int64_t>(seen[i].value->value()) == (int64_t)i);
        }
        EXPECT_EQ(snk->consumed(), (uint64_t)N);
    }
}

// GPU C5 shape over two processes: synth -> fir/2 -> fir/2 [rank 0] ~~> fir/2 -> fir/2
// -[D2H]-> sink [rank 1] (BASELINE C5 with G = 2: stages {1,2} | {3,4}).
TEST(RemoteGpu, DecimatingPipelineC5)
{
    const size_t n = 1u << 20;
    const auto h = lowpass(127, 0.225);
    auto src = hip::synth_source::make(0, n);
    std::vector<hip::fir_filter_ccf::sptr> st;
    for (int i = 0; i < 4; ++i) st.push_back(hip::fir_filter_ccf::make(h, 2));
    auto snk = blocks::vector_sink_c::make(1, n / 16);
    auto fg = flowgraph::make();
    fg->connect(src, 0, st[0], 0);
    for (int i = 1; i < 4; ++i) fg->connect(st[i - 1], 0, st[i], 0);
    fg->connect(st[3], 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 19));
    auto s1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 19));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 40;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, st[0], st[1] }, da), domain_conf(s1, { st[2], st[3], snk }, da) };
    fg->partition(dc);
    auto ref = synth(n);
    for (int i = 0; i < 4; ++i) ref = fir_ref(ref, h, 2);
    for (int run = 0; run < 2; ++run) {
        fg->run();
        if (rank() == 1) EXPECT_TRUE(close_normwise(snk->data(), ref));
    }
    expect_transport(da);
}

// A restarted two-process pipeline whose stream length is not a multiple of the downstream
// decimation: the receiving ring keeps 3 items below one output at the end of each run,
// which must be dropped before the next run's data arrive (they used to
// be prepended to the next run's stream). device rings, fir/4 downstream; every run must
// equal the single-process result.
TEST(RemoteGpu, RestartDropsRemainder)
{
    const size_t n = (1u << 18) + 3;
    const auto h = lowpass(127, 0.1);
    auto x = synth(n, 5);
    auto src = blocks::vector_source_c::make(x);
    auto cp = hip::copy::make(1);
    auto fir = hip::fir_filter_ccf::make(h, 4);
    auto snk = blocks::vector_sink_c::make(1, n / 4);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp, 0)->set_custom_buffer(HIP_BUFFER_ARGS_H2D);
    fg->connect(cp, 0, fir, 0);
    fg->connect(fir, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 19));
    auto s1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 19));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 50;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp }, da), domain_conf(s1, { fir, snk }, da) };
    fg->partition(dc);
    const auto ref = fir_ref(x, h, 4);
    for (int run = 0; run < 3; ++run) {
        // not bit-identical between runs: the MFMA decimator's per-chunk scales follow how the
        // stream was split into work() calls, which the message timing decides; a stream
        // shifted by the 3 stale items would miss the reference by O(1)
        fg->run();
        if (rank() == 1) {
            ASSERT_TRUE(snk->data().size() == ref.size());
            EXPECT_TRUE(close_normwise(snk->data(), ref));
        }
    }
    expect_transport(da);
}

// BASELINE C5 at G = 4: one decimating stage per process, 4 processes, 3 crossings; ranks 1 and 2
// each hold a receiving crossing (adapter stream) and a sending one (partition stream) at once --
// with the rccl transport, two communicators in one process on two streams. synth -> fir/2 [0]
// ~~> fir/2 [1] ~~> fir/2 [2] ~~> fir/2 -[D2H]-> sink [3]; three runs, each within 1e-5
// (norm-wise) of the double-precision chain.
TEST(RemoteGpu, FourStagePipeline)
{
    const size_t n = 1u << 20;
    const auto h = lowpass(127, 0.225);
    auto src = hip::synth_source::make(0, n);
    std::vector<hip::fir_filter_ccf::sptr> st;
    for (int i = 0; i < 4; ++i) st.push_back(hip::fir_filter_ccf::make(h, 2));
    auto snk = blocks::vector_sink_c::make(1, n / 16);
    auto fg = flowgraph::make();
    fg->connect(src, 0, st[0], 0);
    for (int i = 1; i < 4; ++i) fg->connect(st[i - 1], 0, st[i], 0);
    fg->connect(st[3], 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    std::vector<scheduler_sptr> sc;
    for (int g = 0; g < 4; ++g)
        sc.push_back(sched_for(g, schedulers::scheduler_hip::make("g" + std::to_string(g), 0, 1u << 19)));
    fg->set_schedulers(sc);
    auto o = opts();
    o.base_port += 120;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(sc[0], { src, st[0] }, da), domain_conf(sc[1], { st[1] }, da),
                        domain_conf(sc[2], { st[2] }, da), domain_conf(sc[3], { st[3], snk }, da) };
    fg->partition(dc);
    auto ref = synth(n);
    for (int i = 0; i < 4; ++i) ref = fir_ref(ref, h, 2);
    for (int run = 0; run < 3; ++run) {
        fg->run();
        if (rank() == 3) {
            ASSERT_TRUE(snk->data().size() == ref.size());
            EXPECT_TRUE(close_normwise(snk->data(), ref));
        }
    }
    if (rank() == 1 || rank() == 2) EXPECT_EQ(da->adapters().size(), (size_t)2); // one in, one out
    expect_transport(da);
}

// A full receiving ring while the sender's stream is inside the send: hip::synth_source ->
// hip::copy [0] ~~> hip::copy -[D2H]-> slow host copy (1 ms per 4096 items) -> sink [1], small
// rings (64 KiB on the GPU side), so the receiver posts each receive only when its ring has drained
// enough. The data must arrive bit-exact over two runs; with the RCCL test double the sends must
// have waited for their receives (rendezvous held the sender's partition stream).
TEST(RemoteGpu, FullRingBackpressure)
{
    const size_t n = 1u << 19;
    auto src = hip::synth_source::make(0, n);
    auto c0 = hip::copy::make(1);
    auto c1 = hip::copy::make(1);
    auto slow = slow_copy::make(sizeof(gr_complex), 1000);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, c0, 0);
    fg->connect(c0, 0, c1, 0);
    fg->connect(c1, 0, slow, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    fg->connect(slow, 0, snk, 0);
    auto g0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 16));
    auto g1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 16));
    auto h1 = sched_for(1, schedulers::scheduler_mt::make("h1", 1u << 16));
    fg->set_schedulers({ g0, g1, h1 });
    auto o = opts();
    o.base_port += 130;
    auto da = domain_adapter_remote_conf::make(o);
    auto dd = domain_adapter_direct_conf::make(buffer_preference_t::DOWNSTREAM);
    domain_conf_vec dc{ domain_conf(g0, { src, c0 }, dd), domain_conf(g1, { c1 }, da), domain_conf(h1, { slow, snk }, dd) };
    fg->partition(dc);
    const auto ref = synth(n);
    for (int run = 0; run < 2; ++run) {
        fg->run();
        if (rank() == 1) EXPECT_TRUE(snk->data() == ref);
    }
    expect_transport(da);
    unsigned long long sends = 0, waited = 0, max_us = 0;
    if (rank() == 0 && fake_rccl_stats(sends, waited, max_us)) {
        std::printf("  fake rccl: %llu sends, %llu waited > 200 us for their receive, longest %llu us\n", sends, waited,
                    max_us);
        EXPECT_TRUE(sends > 0);
        EXPECT_TRUE(waited > 0 && max_us > 1000);
    }
}

// The negative control of the RCCL test double's rendezvous (FAKE_RCCL_MISORDER=1: the receiver
// posts READY only after the payload arrived, which a rendezvous never satisfies): the first
// message deadlocks until the double's bounded wait gives up, and fg->run() raises in both
// processes. With a double that never blocks the sender (before round 4) this case passed.
TEST(RemoteGpu, RendezvousMisorderTimesOut)
{
    const size_t n = 1u << 18;
    auto src = hip::synth_source::make(0, n);
    auto c0 = hip::copy::make(1);
    auto c1 = hip::copy::make(1);
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, c0, 0);
    fg->connect(c0, 0, c1, 0);
    fg->connect(c1, 0, snk, 0)->set_custom_buffer(HIP_BUFFER_ARGS_D2H);
    auto s0 = sched_for(0, schedulers::scheduler_hip::make("g0", 0, 1u << 18));
    auto s1 = sched_for(1, schedulers::scheduler_hip::make("g1", 0, 1u << 18));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 140;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, c0 }, da), domain_conf(s1, { c1, snk }, da) };
    fg->partition(dc);
    std::string what;
    try {
        fg->run();
    } catch (const std::exception& e) {
        what = e.what();
    }
    std::printf("  rank %d: run() raised: %s\n", rank(), what.empty() ? "(nothing)" : what.c_str());
    EXPECT_TRUE(what.find("rendezvous timed out") != std::string::npos);
}

// The same negative control on host rings (CPU; the double's synchronous receive).
TEST(RemoteCpu, RendezvousMisorderTimesOut)
{
    const size_t n = 100000;
    auto src = blocks::vector_source_c::make(synth(n, 3));
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 150;
    auto conf = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, conf), domain_conf(s1, { cp1, snk }, conf) };
    fg->partition(dc);
    std::string what;
    try {
        fg->run();
    } catch (const std::exception& e) {
        what = e.what();
    }
    std::printf("  rank %d: run() raised: %s\n", rank(), what.empty() ? "(nothing)" : what.c_str());
    EXPECT_TRUE(what.find("rendezvous timed out") != std::string::npos);
}

// Self-connect (GPUTEST_r04's failure, made deterministic): fixed-port mode, the receiver
// [rank 1] starts listening only after 1.5 s, and the sender's first connect attempt binds its
// source to the destination port (NSH_REMOTE_TEST_SELF_CONNECT), which with nobody listening
// yields a socket connected to itself. QA_SELF_MODE=socket: the socket-level check must reject
// it; QA_SELF_MODE=hello: that check is skipped (hook value "hello") and the hello's role check
// must refuse the echo of the sender's own hello. Either way the sender retries, pairs with the
// real receiver, and the data arrive bit-exact.
TEST(RemoteCpu, SelfConnectRejected)
{
    const char* mode = std::getenv("QA_SELF_MODE");
    const bool hello_mode = mode && std::string(mode) == "hello";
    if (rank() == 1) std::this_thread::sleep_for(std::chrono::milliseconds(1500));
    const size_t n = 60000;
    auto x = synth(n, 21);
    auto src = blocks::vector_source_c::make(x);
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 160;
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, da), domain_conf(s1, { cp1, snk }, da) };
    fg->partition(dc);
    fg->run();
    if (rank() == 1) EXPECT_TRUE(snk->data() == x);
    if (rank() == 0) {
        std::printf("  self-connects rejected: %llu, peers refused: %llu\n",
                    (unsigned long long)remote::self_connects_rejected(), (unsigned long long)remote::peers_refused());
        if (hello_mode)
            EXPECT_TRUE(remote::peers_refused() >= 1);
        else
            EXPECT_TRUE(remote::self_connects_rejected() >= 1);
    }
    expect_transport(da);
}

// Two jobs on one port: the ranks carry different nonces (QA_NONCE + rank), as if each had met
// another job's process on a reused port. The receiver refuses the sender's hello, the sender
// sees its connection dropped, both retry until QA_TIMEOUT and fg->run() raises in both
// processes; the receiver names the nonce. Nothing is paired, nothing is transferred.
TEST(RemoteCpu, ForeignNonceRefused)
{
    const size_t n = 20000;
    auto src = blocks::vector_source_c::make(synth(n, 4));
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto o = opts();
    o.base_port += 170;
    o.nonce += (uint64_t)rank() + 1;
    auto conf = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, conf), domain_conf(s1, { cp1, snk }, conf) };
    fg->partition(dc);
    std::string what;
    try {
        fg->run();
    } catch (const std::exception& e) {
        what = e.what();
    }
    std::printf("  rank %d: run() raised: %s\n", rank(), what.empty() ? "(nothing)" : what.c_str());
    std::printf("  peers refused: %llu\n", (unsigned long long)remote::peers_refused());
    EXPECT_TRUE(!what.empty());
    if (rank() == 1) {
        EXPECT_TRUE(what.find("another job") != std::string::npos);
        EXPECT_TRUE(remote::peers_refused() >= 1);
    }
}

// A stale rendezvous entry with this job's nonce: before the receiver [rank 1]
// exists, the sender [rank 0] finds <dir>/crossing0 naming a port nobody listens on (a receiver
// that died before removing its entry). The receiver starts 1.5 s later and republishes; the
// sender, which re-reads the entry after each 1 s connect slice, must pair with it and move the
// data bit-exact -- instead of retrying the dead port until the timeout.
TEST(RemoteCpu, StaleRendezvousEntry)
{
    auto o = opts();
    if (o.rendezvous_dir.empty()) {
        std::printf("  needs QA_RDV\n");
        EXPECT_TRUE(false);
        return;
    }
    if (rank() == 0) { // the stale entry: a port that was bound once and is closed now
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        a.sin_port = 0;
        ::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a));
        socklen_t len = sizeof(a);
        ::getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
        ::close(fd);
        FILE* f = std::fopen((o.rendezvous_dir + "/crossing0").c_str(), "w");
        std::fprintf(f, "%d %llu\n", (int)ntohs(a.sin_port), (unsigned long long)o.nonce);
        std::fclose(f);
    } else {
        std::this_thread::sleep_for(std::chrono::milliseconds(1500));
    }
    const size_t n = 50000;
    auto x = synth(n, 31);
    auto src = blocks::vector_source_c::make(x);
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, da), domain_conf(s1, { cp1, snk }, da) };
    fg->partition(dc);
    fg->run();
    if (rank() == 1) EXPECT_TRUE(snk->data() == x);
    if (rank() == 0) {
        std::printf("  peers refused: %llu\n", (unsigned long long)remote::peers_refused());
        EXPECT_TRUE(remote::peers_refused() >= 1); // the dead port was seen and left
    }
}

// A silent client on the receiver's fixed port: rank 0 first connects a raw TCP
// socket that never says hello and keeps it open, then starts the real sender. The receiver drops
// the silent client after 2 s and pairs with the sender queued behind it (before, it waited for
// the silent client until the timeout and both ends failed).
TEST(RemoteCpu, SilentClientDropped)
{
    auto o = opts();
    o.base_port += 180;
    int silent = -1;
    if (rank() == 0) {
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        a.sin_port = htons((uint16_t)o.base_port);
        for (int i = 0; i < 500 && silent < 0; ++i) { // until the receiver listens
            const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
            if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0)
                silent = fd;
            else {
                ::close(fd);
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
        }
        EXPECT_TRUE(silent >= 0);
        std::this_thread::sleep_for(std::chrono::milliseconds(200)); // queued first
    }
    const size_t n = 50000;
    auto x = synth(n, 37);
    auto src = blocks::vector_source_c::make(x);
    auto cp0 = blocks::copy::make(sizeof(gr_complex));
    auto cp1 = blocks::copy::make(sizeof(gr_complex));
    auto snk = blocks::vector_sink_c::make(1, n);
    auto fg = flowgraph::make();
    fg->connect(src, 0, cp0, 0);
    fg->connect(cp0, 0, cp1, 0);
    fg->connect(cp1, 0, snk, 0);
    auto s0 = sched_for(0, schedulers::scheduler_mt::make("r0", 8192));
    auto s1 = sched_for(1, schedulers::scheduler_mt::make("r1", 8192));
    fg->set_schedulers({ s0, s1 });
    auto da = domain_adapter_remote_conf::make(o);
    domain_conf_vec dc{ domain_conf(s0, { src, cp0 }, da), domain_conf(s1, { cp1, snk }, da) };
    fg->partition(dc);
    fg->run();
    if (rank() == 1) {
        EXPECT_TRUE(snk->data() == x);
        std::printf("  peers refused: %llu\n", (unsigned long long)remote::peers_refused());
        EXPECT_TRUE(remote::peers_refused() >= 1);
    }
    if (silent >= 0) ::close(silent);
}
