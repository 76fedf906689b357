"""Cross-process flowgraphs (gr::domain_adapter_remote): each C++ case in
tests/cpp/qa_remote_edge.cpp runs as TWO processes (ranks 0 and 1) that build the same
flowgraph and domain list and each run their own domains, joined by TCP-controlled
crossing edges -- host rings over the socket on CPU (plus the "deferred_test" transport,
whose reads of the sender's ring complete late on another thread: the edge's release rule);
device rings (hip_buffer) on the GPU, where both ranks share the box's one GPU: the "p2p"
transport (stream-ordered copies into IPC-mapped landing slots, auto's choice on one GPU) and
the pinned-memory "socket" staging. RCCL needs two devices; auto selects it on a multi-GPU
node (test_bench.py::test_bench_c5_rccl_two_gpus). Until then the "rccl" transport's own code
runs against the RCCL test double tests/cpp/fake_rccl.hip, which keeps RCCL's rendezvous: a
send holds the sender's stream until the peer's stream has reached the matching receive (its
negative control, a mis-ordered receive, deadlocks and is reported as a rendezvous timeout)."""
import os
import random
import shutil
import socket
import subprocess
import tempfile

import pytest

from tests.conftest import ROOT

EXE = os.path.join(ROOT, "build", "tests", "qa_remote_edge")
FAKE_RCCL = os.path.join(ROOT, "build", "tests", "libfake_rccl.so")


def fixed_port_block(width=256):
    """A free block of ports BELOW the kernel's ephemeral range (ip_local_port_range), for the
    fixed-port cases: a port inside that range can be handed to some connect() as its source
    port while nobody listens on it -- the self-connect of GPUTEST_r04."""
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        lo = 32768
    hi = max(lo - width, 12000)
    for _ in range(200):
        base = random.randrange(10000, hi)
        ok = True
        for p in range(base, base + width):
            s = socket.socket()
            try:
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                s.bind(("127.0.0.1", p))
            except OSError:
                ok = False
            finally:
                s.close()
            if not ok:
                break
        if ok:
            return base
    raise RuntimeError("no free port block")


def run_pair(case, timeout=120, env_extra=None, ranks=2, fixed_port=False, expect_ok=True):
    """Run `case` as `ranks` processes. Default: a fresh rendezvous directory and job nonce
    (receivers listen on kernel-chosen ports and publish them there); fixed_port=True: the
    fixed-port mode on a block below the ephemeral range."""
    if not (os.path.exists(EXE) and os.path.exists(FAKE_RCCL)):
        subprocess.run(["make", "-s", "-C", ROOT, "tests"], check=True)
    rdv = tempfile.mkdtemp(prefix="nsh_rdv_")
    base = dict(QA_NONCE=str(random.getrandbits(62)))
    if fixed_port:
        base["QA_PORT"] = str(fixed_port_block())
    else:
        base["QA_RDV"] = rdv
    procs = []
    try:
        for r in range(ranks):
            env = dict(os.environ, QA_RANK=str(r), **base, **(env_extra or {}))
            procs.append(subprocess.Popen([EXE, case], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                          text=True))
        outs = []
        for p in procs:
            try:
                out, _ = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
            outs.append(out)
    finally:
        shutil.rmtree(rdv, ignore_errors=True)
    for r, (p, out) in enumerate(zip(procs, outs)):
        print(f"--- rank {r} ---\n{out}")
        assert p.returncode == 0, f"rank {r} failed:\n{out}"
        assert "0 failure(s)" in out and "1 test(s)" in out, out
    return outs


@pytest.mark.parametrize("mode", ["socket", "hello"])
def test_self_connect_rejected(mode):
    """GPUTEST_r04's failure forced deterministically: the sender's first connect binds its source
    to the destination port while the receiver is not yet listening, so the socket is connected to
    itself. mode=socket: the getsockname == getpeername check rejects it; mode=hello: with that check
    skipped, the hello's role check refuses the echo of the sender's own hello. Either way the
    sender retries and pairs with the real receiver; the data arrive bit-exact."""
    outs = run_pair("RemoteCpu.SelfConnectRejected", fixed_port=True,
                    env_extra={"NSH_REMOTE_TEST_SELF_CONNECT": "1" if mode == "socket" else "hello",
                               "QA_SELF_MODE": mode})
    if mode == "socket":
        assert "rejected a socket connected to itself" in outs[0]
    else:
        assert "own sender" in outs[0]


def test_foreign_nonce_refused():
    """Two jobs meeting on one port (different nonces): the receiver refuses the hello, nothing
    pairs, and fg->run() raises in both processes after the timeout, naming the nonce."""
    outs = run_pair("RemoteCpu.ForeignNonceRefused", fixed_port=True, env_extra={"QA_TIMEOUT": "4"})
    assert "another job" in outs[1]


def test_stale_rendezvous_entry_is_read_again():
    """a stale crossing entry carrying this job's nonce (a dead port) before the
    receiver starts: the sender re-reads the entry after each short connect slice and pairs with
    the receiver that republishes it; bit-exact, well inside the timeout."""
    outs = run_pair("RemoteCpu.StaleRendezvousEntry", env_extra={"QA_TIMEOUT": "20"})
    assert "nothing listens on published port" in outs[0]


def test_silent_client_is_dropped():
    """a client on the receiver's fixed port that never says hello is dropped after
    2 s, and the real sender queued behind it pairs; bit-exact."""
    outs = run_pair("RemoteCpu.SilentClientDropped", fixed_port=True, env_extra={"QA_TIMEOUT": "20"})
    assert "sent no hello within 2 s" in outs[1]


def test_rendezvous_dir_isolates_jobs():
    """Two pipelines of the same case at once, each with its own rendezvous directory and nonce:
    kernel-chosen ports, no collisions, both bit-exact."""
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(2) as ex:
        futs = [ex.submit(run_pair, "RemoteCpu.ChainRestart") for _ in range(2)]
        for f in futs:
            f.result()


@pytest.mark.parametrize("case", ["RemoteCpu.ChainRestart", "RemoteCpu.TwoCrossingsBothWays",
                                  "RemoteCpu.ReaderFinishesFirst", "RemoteCpu.TagsCrossProcesses",
                                  "RemoteCpu.RestartDropsRemainder", "RemoteCpu.SetupRefusedIsAnError"])
def test_remote_edges_cpu(case):
    run_pair(case)


@pytest.mark.parametrize("case", ["RemoteCpu.ChainRestart", "RemoteCpu.TwoCrossingsBothWays",
                                  "RemoteCpu.ReaderFinishesFirst", "RemoteCpu.TagsCrossProcesses",
                                  "RemoteCpu.RestartDropsRemainder"])
def test_remote_edges_cpu_rccl_protocol(case):
    """The "rccl" transport's own code path -- unique-id exchange over the control channel, a
    2-rank communicator per crossing, the DATA header then the payload's ncclSend / ncclRecv, the
    span released at send (RCCL reads it stream-ordered), discarded messages still received,
    restarts, two crossings between one pair of processes, teardown -- over host rings, through
    the RCCL test double tests/cpp/fake_rccl.c (NSH_RCCL_LIB; NSH_REMOTE_TEST_RCCL=1 lets the
    receiver accept rccl without two GPUs). The real library needs two GPUs, so this is what
    runs the transport before a multi-GPU node does; every crossing must report "rccl"."""
    outs = run_pair(case, env_extra={"QA_TRANSPORT": "rccl", "QA_EXPECT_TRANSPORT": "rccl",
                                     "NSH_RCCL_LIB": FAKE_RCCL, "NSH_REMOTE_TEST_RCCL": "1"})
    assert all("transport rccl" in o for o in outs)


RCCL_FAKE = {"QA_TRANSPORT": "rccl", "NSH_RCCL_LIB": FAKE_RCCL, "NSH_REMOTE_TEST_RCCL": "1"}


def test_rccl_rendezvous_negative_control_cpu():
    """The test double's rendezvous is real: with the receiver posting READY only after its payload
    (FAKE_RCCL_MISORDER=1), the sender never gets its READY and the receiver never gets its payload
    -- a deadlock, bounded by the double's wait (FAKE_RCCL_TIMEOUT_S) and reported by fg->run() in
    both processes as "rendezvous timed out". (The pre-round-4 double, which sent without waiting
    for the receive, passed this mis-order.)"""
    outs = run_pair("RemoteCpu.RendezvousMisorderTimesOut", timeout=90,
                    env_extra=dict(RCCL_FAKE, FAKE_RCCL_MISORDER="1", FAKE_RCCL_TIMEOUT_S="4"))
    assert all("rendezvous timed out" in o for o in outs)


def test_rccl_on_host_rings_refused_without_the_test_double():
    """Without the test hook, "rccl" asked for host rings is refused by the receiver: an error of
    fg->run() in both processes (the real library would be handed host pointers)."""
    outs = run_pair("RemoteCpu.RcclRefusedOnHostRings")
    assert "two different GPUs" in outs[1]


def test_deferred_release_keeps_span_until_read():
    """The release rule with an asynchronous reader: no span is overwritten before the
    transport read it (checksums at send and at the delayed read), data bit-exact, 3 runs."""
    outs = run_pair("RemoteCpu.DeferredRelease", env_extra={"NSH_REMOTE_TEST_DELAY_US": "1500"})
    assert "deferred_test violations: 0" in outs[0]


def test_deferred_release_negative_control():
    """The same transport releasing at send() (what the rule forbids for an unordered read):
    the upstream block overwrites spans before they are read, and the checksums see it --
    the positive test above can fail."""
    outs = run_pair("RemoteCpu.DeferredRelease", env_extra={
        "NSH_REMOTE_TEST_DELAY_US": "3000", "NSH_REMOTE_TEST_EARLY_RELEASE": "1", "QA_EXPECT_VIOLATIONS": "1"})
    assert "deferred_test(early)" in outs[0]


GPU_CASES = ["RemoteGpu.DeviceChainRestart", "RemoteGpu.DecimatingPipelineC5", "RemoteGpu.DeviceTags",
             "RemoteGpu.RestartDropsRemainder", "RemoteGpu.FullRingBackpressure"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU_CASES)
@pytest.mark.parametrize("transport", ["auto", "p2p", "socket"])
def test_remote_edges_gpu(case, transport):
    """Both ranks on the box's one GPU: auto must negotiate p2p (IPC landing slots); socket is
    the pinned-memory staging it replaces."""
    expect = {"auto": "p2p", "p2p": "p2p", "socket": "socket(staged)"}[transport]
    run_pair(case, timeout=300, env_extra={"QA_TRANSPORT": transport, "QA_EXPECT_TRANSPORT": expect})


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU_CASES)
def test_remote_edges_gpu_rccl_protocol(case):
    """The "rccl" transport on device rings, both ranks on the box's one GPU, with the RCCL test
    double in place of the library (which refuses two ranks on one device): the sender's payload
    read in stream order on its partition stream and the span released at once, the receiver's
    landing in stream order on its adapter stream ahead of post_write's event -- the ordering the
    real library gives -- through every GPU case (restarts, tags, the C5 {1,2}|{3,4} split,
    a decimator's remainder dropped across runs)."""
    run_pair(case, timeout=300, env_extra={"QA_TRANSPORT": "rccl", "QA_EXPECT_TRANSPORT": "rccl",
                                           "NSH_RCCL_LIB": FAKE_RCCL, "NSH_REMOTE_TEST_RCCL": "1"})


@pytest.mark.gpu
def test_rccl_refused_on_one_gpu():
    """transport "rccl" with both device rings on the one GPU: refused by the receiver, an error
    of fg->run() in both processes (no abort, no hang)."""
    outs = run_pair("RemoteGpu.RcclRefusedOnOneGpu", timeout=120)
    assert "two different GPUs" in outs[1]


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "p2p"])
def test_four_stage_pipeline_gpu(transport):
    """BASELINE C5 at G = 4 as four processes on the one GPU (one decimating stage each, three
    crossings): the middle ranks each hold a receiving crossing on their adapter stream and a sending
    one on their partition stream -- with rccl (the rendezvous test double), two communicators in
    one process, both blocking their streams. Three runs, 1e-5 norm-wise vs the double-precision
    chain at the last rank."""
    env = dict(RCCL_FAKE, QA_EXPECT_TRANSPORT="rccl") if transport == "rccl" else \
        {"QA_TRANSPORT": "p2p", "QA_EXPECT_TRANSPORT": "p2p"}
    run_pair("RemoteGpu.FourStagePipeline", timeout=300, env_extra=env, ranks=4)


@pytest.mark.gpu
def test_rccl_backpressure_holds_sender_stream():
    """A full receiving ring (slow host consumer) while the sender is inside ncclSend: bit-exact
    over two runs, and the double reports that sends waited for their receives (> 1 ms)."""
    outs = run_pair("RemoteGpu.FullRingBackpressure", timeout=300, env_extra=dict(RCCL_FAKE, QA_EXPECT_TRANSPORT="rccl"))
    assert "waited > 200 us" in outs[0]


@pytest.mark.gpu
def test_rccl_rendezvous_negative_control_gpu():
    """The negative control on device rings: the gate kernels hold both streams until the double's
    bounded wait (4 s) gives up; fg->run() raises "rendezvous timed out" in both processes and every
    stream drains (no kernel outlives its bound)."""
    outs = run_pair("RemoteGpu.RendezvousMisorderTimesOut", timeout=120,
                    env_extra=dict(RCCL_FAKE, FAKE_RCCL_MISORDER="1", FAKE_RCCL_TIMEOUT_S="4"))
    assert all("rendezvous timed out" in o for o in outs)
