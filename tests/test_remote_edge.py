"""Cross-process flowgraphs (gr::domain_adapter_remote): each C++ case in
tests/cpp/qa_remote_edge.cpp runs as TWO processes (ranks 0 and 1) that build the same
flowgraph and domain list and each run their own domains, joined by TCP-controlled
crossing edges -- host rings over the socket on CPU (plus the "deferred_test" transport,
whose reads of the sender's ring complete late on another thread: the edge's release rule);
device rings (hip_buffer) on the GPU, where both ranks share the box's one GPU: the "p2p"
transport (stream-ordered copies into IPC-mapped landing slots, auto's choice on one GPU) and
the pinned-memory "socket" staging. RCCL needs two devices; auto selects it on a multi-GPU
node (test_bench.py::test_bench_c5_rccl_two_gpus)."""
import os
import random
import socket
import subprocess

import pytest

from tests.conftest import ROOT

EXE = os.path.join(ROOT, "build", "tests", "qa_remote_edge")
FAKE_RCCL = os.path.join(ROOT, "build", "tests", "libfake_rccl.so")


def free_port_block(width=64):
    for _ in range(200):
        base = random.randrange(20000, 60000 - width)
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


def run_pair(case, timeout=120, env_extra=None):
    if not (os.path.exists(EXE) and os.path.exists(FAKE_RCCL)):
        subprocess.run(["make", "-s", "-C", ROOT, "tests"], check=True)
    port = free_port_block(128)
    procs = []
    for r in (0, 1):
        env = dict(os.environ, QA_RANK=str(r), QA_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen([EXE, case], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        print(f"--- rank {r} ---\n{out}")
        assert p.returncode == 0, f"rank {r} failed:\n{out}"
        assert "0 failure(s)" in out and "1 test(s)" in out, out
    return outs


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
             "RemoteGpu.RestartDropsRemainder"]


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
