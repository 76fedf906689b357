"""Cross-process flowgraphs (gr::domain_adapter_remote): each C++ case in
tests/cpp/qa_remote_edge.cpp runs as TWO processes (ranks 0 and 1) that build the same
flowgraph and domain list and each run their own domains, joined by TCP-controlled
crossing edges -- host rings over the socket on CPU; device rings (hip_buffer) on the GPU,
staged through pinned memory because both ranks share the box's one GPU (RCCL needs two
devices; that transport is selected automatically on a multi-GPU node)."""
import os
import random
import socket
import subprocess

import pytest

from tests.conftest import ROOT

EXE = os.path.join(ROOT, "build", "tests", "qa_remote_edge")


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


def run_pair(case, timeout=120):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-s", "-C", ROOT, "tests"], check=True)
    port = free_port_block()
    procs = []
    for r in (0, 1):
        env = dict(os.environ, QA_RANK=str(r), QA_PORT=str(port))
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


@pytest.mark.parametrize("case", ["RemoteCpu.ChainRestart", "RemoteCpu.TwoCrossingsBothWays",
                                  "RemoteCpu.ReaderFinishesFirst", "RemoteCpu.TagsCrossProcesses"])
def test_remote_edges_cpu(case):
    run_pair(case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["RemoteGpu.DeviceChainRestart", "RemoteGpu.DecimatingPipelineC5",
                                  "RemoteGpu.DeviceTags"])
def test_remote_edges_gpu(case):
    run_pair(case, timeout=300)
