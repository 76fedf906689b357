"""Run the C++ behaviour tests (tests/cpp/*.cpp, built by `make tests`): the reference's
own scheduler_mt gtests restated against this runtime (CPU), and the GPU flowgraph
tests through scheduler_hip / hip_buffer / gr::hip blocks (GPU)."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

BIN = os.path.join(ROOT, "build", "tests")


def run(name, timeout, *cases):
    exe = os.path.join(BIN, name)
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", ROOT, "tests"], check=True)
    p = subprocess.run([exe, *cases], capture_output=True, text=True, timeout=timeout)
    print(p.stdout)
    print(p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_scheduler_mt_behaviour():
    out = run("qa_scheduler_mt", 600)
    assert "0 failure(s)" in out


@pytest.mark.gpu
def test_hip_flowgraphs():
    out = run("qa_hip_flowgraph", 900)
    assert "0 failure(s)" in out


def test_tags_reference_counts():
    """Reference schedulers/mt/test/qa_tags.cpp OneToOne/t1/t2/t3 with its expected counts, plus
    tags across an in-process domain boundary."""
    out = run("qa_tags", 300, "SchedulerMTTags")
    assert "5 test(s), 0 failure(s)" in out


@pytest.mark.gpu
def test_tags_through_device_edges():
    out = run("qa_tags", 300, "DeviceTags")
    assert "2 test(s), 0 failure(s)" in out


def test_fusion_pass_graph_rewrite():
    """scheduler_hip's fusion passes (elementwise chains, fft -> w -> ifft channelizer) as host
    logic (no device touched)."""
    out = run("qa_fusion", 120)
    assert "10 test(s), 0 failure(s)" in out
