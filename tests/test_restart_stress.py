"""Regression: restarting a cross-domain flowgraph (host scheduler_mt domain -> H2D ->
scheduler_hip FIR -> D2H -> host sink) must never hang. Before the two-phase start
(flowgraph::start calls prepare_run() on every scheduler before starting any) the second run of
a fresh flowgraph hung within ~3-40 iterations: the GPU scheduler reset its edges' done flags
after the host threads had already started the run and acted on a stale flag
(tools/c3host_stress.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_cross_domain_restart_does_not_hang(torch_cuda):
    exe = os.path.join(ROOT, "build", "tools", "c3host_stress")
    assert os.path.exists(exe), "build() first"
    r = subprocess.run([exe, "120", "18"], capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stdout[-500:] + r.stderr[-500:]
    assert "iter 119 destroyed" in r.stdout
    assert "sink consumed" not in r.stdout, r.stdout[-500:]
