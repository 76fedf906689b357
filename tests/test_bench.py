"""bench.py end to end on the GPU box: the JSON line's contract at N=1, and the N>1 path
(time-sharded ranks, barrier, max-over-ranks time, per-rank tail parity) rehearsed with two
ranks on one GPU over gloo (RCCL refuses two ranks on one device; the driver's 8-GPU run uses
RCCL on the same code path)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--steps", "3", "--warmup", "1", "--log2n", "22", "--out-buf-mib", "64", "--no-cpu"]


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_one_gpu(torch_cuda):
    out = subprocess.run([sys.executable, "bench.py"] + ARGS, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "parity"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["scaling"] == "weak"
    assert d["parity"]["ok"], d["parity"]
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0 and 0 < d["roofline"]["frac"] < 1
    assert d["config"]["workload"].startswith("C3")


def test_bench_two_ranks_rehearsal(torch_cuda):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, NSH_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2"] + ARGS
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    assert d["n_gpus"] == 2
    assert d["parity"]["ok"], d["parity"]  # both shards' tails (rank 1 starts at sample 2^22)
    assert "2" in d["config"]["parallelism"]
