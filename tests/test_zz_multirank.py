"""bench.py's N>1 path on the GPU box, rehearsed with several ranks on the box's one GPU:
time-sharded ranks (gloo; RCCL refuses two ranks on one device), and BASELINE C5
domain-partitioned over 2, 4 and 8 processes through domain_adapter_remote (p2p, and the rccl
transport against the RCCL rendezvous test double).

This file is named to be collected LAST: these multi-process rehearsals are the
slowest and most environment-sensitive GPU tests, and under `pytest -x` a failure here must not
keep the single-process kernel-parity suites (test_gpu_kernels.py, test_gpu_pfft.py,
test_cpp_runtime.py) from running."""
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT
from tests.test_bench import ARGS, _json_line


@pytest.mark.gpu
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


@pytest.mark.gpu
def test_bench_spawns_ranks_and_c5_leg(torch_cuda):
    """The driver's N>1 form without torchrun: bench.py starts the ranks itself; both shards'
    tails pass; the C5 pipeline leg ({1,2}|{3,4} over domain_adapter_remote; two ranks on one
    GPU negotiate the p2p transport, RCCL needs two GPUs) is parity-green."""
    env = dict(os.environ, NSH_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--c5-log2n", "20"] + ARGS, cwd=ROOT,
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    assert d["n_gpus"] == 2 and d["parity"]["ok"], d
    c5 = d["c5_pipeline"]
    assert c5["ok"] and c5["parity"]["ok"], c5
    assert c5["value"] > 0
    # both ranks share the box's one GPU: auto negotiates the IPC landing-slot transport
    assert "p2p" in c5["transports"]["0"] and "p2p" in c5["transports"]["1"], c5


@pytest.mark.gpu
def test_bench_c5_leg_rccl_transport_with_test_double(torch_cuda):
    """The driver's multi-GPU C5 leg as it will run there (--c5-transport rccl: the ranks' edges on
    domain_adapter_remote's rccl transport, stream-ordered sends / receives on the partition and
    adapter streams) with the RCCL test double (tests/cpp/fake_rccl.c) standing in for the
    library, which refuses two ranks on one GPU: parity-green, every rank reports rccl."""
    fake = os.path.join(ROOT, "build", "tests", "libfake_rccl.so")
    assert os.path.exists(fake), "make tests builds the RCCL test double"
    env = dict(os.environ, NSH_BENCH_BACKEND="gloo", NSH_RCCL_LIB=fake, NSH_REMOTE_TEST_RCCL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--c5-log2n", "20", "--c5-transport", "rccl"] + ARGS,
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    c5 = _json_line(out.stdout)["c5_pipeline"]
    assert c5["ok"] and c5["parity"]["ok"], c5
    assert len(c5["transports"]) == 2 and all(":rccl" in t for t in c5["transports"].values()), c5
    assert all("libfake_rccl.so" in t for t in c5["transports"].values()), c5  # the library bound, recorded


@pytest.mark.gpu
def test_bench_c5_leg_g4_rccl_transport_with_test_double(torch_cuda):
    """The driver's 4-GPU C5 layout (G = 4: one stage per rank, the middle ranks holding a receiving
    and a sending communicator at once) on the rendezvous test double, 4 ranks on the one GPU."""
    fake = os.path.join(ROOT, "build", "tests", "libfake_rccl.so")
    env = dict(os.environ, NSH_BENCH_BACKEND="gloo", NSH_RCCL_LIB=fake, NSH_REMOTE_TEST_RCCL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--c5-log2n", "20", "--c5-transport", "rccl",
                          "--fp32-leg", "off", "--c5-fused", "off"] + ARGS,
                         cwd=ROOT, capture_output=True, text=True, timeout=400, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    c5 = d["c5_pipeline"]
    assert c5["layout"].startswith("G=4"), c5
    assert c5["ok"] and c5["parity"]["ok"], c5
    assert len(c5["transports"]) == 4 and all(":rccl" in t for t in c5["transports"].values()), c5
    # the middle ranks: one receiving and one sending crossing each
    for r in ("1", "2"):
        assert "send" in c5["transports"][r] and "recv" in c5["transports"][r], c5


@pytest.mark.gpu
def test_bench_c5_rccl_two_gpus(torch_cuda):
    """The RCCL edge transport (domain_adapter_remote rccl_transport) end to end: needs two
    GPUs, so it is skipped on the 1-GPU test box and runs on the first multi-GPU lease."""
    if torch_cuda.cuda.device_count() < 2:
        pytest.skip("RCCL edges need two GPUs")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NSH_BENCH_BACKEND")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--c5-log2n", "22", "--c5-transport", "rccl"]
                         + ARGS, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    c5 = _json_line(out.stdout)["c5_pipeline"]
    assert c5["ok"] and c5["parity"]["ok"], c5
    assert all("rccl" in t for t in c5["transports"].values()), c5


@pytest.mark.gpu
def test_bench_c5_leg_g8_rccl_transport_with_test_double(torch_cuda):
    """The driver's 8-GPU C5 layout (two time shards x G = 4, eight ranks: shard s's stage g on rank
    4 s + g, three crossings per shard) on the rendezvous test double, 8 ranks on the one GPU: both
    shards' tails parity-green, every rank on rccl."""
    fake = os.path.join(ROOT, "build", "tests", "libfake_rccl.so")
    env = dict(os.environ, NSH_BENCH_BACKEND="gloo", NSH_RCCL_LIB=fake, NSH_REMOTE_TEST_RCCL="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--c5-log2n", "20", "--c5-transport", "rccl",
                          "--fp32-leg", "off", "--c5-fused", "off"] + ARGS,
                         cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    d = _json_line(out.stdout)
    assert d["n_gpus"] == 8 and d["parity"]["ok"], d
    c5 = d["c5_pipeline"]
    assert c5["layout"] == "G=4 stage groups x 2 time shards", c5
    assert c5["ok"] and c5["parity"]["ok"], c5
    assert len(c5["transports"]) == 8 and all(":rccl" in t for t in c5["transports"].values()), c5
