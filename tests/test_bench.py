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


ARGS = ["--steps", "3", "--warmup", "1", "--log2n", "22", "--out-buf-mib", "64", "--no-cpu"]


def _json_line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_launcher_spawns_ranks_cpu():
    """`bench.py --gpus 2` without torchrun starts two ranks itself (the driver's form);
    n_gpus is what the process group counted (gloo here, no GPU touched)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--rank-check"], cwd=ROOT, capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert _json_line(out.stdout) == {"n_gpus": 2, "world": 2}


def test_launcher_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--rank-check"], cwd=ROOT, capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_launcher_without_gpus_flag_takes_world_size():
    """`torchrun --nproc_per_node 2 bench.py` (no --gpus): each rank takes WORLD_SIZE."""
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in (0, 1):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "bench.py", "--rank-check"], cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, env=env))
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    assert _json_line(outs[0][0]) == {"n_gpus": 2, "world": 2}


def test_c5_layout():
    import bench

    assert bench.c5_layout(2) == (2, 1)
    assert bench.c5_layout(4) == (4, 1)
    assert bench.c5_layout(8) == (4, 2)
    assert bench.c5_layout(1) == (1, 1)
    assert bench.c5_layout(6) == (2, 3)


@pytest.mark.gpu
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
    cp = d["roofline"]["copy_measured"]  # the measured copy ceiling beside the spec peak
    assert cp["kernel"] == "k_copy_v4" and 0 < cp["frac_of_peak"] < 1 and d["roofline"]["frac_of_copy"] > 0
    assert d["config"]["workload"].startswith("C3")


@pytest.mark.gpu
def test_fir_bench_stats_cumulative(torch_cuda):
    """nsr_fir_bench_stats counts every timed launch since create (bench.py reads it once on each
    side of its timed loop): launches, samples and kernel time grow run by run."""
    import numpy as np
    from newsched_amd import nsr
    n = 1 << 16
    fb = nsr.FirBench(np.hamming(127).astype(np.float32) / 64, n, out_buf_bytes=8 << 20)
    prev = fb.stats()
    assert prev["launches"] == 0 and prev["samples"] == 0 and prev["kernel_ms"] == 0
    for _ in range(3):
        fb.run()
        st = fb.stats()
        assert st["launches"] > prev["launches"] and st["samples"] == prev["samples"] + n
        assert st["kernel_ms"] > prev["kernel_ms"]
        prev = st
    fb.close()


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
def test_bench_c5_single_gpu(torch_cuda):
    """C5 at G = 1 (all four stages in one scheduler_hip domain) through the same leg."""
    out = subprocess.run([sys.executable, "bench.py", "--c5", "on", "--c5-log2n", "22"] + ARGS, cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    c5 = _json_line(out.stdout)["c5_pipeline"]
    assert c5["ok"] and c5["parity"]["ok"], c5


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
