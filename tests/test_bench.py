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


ARGS = ["--steps", "3", "--warmup", "1", "--log2n", "22", "--out-buf-mib", "64", "--no-cpu", "--legs-log2n", "22"]


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
    # the other single-GPU configs beside the headline, each with its kernel roofline and parity
    for leg in ("c2", "c4", "decim2", "decim4"):
        L = d[leg]
        assert "error" not in L, (leg, L)
        assert L["parity"]["ok"], (leg, L)
        assert L["timed_launches"] >= 10 and 0 < L["frac"] < 1.2 and L["value"] > 0, (leg, L)
        assert L["launching_blocks"] == 1, (leg, L)  # fused: one launching block per flowgraph
        assert L["timed_launches"] == L["steps"], (leg, L)  # one launch per batch
    assert d["c2"]["parity"]["mismatches"] == 0
    assert d["c2"]["block"].startswith("fused(multiply_const") and d["c4"]["block"].startswith("fused(fft_vcc"), d
    assert d["c1"]["value"] > 0 and d["c1"]["threads"] == 4


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
def test_chain_bench_kernel_timing(torch_cuda):
    """scheduler_hip's kernel timing (nsr_chain_bench_stats): only launching work() calls are
    counted -- the nop source / head and the sink are not -- and with fusion the four
    multiply_const_cc blocks are one block with one launch per batch, timed every launch."""
    import numpy as np
    from newsched_amd import nsr
    import bench

    n = 1 << 20
    cb = nsr.ChainBench(nsr.CHAIN_MUL_CONST_CC, bench.C2_KS, n, out_buf_bytes=16 << 20)
    assert cb.stats()["launches"] == 0
    cb.set_batches(3)
    cb.run()
    st = cb.stats()
    assert st["launching_blocks"] == 1 and st["launches"] == 3 and st["samples"] == 3 * n, st
    assert st["kernel_ms"] > 0
    cb.close()
    # the decimator: output samples counted (n / D per batch)
    cb = nsr.ChainBench(nsr.CHAIN_FIR, bench.firwin(127, 0.45), n, decim=4, out_buf_bytes=16 << 20)
    cb.run()
    st = cb.stats()
    assert st["launches"] >= 1 and st["samples"] == n // 4, st
    cb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("decim", [1, 2, 4])
def test_chain_bench_time_shard(torch_cuda, decim):
    """A leg's flowgraph on a time shard (first_index > 0, as rank r streams x[rN, (r+1)N)): the FIR's
    initial history is the shard's regenerated halo, so EVERY output of the first batch -- the head
    included -- equals the oracle's filter of the continuous stream; C2 / C4 tails start at the
    shard's offset (bit-exact / 1e-5)."""
    import numpy as np
    from newsched_amd import nsr
    from oracle import oracle as orc
    import bench

    n, first = 1 << 14, 3 * (1 << 14) + 1024
    taps = bench.firwin(127, 0.45)
    cb = nsr.ChainBench(nsr.CHAIN_FIR, taps, n, decim=decim, first_index=first, out_buf_bytes=1 << 20)
    cb.run()
    y = cb.tail(n // decim)
    cb.close()
    xw = orc.synth(n + 126, first - 126)
    ok, err, scale = orc.tol_ok(y, orc.fir_ccf(xw[126:], taps, decim, hist=xw[:126]))
    assert ok, (decim, err, scale)
    if decim == 1:
        cb = nsr.ChainBench(nsr.CHAIN_MUL_CONST_CC, bench.C2_KS, n, first_index=first, out_buf_bytes=1 << 20)
        cb.run()
        y = cb.tail(n)
        cb.close()
        assert np.array_equal(y, orc.mul_const_chain_cc(orc.synth(n, first), bench.C2_KS))
        n4 = 1 << 18
        cb = nsr.ChainBench(nsr.CHAIN_CHANNELIZER, bench.c4_weights(), n4, first_index=first, out_buf_bytes=4 << 20)
        cb.run()
        y = cb.tail(4096)
        cb.close()
        ok, err, scale = orc.tol_ok(y, orc.channelizer1024(orc.synth(4096, first + n4 - 4096), bench.c4_weights()))
        assert ok, ("c4", err, scale)


@pytest.mark.gpu
def test_chain_bench_shard_near_stream_start(torch_cuda):
    """A shard that starts fewer than L - 1 samples into the stream: its history is the stream's
    first samples preceded by zeros (before the round-6 fix the history indices wrapped below 0 and
    regenerated unrelated samples), so the outputs equal the oracle's filter from the stream start."""
    import numpy as np
    from newsched_amd import nsh, nsr
    from oracle import oracle as orc
    import bench

    n, first = 1 << 14, 40
    taps = bench.firwin(127, 0.45)
    for decim in (1, 4):
        cb = nsr.ChainBench(nsr.CHAIN_FIR, taps, n, decim=decim, first_index=first, out_buf_bytes=1 << 20)
        cb.run()
        y = cb.tail(n // decim)
        cb.close()
        xs = orc.synth(first + n, 0)
        ref = orc.fir_ccf(xs[first:], taps, decim, hist=np.concatenate([np.zeros(126 - first, np.complex64), xs[:first]]))
        ok, err, scale = orc.tol_ok(y, ref)
        assert ok, (decim, err, scale)
    with pytest.raises(nsh.NshError, match="decim"):
        nsr.ChainBench(nsr.CHAIN_FIR, taps, n, decim=0, out_buf_bytes=1 << 20)


@pytest.mark.gpu
def test_bench_c5_single_gpu(torch_cuda):
    """C5 at G = 1 (all four stages in one scheduler_hip domain) through the same leg."""
    out = subprocess.run([sys.executable, "bench.py", "--c5", "on", "--c5-log2n", "22"] + ARGS, cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    c5 = _json_line(out.stdout)["c5_pipeline"]
    assert c5["ok"] and c5["parity"]["ok"], c5
