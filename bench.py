#!/usr/bin/env python3
"""Headline benchmark: MSamples/s through the 127-tap fir_filter_ccf flowgraph (BASELINE
config C3: 2^28-sample complex-float stream, one MI355X per rank).

A step = one N-sample batch of the rank's shard through the flowgraph nop_source ->
nop_head -> [HBM-resident hip_buffer ring, preloaded] -> gr::hip::fir_filter_ccf -> [hip_buffer]
-> null_sink, all inside one scheduler_hip GPU domain (include/nsr_flowgraph.h). The timed
region is ONE flowgraph run that streams K batches (nop_head passes K*N items; the resident ring
holds x twice, so every batch reads x from HBM and the FIR's history carries over as in any
continuous stream): K launches queued back to back on the partition stream, start and drain of
the run inside the timed region. Inputs are resident in HBM before timing starts. (The restart
cost of a run -- start, the executor pass, launch latency, drain detection, ~20-35 us -- is
measured by tools/probe/stream_gap.py at K = 1) With --gpus N every rank (one process per GPU) streams its own contiguous time
shard x[rank*N, (rank+1)*N) with the 126-sample halo regenerated from the counter-based
source: weak scaling, no data-path collective.

Ranks: under torchrun (WORLD_SIZE set) this process is one rank. Without it, `--gpus N > 1`
starts N child processes of this script itself (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set,
before anything here touches the GPU), relays rank 0's line and exits with the first
failing child's code. `n_gpus` is the number of ranks the process group saw (all_reduce).

At world > 1, after the headline timing, a second leg runs BASELINE config 5: the 4-stage
decimating FIR chain domain-partitioned across the ranks (G = 2: stages {1,2}|{3,4};
G = 4: one stage per rank; 8 ranks = 2 time shards x 4) over domain_adapter_remote, RCCL
forced when every rank has its own GPU. Its rate, transports and tail parity go into the
`c5_pipeline` field; a failure there is reported, not fatal to the headline.

Prints ONE JSON line (rank 0) with the roofline of the FIR kernel (HIP events around each
launch on the partition stream, algorithmic 16 B/sample) and the CPU baseline (the
scheduler_mt CPU path restated, timed on this host, rank 0 at N=1).

    python bench.py [--gpus N --steps K --warmup W] [--log2n 28] [--algo auto|mfma|direct]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_SAMPLE = 16  # algorithmic: read x (8 B) + write y (8 B) per output sample
FLOP_PER_SAMPLE = 508  # 127 taps x 2 (re, im) x FMA
METRIC = "MSamples/s through 127-tap fir_filter_ccf flowgraph; % HBM roofline at 1/8 GPU"
C5_HALO = 1904  # >= 126*(1+2+4+8) = 1890 input samples, a multiple of the total decimation 16


def firwin(ntaps, cutoff):
    import scipy.signal as ss

    return ss.firwin(ntaps, cutoff).astype(np.float32)  # C3: (127, 0.2); C5: (127, 0.45)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def free_port():
    """A free TCP port below the kernel's ephemeral range (ip_local_port_range): a port inside it
    can be handed to a client's connect() as its source port while the server is not listening
    yet, and such a client then connects to itself (GPUTEST_r04)."""
    import random
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo = int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        lo = 32768
    for _ in range(500):
        p = random.randrange(10000, max(lo, 10001))
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
            return p
    with socket.socket() as s:  # nothing free below the range: let the kernel choose
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def load_pmc_traffic(kernel, samples_per_launch, summary="pmc_fir.json"):
    """HBM bytes per launch from a committed PMC summary (profiles/pmc_fir.json for the FIR,
    profiles/pmc_casc.json for the C5 kernel; produced by tools/pmc_summary.py from separate
    rocprofv3 --pmc passes, gfx950 FETCH_SIZE x2 correction applied there), scaled to this
    launch size. kernel: the template name as rocprof reports it, e.g. "k_fir_mfma12<5>"."""
    p = os.path.join(ROOT, "profiles", summary)
    try:
        with open(p) as f:
            d = json.load(f)
        return float(d[kernel]["hbm_bytes_per_sample"]) * samples_per_launch, d.get("_source", "profiles/" + summary)
    except (OSError, KeyError, ValueError, TypeError):
        return None, None


def spawn_ranks(n):
    """Start n ranks of this script (never exec: the children are fresh processes) and
    relay their output; returns the exit code. Nothing in this process touches the GPU."""
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               LOCAL_WORLD_SIZE=str(n), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
    rc = 0
    failed_at = None
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc, failed_at = c, time.time()
        if rc != 0 and procs and time.time() - failed_at > 30:
            for p in procs:  # peers left waiting in a collective on the failed rank
                p.kill()
        time.sleep(0.05)
    return rc


def c5_layout(world):
    """(stage groups G, time shards) for `world` ranks: G = 4 when it divides world, else 2,
    else 1 (G=2 {1,2}|{3,4}; G=4 one stage per GPU; G=8 2 shards x 4)."""
    for g in (4, 2, 1):
        if world % g == 0:
            return g, world // g
    return 1, world


def run_c5(a, dist, backend, rank, world, device, torch, orc, nsr):
    """BASELINE config 5 over the ranks (see the module docstring)."""
    G, shards = c5_layout(world)
    group, shard = rank % G, rank // G
    n = 1 << a.c5_log2n
    taps = firwin(127, 0.45)
    first = max(0, shard * n - C5_HALO)  # shards > 0 start with the chain's halo (discarded)
    n_in = shard * n + n - first
    # Rendezvous: rank 0 makes a fresh directory (one node) and a job nonce; the receiving end of
    # each crossing listens on a port the kernel picks and publishes it in <dir>/shard<s>/, the
    # sending end waits for that entry (no derived port numbers: GPUTEST_r04).
    rdv = [None, None]
    if rank == 0 and world > 1:
        import random
        import tempfile
        rdv = [tempfile.mkdtemp(prefix="nsh_c5_"), random.getrandbits(63)]
        for s_ in range(shards):
            os.makedirs(os.path.join(rdv[0], "shard%d" % s_))
    if dist is not None:
        dist.broadcast_object_list(rdv, src=0)
    rdv_dir = os.path.join(rdv[0], "shard%d" % shard) if rdv[0] else ""
    own_gpus = torch.cuda.device_count() >= world
    transport = a.c5_transport if a.c5_transport != "default" else ("rccl" if own_gpus and world > 1 else "auto")
    res = {"layout": "G=%d stage groups x %d time shards" % (G, shards), "stages": "4 x fir_filter_ccf(firwin(127,0.45), D=2)",
           "samples_per_shard": n, "transport_requested": transport}
    # The leg runs in a daemon thread under a deadline (--c5-timeout): on the driver's first
    # multi-GPU run it is the first execution of the RCCL edge transport, and a hang there must
    # not cost the headline line. No collective is issued inside the thread (a rank stuck in it
    # would pair its peers' collectives wrongly); each rank times its own runs, max over ranks.
    box = {"pipe": None, "el": 0.0, "ok": False, "err": 0.0, "tr": "", "status": 2.0}

    def leg():
        try:
            pipe = box["pipe"] = nsr.C5Pipeline(taps, n_in, group=group, n_groups=G, device=device, first_index=first,
                                                rendezvous_dir=rdv_dir, nonce=rdv[1] or 0, transport=transport,
                                                buf_bytes=a.c5_buf_mib << 20)
            for _ in range(a.c5_warmup):
                pipe.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.c5_steps):
                pipe.run()
            torch.cuda.synchronize()
            box["el"] = time.perf_counter() - t0
            ok, err = True, 0.0
            if pipe.last:
                m = 4096
                J = (first + n_in) // 16  # one past the last output (global output index)
                lo = 16 * (J - m) - C5_HALO
                y_ref = orc.synth(16 * m + C5_HALO, lo)
                for _ in range(4):
                    y_ref = orc.fir_ccf(y_ref, taps, decim=2)
                ok, err, _ = orc.tol_ok(pipe.tail(m), y_ref[-m:])
            tr = pipe.transport()
            if "rccl" in tr:
                tr += " [%s]" % (nsr.rccl_library() or "?")
            box.update(ok=ok, err=err, tr=tr, status=0.0)
        except Exception as e:  # reported, not fatal: the headline is already measured
            box.update(status=1.0, error=str(e)[:300])

    import threading

    th = threading.Thread(target=leg, daemon=True)
    th.start()
    th.join(a.c5_timeout)
    if th.is_alive():
        box["error"] = "timed out after %.0f s" % a.c5_timeout
        res["timed_out"] = True
    el, ok, err, tr, status = box["el"], box["ok"], box["err"], box["tr"], box["status"]
    if "error" in box:
        res["error_rank%d" % rank] = box["error"]
    pipe = None if th.is_alive() else box["pipe"]
    if dist is not None:
        dev_kind = "cuda" if backend == "nccl" else "cpu"
        v = torch.tensor([el, 0.0 if ok else 1.0, err, status], dtype=torch.float64, device=dev_kind)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        el, ok, err, status = float(v[0]), v[1].item() == 0.0, float(v[2]), float(v[3])
        trs = [None] * world
        errs = [None] * world
        dist.all_gather_object(trs, tr)
        dist.all_gather_object(errs, res.get("error_rank%d" % rank))
        res["transports"] = {str(r): t for r, t in enumerate(trs) if t}
        for r, e in enumerate(errs):
            if e:
                res["error_rank%d" % r] = e
    else:
        res["transports"] = {"0": tr}
    if pipe is not None:
        pipe.close()
    if rdv[0] and status != 2.0:  # (status is the max over ranks: the same decision everywhere)
        if dist is not None:
            dist.barrier()  # every rank's pipeline is closed
        if rank == 0:
            import shutil
            shutil.rmtree(rdv[0], ignore_errors=True)
    res["ok"] = status == 0.0
    res["_abandoned_any"] = status == 2.0  # some rank's leg is still running: exit hard after the line
    if status == 0.0:
        res.update({"steps": a.c5_steps, "warmup": a.c5_warmup, "ms_per_step": round(el / a.c5_steps * 1e3, 3),
                    "value": round(shards * n * a.c5_steps / el / 1e6, 1), "unit": "MSamples/s (input, whole job)",
                    "parity": {"check": "last 4096 outputs of every shard vs the oracle's 4-stage chain",
                               "max_abs_err": err, "ok": bool(ok)}})
    return res


def leg_clock(work, nsh, real_ms=8.0):
    """The shader clock while `work` (untimed repeats of a leg, >= real_ms long) runs: a one-wave
    sampler on a side stream (nsh_clock_sample: SQ cycles over the 100 MHz real-time counter),
    MI355X_MICROARCH.md's DVFS give-back read in-process (tools/pmc_clock.sh measures the same with
    GRBM_GUI_ACTIVE). None if it could not be taken."""
    try:
        cs = nsh.ClockSampler(real_ms)
        cs.start()
        work()
        return round(cs.mhz(), 1)
    except Exception:  # a measurement aid, never fatal to the line
        return None


def run_fp32_leg(a, n, taps, first, device, barrier, dist, tdev, torch, orc, nsr, nsh):
    """The same C3 flowgraph with the exact-fp32 matrix form (NSH_FIR_MFMA_F32: no operand
    split, fp32 products and sums) -- what the ceiling is without split precision."""
    fb = nsr.FirBench(taps, n, device=device, algo=nsh.FIR_MFMA_F32, first_index=first,
                      out_buf_bytes=a.out_buf_mib << 20)
    steps = max(10, a.steps // 4)
    # warm-up by time as well as by count: the chip comes from the headline's power-limited ~1.1 GHz
    # and this MFMA-bound leg follows the clock; 3 launches (~4 ms) left it mid-ramp at --steps 20
    # (r06l: 37.6 % at 2022 MHz there vs 42.8 % at 2168 MHz with the default --steps 100, r06g)
    tw, runs = time.perf_counter(), 0
    while runs < max(3, a.warmup // 2) or time.perf_counter() - tw < a.legs_warmup_s:
        fb.run()
        runs += 1
    barrier()
    st0 = fb.stats()  # cumulative over the FIR's timed launches
    l0 = st0["launches"]
    t0 = time.perf_counter()
    for _ in range(steps):
        fb.run()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    st = fb.stats()
    launches = st["launches"] - l0
    kms, samples = st["kernel_ms"] - st0["kernel_ms"], st["samples"] - st0["samples"]
    avg_ms = kms / launches
    m = 4096
    y = fb.tail(m)  # the timed runs' last output, before the clock's repeats
    lo = first + n - m - (taps.size - 1)
    xw = orc.synth(m + taps.size - 1, lo)
    ok, err, _ = orc.tol_ok(y, orc.fir_ccf(xw[taps.size - 1:], taps, hist=xw[: taps.size - 1]))
    mhz = leg_clock(lambda: [fb.run() for _ in range(10)], nsh)
    fb.close()
    achieved = BYTES_PER_SAMPLE * (samples / launches) / (avg_ms * 1e-3) / 1e9
    world = dist.get_world_size() if dist is not None else 1
    return {"kernel": st["kernel"], "steps": steps, "value": round(world * n * steps / el / 1e6, 1), "unit": "MSamples/s",
            "avg_launch_us": round(avg_ms * 1e3, 2), "achieved_GBs": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "clock_mhz": mhz,
            "parity": {"max_abs_err": err, "ok": bool(ok)}}


def run_copy_leg(n, barrier, torch, nsh):
    """The measured STREAM-copy ceiling beside the spec peak: nsh_copy (k_copy_v4) of
    the headline's 2^log2n complex samples, i.e. the same 16 B per sample the FIR moves, timed with
    HIP events on its stream after a short warm-up, best of 3 x 10 launches. The copy's rate depends
    on where its input and output sit relative to each other in HBM -- 70.4-77.7 % for the same code
    as the output moves by 128 KiB steps inside one allocation (tools/probe/offset_sweep.py,
    profiles/r06p_offset_sweep_fine.log), while the FIR kernels are flat (r06q, r06r) -- so the
    input and output are carved from ONE allocation and the copy is timed at three output offsets
    (2^log2n samples + 0 / 128 KiB / 1 MiB): `GBs` is the best, `by_offset` all three. (Earlier
    rounds timed one pair of fresh buffers: a draw from that range.)"""
    offs = [0, 128 << 10, 1 << 20]
    buf = torch.empty(16 * n + max(offs) + 4096, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    nsh.synth(base, n, 0)
    s = torch.cuda.Stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        nsh.copy(base, base + 8 * n, 8 * n, stream=s)
        s.synchronize()
    reps = 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    by = {}
    for d in offs:
        ms = None
        for _ in range(3):  # best of 3
            e0.record(s)
            for _ in range(reps):
                nsh.copy(base, base + 8 * n + d, 8 * n, stream=s)
            e1.record(s)
            s.synchronize()
            m = e0.elapsed_time(e1) / reps
            ms = m if ms is None else min(ms, m)
        by[d] = ms
    del buf
    best = min(by.values())
    gbs = BYTES_PER_SAMPLE * n / (best * 1e-3) / 1e9
    return {"kernel": "k_copy_v4", "avg_launch_us": round(best * 1e3, 2), "GBs": round(gbs, 1),
            "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4),
            "by_offset": {str(d): round(BYTES_PER_SAMPLE * n / (m * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for d, m in by.items()},
            "placement": "input and output in one allocation, output at 2^log2n samples + offset bytes; best of the offsets"}


C2_KS = [complex(np.float32(np.cos(t)), np.float32(np.sin(t))) for t in (0.1, 0.2, 0.3, 0.4)]  # e^{j{.1,.2,.3,.4}}


def c4_weights():
    """C4's channel weights W[b] = (1 + cos(2 pi b / 1024) / 2) / 1024 (real, complex64)."""
    b = np.arange(1024)
    return ((1.0 + 0.5 * np.cos(2 * np.pi * b / 1024.0)) / 1024.0).astype(np.complex64)


def chain_specs(a):
    """The single-GPU BASELINE configs other than C3 (and C5's fused chain), as scheduler_hip
    flowgraphs over an HBM-resident input ring (nsr.ChainBench): name -> spec."""
    n = 1 << a.legs_log2n
    taps_d = firwin(127, 0.45)  # the C5 stage filter, alone, at D = 2 and 4
    return {
        "c2": dict(kind="CHAIN_MUL_CONST_CC", params=C2_KS, decim=1, n=n, bps=16.0,
                   workload="C2: 4 x hip::multiply_const_cc (k = e^{j{0.1,0.2,0.3,0.4}}) fused by scheduler_hip into one "
                            "launch per work(), 2^%d-sample batches" % a.legs_log2n),
        "c4": dict(kind="CHAIN_CHANNELIZER", params=c4_weights(), decim=1, n=n, bps=16.0,
                   workload="C4: hip::fft_vcc(1024) -> hip::multiply_const_vcc(W) -> hip::fft_vcc(1024, inverse) fused by "
                            "scheduler_hip into the channelizer, 2^%d samples (2^%d frames) per batch"
                            % (a.legs_log2n, a.legs_log2n - 10)),
        "decim2": dict(kind="CHAIN_FIR", params=taps_d, decim=2, n=n, bps=8.0 + 8.0 / 2,
                       workload="hip::fir_filter_ccf(firwin(127,0.45), decim 2), 2^%d input samples per batch" % a.legs_log2n),
        "decim4": dict(kind="CHAIN_FIR", params=taps_d, decim=4, n=n, bps=8.0 + 8.0 / 4,
                       workload="hip::fir_filter_ccf(firwin(127,0.45), decim 4), 2^%d input samples per batch" % a.legs_log2n),
    }


def chain_parity(name, spec, y, first, orc):
    """Tail of the last batch vs the oracle: C2 bit-exact, the rest within the north-star 1e-5."""
    n, m = spec["n"], y.size
    if name == "c2":
        ref = orc.mul_const_chain_cc(orc.synth(m, first + n - m), spec["params"])
        ok = bool(np.array_equal(y.view(np.uint64), ref.view(np.uint64)))
        return {"check": "last %d outputs bit-exact vs the oracle's chain" % m, "ok": ok,
                "mismatches": int(np.count_nonzero(y.view(np.uint64) != ref.view(np.uint64)))}
    if name == "c4":
        ref = orc.channelizer1024(orc.synth(m, first + n - m), spec["params"])
        ok, err, scale = orc.tol_ok(y, ref)
        return {"check": "last %d frame(s) vs the oracle's double-precision DFT channelizer" % (m // 1024),
                "max_abs_err": err, "scale": scale, "ok": bool(ok)}
    D, taps = spec["decim"], spec["params"]
    L1 = taps.size - 1  # the window lies inside the batch (its history: the batch's own samples)
    xw = orc.synth(m * D + L1, first + n - m * D - L1)
    ok, err, scale = orc.tol_ok(y, orc.fir_ccf(xw[L1:], taps, D, hist=xw[:L1]))
    return {"check": "last %d outputs vs the oracle (double accumulation)" % m, "max_abs_err": err, "scale": scale,
            "ok": bool(ok)}


def run_chain_leg(a, name, spec, rank, device, barrier, dist, tdev, torch, orc, nsr, nsh):
    """One config as a scheduler_hip flowgraph streaming K batches in one run (as the headline):
    wall rate, HIP-event time of every launch of the (fused) block that does the work
    (scheduler_hip kernel timing), the shader clock, and the last batch's tail against the oracle."""
    n, D = spec["n"], spec["decim"]
    first = rank * n
    fb = nsr.ChainBench(getattr(nsr, spec["kind"]), spec["params"], n, device=device, decim=D, first_index=first,
                        out_buf_bytes=max(64 << 20, n * 8))  # edges of a whole batch: one launch per batch
    try:
        t0 = time.perf_counter()
        fb.set_batches(4)
        while time.perf_counter() - t0 < a.legs_warmup_s:
            fb.run()
        steps = max(10, a.steps // 4)
        fb.set_batches(steps)
        barrier()
        st0 = fb.stats()
        t0 = time.perf_counter()
        fb.run()
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        st = fb.stats()
        m = 4096 if name != "c4" else 2048
        par = chain_parity(name, spec, fb.tail(m), first, orc)  # the timed run's last batch

        def more():
            fb.set_batches(16)
            fb.run()

        mhz = leg_clock(more, nsh)
    finally:
        fb.close()
    launches = st["launches"] - st0["launches"]
    if launches <= 0:
        raise RuntimeError("no timed launches of %s (scheduler_hip kernel timing)" % st["block"])
    kms = st["kernel_ms"] - st0["kernel_ms"]
    in_samples = (st["samples"] - st0["samples"]) * D
    avg_ms = kms / launches
    achieved = spec["bps"] * (in_samples / launches) / (avg_ms * 1e-3) / 1e9
    world = dist.get_world_size() if dist is not None else 1
    kernel = {"c2": "k_map_c_v4", "c4": "k_chan1024"}.get(name)
    if kernel is None:  # the decimators: the kernel their plan resolves to
        fp = nsh.FirPlan(spec["params"], D, device=device)
        kernel = fp.kernel
        fp.close()
    out = {"workload": spec["workload"], "kernel": kernel, "block": st["block"], "launching_blocks": st["launching_blocks"],
            "steps": steps, "value": round(world * n * steps / el / 1e6, 1), "unit": "MSamples/s (input)",
            "ms_per_step": round(el / steps * 1e3, 4), "timed_launches": launches,
            "avg_launch_us": round(avg_ms * 1e3, 2), "bytes_per_input_sample": spec["bps"],
            "achieved_GBs": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
            "flowgraph_frac": round(spec["bps"] * n / (el / steps) / 1e9 / HBM_PEAK_GBS, 4),
            "clock_mhz": mhz, "parity": par}
    tr, src = load_pmc_traffic(kernel, in_samples / launches, "pmc_legs.json")
    if tr is not None:
        out["traffic"] = int(tr)
        out["traffic_source"] = ("HBM B/input sample from separate rocprofv3 --pmc passes (%s), scaled to this "
                                 "launch size; not measured in this run" % src)
    return out


def run_c1_leg(reps=7):
    """BASELINE C1 on the host (the reference's bm_copy flowgraph): null_source -> head(2^20) ->
    copy -> null_sink on scheduler_mt, 32 KiB buffers, median of `reps` runs."""
    runs = [nsr_c1_run() for _ in range(reps)]
    secs = sorted(r[0] for r in runs)
    med = secs[len(secs) // 2]
    return {"workload": "C1: null_source -> head(2^20) -> copy -> null_sink, scheduler_mt thread per block, "
                        "vmcircbuf 32 KiB buffers (CPU only)", "value": round((1 << 20) / med / 1e6, 2),
            "unit": "MSamples/s", "median_of": reps, "ms_per_run": round(med * 1e3, 3), "threads": runs[0][1],
            "us_per_4096_item_call": round(med / ((1 << 20) / 4096) * 1e6, 2),
            "note": "drain-based termination: the reference's fixed 100 ms sleep per run "
                    "(runtime/lib/flowgraph_monitor.cpp:27) is not paid"}


def nsr_c1_run():
    from newsched_amd import nsr

    return nsr.c1_run(1 << 20, 32768)


def run_c5_fused_leg(a, first, device, barrier, dist, tdev, torch, orc, nsh):
    """BASELINE config C5's chain 4 x fir_filter_ccf(firwin(127, 0.45), 2) as the fused kernel
    scheduler_hip puts in its place (hip::fir_filter_cascade_ccf -> nsh_fir_cascade_ccf,
    k_fir_pfft2<16>): 2^log2n resident input samples per GPU, one launch per step, HIP events on
    the launch stream; roofline against the chain's 8.5 B per input sample (read 8, write 0.5)."""
    n = 1 << a.c5_fused_log2n
    taps = firwin(127, 0.45)
    plan = nsh.FirCascadePlan([(taps, 2)] * 4, device=device)
    n_out = n // 16
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, first)
    hist = None
    if first > 0:  # the shard's halo, regenerated
        hist = torch.from_numpy(orc.synth(plan.hist_len, first - plan.hist_len)).cuda()
    y = torch.empty(n_out, dtype=torch.complex64, device="cuda")
    hout = torch.empty(plan.hist_len, dtype=torch.complex64, device="cuda")
    s = torch.cuda.Stream()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        plan(x, hist, hout, y, n_out, stream=s)
        s.synchronize()
    steps = max(10, a.steps // 4)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    barrier()
    t0 = time.perf_counter()
    with torch.cuda.stream(s):
        for e0, e1 in ev:
            e0.record(s)
            plan(x, hist, hout, y, n_out, stream=s)
            e1.record(s)
    s.synchronize()
    barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    avg_ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / steps

    def more():
        with torch.cuda.stream(s):
            for _ in range(24):
                plan(x, hist, hout, y, n_out, stream=s)
        s.synchronize()

    m = 4096
    lo = first + n - 16 * m - C5_HALO
    xr = orc.synth(16 * m + C5_HALO, lo)
    for _ in range(4):
        xr = orc.fir_ccf(xr, taps, 2)
    ok, err, _ = orc.tol_ok(y[-m:].cpu().numpy(), xr[-m:])  # the timed launches' output
    mhz = leg_clock(more, nsh)
    kernel = plan.kernel
    plan.close()
    achieved = 8.5 * n / (avg_ms * 1e-3) / 1e9
    world = dist.get_world_size() if dist is not None else 1
    out = {"kernel": kernel, "workload": "C5: 4 x fir_filter_ccf(firwin(127,0.45), 2) fused into one "
           "fir_filter_cascade_ccf, 2^%d resident input samples per GPU" % a.c5_fused_log2n,
           "steps": steps, "value": round(world * n * steps / el / 1e6, 1), "unit": "MSamples/s (input)",
           "avg_launch_us": round(avg_ms * 1e3, 2), "achieved_GBs": round(achieved, 1),
           "bytes_per_input_sample": 8.5, "frac": round(achieved / HBM_PEAK_GBS, 4), "clock_mhz": mhz,
           "parity": {"check": "last 4096 outputs vs the oracle's 4-stage chain (double accumulation)",
                      "max_abs_err": err, "ok": bool(ok)}}
    tr, src = load_pmc_traffic(kernel, n, "pmc_casc.json")
    if tr is not None:
        out["traffic"] = int(tr)
        out["traffic_source"] = ("HBM B/input sample from separate rocprofv3 --pmc passes (%s), scaled to this "
                                 "launch size; not measured in this run" % src)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--min-warmup-s", type=float, default=1.0,
                    help="keep warming up (untimed runs) until this long has passed: clocks settle")
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--algo", default="auto", choices=["auto", "mfma", "mfma_f32", "direct"])
    ap.add_argument("--fp32-leg", choices=["on", "off"], default="on",
                    help="also time the exact-fp32 matrix form (NSH_FIR_MFMA_F32) on the same flowgraph")
    ap.add_argument("--timing-stride", type=int, default=2,
                    help="HIP-event timing on every k-th FIR launch of the timed run (each timed launch costs its "
                         "event packets, ~7 us)")
    ap.add_argument("--out-buf-mib", type=int, default=2048, help="FIR output hip_buffer (default: one launch per 2^28-sample step)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-log2n", type=int, default=28, help="CPU baseline sample (default: the full stream)")
    ap.add_argument("--c5", choices=["auto", "on", "off"], default="auto", help="C5 pipeline leg (auto: at world > 1)")
    ap.add_argument("--c5-fused", choices=["on", "off"], default="on",
                    help="C5's chain as the fused kernel (k_fir_pfft2<16>) on resident input, every rank")
    ap.add_argument("--c5-fused-log2n", type=int, default=28)
    ap.add_argument("--legs", choices=["auto", "on", "off"], default="auto",
                    help="the other single-GPU configs beside the headline: C1 (CPU), C2, C4, decimators D=2/4 "
                         "(auto: at world 1 only -- they are single-GPU configs, and a rank that fails one must "
                         "not leave its peers waiting in the leg's barriers of a multi-GPU run)")
    ap.add_argument("--legs-log2n", type=int, default=28)
    ap.add_argument("--legs-warmup-s", type=float, default=0.5,
                    help="untimed warm-up per leg (seconds, at least): the clock settles for that leg's kernel")
    ap.add_argument("--c5-log2n", type=int, default=26)
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--c5-warmup", type=int, default=2)
    ap.add_argument("--c5-buf-mib", type=int, default=64)
    ap.add_argument("--c5-transport", default="default", choices=["default", "auto", "rccl", "p2p", "socket"])
    ap.add_argument("--c5-timeout", type=float, default=120.0, help="deadline for the C5 leg (s)")
    ap.add_argument("--rank-check", action="store_true", help=argparse.SUPPRESS)  # launcher test (CPU, gloo)
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(spawn_ranks(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is None:  # under torchrun without --gpus: one rank per launched process
        a.gpus = world
    if world != a.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world))

    import torch

    backend = os.environ.get("NSH_BENCH_BACKEND", "nccl")  # nccl = RCCL; gloo only for rehearsals
    if a.rank_check:
        backend = "gloo"
    dist = None
    device = 0
    if not a.rank_check:
        # one process per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share devices
        device = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend=backend)
    tdev = "cuda" if backend == "nccl" else "cpu"
    ranks_seen = world
    if dist is not None:
        one = torch.ones(1, dtype=torch.int64, device=tdev)
        dist.all_reduce(one)
        ranks_seen = int(one.item())
    if a.rank_check:
        if rank == 0:
            print(json.dumps({"n_gpus": ranks_seen, "world": world}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    from newsched_amd import nsh, nsr
    from oracle import oracle as orc  # checker only: tail parity + CPU-baseline inputs

    algo = {"auto": nsh.FIR_AUTO, "mfma": nsh.FIR_MFMA, "mfma_f32": nsh.FIR_MFMA_F32, "direct": nsh.FIR_DIRECT}[a.algo]
    n = 1 << a.log2n
    taps = firwin(127, 0.2)
    first = rank * n  # this rank's time shard
    fb = nsr.FirBench(taps, n, device=device, algo=algo, first_index=first, out_buf_bytes=a.out_buf_mib << 20)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # Warm-up: at least --warmup batches and at least --min-warmup-s seconds of them (the
    # chip's clocks take ~20 back-to-back launches to settle), untimed.
    tw = time.perf_counter()
    warm = 0
    fb.set_batches(max(1, a.warmup))
    while warm < a.warmup or time.perf_counter() - tw < a.min_warmup_s:
        fb.run()
        warm += max(1, a.warmup)
    warm_s = time.perf_counter() - tw
    fb.set_batches(a.steps)
    fb.set_timing_stride(a.timing_stride)  # every stride-th launch carries its event pair
    barrier()
    st0 = fb.stats()  # cumulative HIP-event kernel time / samples of the FIR's timed launches
    launches0 = st0["launches"]
    t0 = time.perf_counter()
    fb.run()  # one flowgraph run streaming K batches = K steps
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = fb.stats()

    # parity on the measured path: the last 4096 outputs of the timed run vs the oracle, read
    # before anything else runs the flowgraph again
    m = 4096
    y = fb.tail(m)
    lo = first + n - m - (taps.size - 1)
    xw = orc.synth(m + taps.size - 1, lo)
    y_ref = orc.fir_ccf(xw[taps.size - 1:], taps, hist=xw[: taps.size - 1])
    ok, err, scale = orc.tol_ok(y, y_ref)

    def more():  # untimed: the clock the FIR runs at under the same stream of batches
        fb.set_batches(24)
        fb.run()

    clock_mhz = leg_clock(more, nsh)
    kms = st["kernel_ms"] - st0["kernel_ms"]
    samples = st["samples"] - st0["samples"]
    algo_used = {1: "direct", 2: "mfma", 5: "mfma_f32"}.get(st["algo"], str(st["algo"]))
    kernel = st["kernel"]
    timed_launches = st["launches"] - launches0
    per_launch_samples = samples / timed_launches
    launches_per_run = n / per_launch_samples  # launches per step (batch); all of one size
    avg_launch_ms = kms / timed_launches
    achieved = BYTES_PER_SAMPLE * per_launch_samples / (avg_launch_ms * 1e-3) / 1e9  # GB/s

    if dist is not None:  # every rank's shard tail must pass; report the worst error
        r = torch.tensor([0.0 if ok else 1.0, err], dtype=torch.float64, device=tdev)
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
        ok, err = r[0].item() == 0.0, float(r[1].item())

    value = world * n * a.steps / elapsed / 1e6  # MSamples/s, whole job
    step_us = elapsed / a.steps * 1e6
    # the flowgraph's own fraction (16 B x samples per step over the whole step, host overhead
    # included) next to the kernel's; the difference is the per-run start / drain overhead
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "MSamples/s",
        "n_gpus": ranks_seen,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "arith": "complex fp32 in and out; 127-tap products as a three-product fp16x2 operand split on the fp16 "
                 "matrix cores with fp32 accumulation (k_fir_mfma12), chunks the split cannot hold on exact fp32 paths; "
                 "the fp32-by-instruction form is the fp32_exact leg",
        "data": "synthetic: counter-based splitmix64 complex-float stream (BASELINE.md §2), HBM-resident before timing",
        "config": {
            "workload": "C3: 127-tap fir_filter_ccf (firwin(127,0.2) fp32 taps) over 2^%d-sample complex-float batches per GPU, "
                        "nop_source->nop_head->[resident hip_buffer]->hip::fir_filter_ccf->[hip_buffer]->null_sink in scheduler_hip; "
                        "the K steps are one flowgraph run streaming K batches" % a.log2n,
            "samples_per_gpu": n,
            "ntaps": int(taps.size),
            "fir_algo": algo_used,
            "fir_launches_per_step": launches_per_run,
            "timed_launches": timed_launches,
            "samples_per_launch": int(per_launch_samples),
            "parallelism": "time-sharded replicas x%d (126-sample halo regenerated, no collective)" % world,
        },
        "warmup_done": {"runs": warm, "seconds": round(warm_s, 3), "min_seconds": a.min_warmup_s},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": kernel,
            "avg_launch_us": round(avg_launch_ms * 1e3, 2),
            "algorithmic_bytes_per_launch": int(BYTES_PER_SAMPLE * per_launch_samples),
            "kernel_gflops": round(FLOP_PER_SAMPLE * per_launch_samples / (avg_launch_ms * 1e-3) / 1e9, 1),
            "flowgraph_achieved": round(BYTES_PER_SAMPLE * n / (step_us * 1e-6) / 1e9, 1),
            "flowgraph_frac": round(BYTES_PER_SAMPLE * n / (step_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "overhead_us_per_step": round(step_us - avg_launch_ms * 1e3 * launches_per_run, 2),  # incl. the run's start / drain
            "clock_mhz": clock_mhz,  # shader clock over an untimed repeat (leg_clock)
        },
        "parity": {"check": "last 4096 outputs of the timed run's last step vs oracle (double accumulation), every rank",
                   "max_abs_err": err, "scale": scale, "ok": bool(ok)},
    }
    cp = run_copy_leg(n, barrier, torch, nsh)
    out["roofline"]["copy_measured"] = cp
    out["roofline"]["frac_of_copy"] = round(achieved / cp["GBs"], 4)
    tr, src = load_pmc_traffic(kernel, per_launch_samples)
    if tr is not None:
        out["roofline"]["traffic"] = int(tr)
        out["roofline"]["traffic_source"] = ("HBM B/sample from separate rocprofv3 --pmc passes (%s), scaled to this "
                                             "launch size; not measured in this run" % src)
    fb.close()

    abandoned = False
    if a.fp32_leg == "on" and a.algo == "auto":
        out["fp32_exact"] = run_fp32_leg(a, n, taps, first, device, barrier, dist, tdev, torch, orc, nsr, nsh)

    if a.c5_fused == "on":
        out["c5_fused"] = run_c5_fused_leg(a, rank * (1 << a.c5_fused_log2n), device, barrier, dist, tdev, torch, orc, nsh)

    if a.legs == "on" or (a.legs == "auto" and world == 1):
        for name, spec in chain_specs(a).items():
            try:
                out[name] = run_chain_leg(a, name, spec, rank, device, barrier, dist, tdev, torch, orc, nsr, nsh)
            except Exception as e:  # reported, not fatal: the headline is already measured
                out[name] = {"error": str(e)[:300]}
        if rank == 0:
            out["c1"] = run_c1_leg()

    if a.c5 == "on" or (a.c5 == "auto" and world > 1):
        out["c5_pipeline"] = run_c5(a, dist, backend, rank, world, device, torch, orc, nsr)
        abandoned = out["c5_pipeline"].pop("_abandoned_any")

    if rank == 0 and world == 1 and not a.no_cpu:
        ncpu = 1 << a.cpu_log2n
        xs = orc.synth(1 << 20)  # vector_source data (repeated)
        secs, threads = nsr.cpu_fir_run(taps, xs, ncpu, fixed_buf_size=32768, with_threads=True)
        n_wo = 1 << 24  # the FIR arithmetic alone: the same block's filter() on 4096-sample calls
        wsecs, isa = nsr.cpu_fir_work_only(taps, xs, n_wo, chunk=4096)
        calls = ncpu / 4096
        try:
            affinity = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            affinity = None
        out["cpu_baseline"] = {
            "value": round(ncpu / secs / 1e6, 2),
            "unit": "MSamples/s",
            "cores": threads,  # threads the run used (scheduler_mt: one per block), as the run reports them
            "threads": threads,
            "fir_cores": 1,  # the FIR block's work() runs on its one thread
            "nproc": os.cpu_count(),
            "cpus_allowed": affinity,
            "kind": "port",
            "isa": isa,
            "fir_work_only_msps": round(n_wo / wsecs / 1e6, 2),
            "us_per_call": round(secs / calls * 1e6, 2),
            "us_per_call_split": {"fir_work": round(wsecs / (n_wo / 4096) * 1e6, 2),
                                  "scheduler_handoff": round(secs / calls * 1e6 - wsecs / (n_wo / 4096) * 1e6, 2)},
            "sample": "2^%d samples through vector_source->head->fir_filter_ccf(127 taps, %s fp32)->null_sink, "
                      "scheduler_mt thread-per-block (%d threads; the FIR on one core), vmcircbuf 32768 B default buffers "
                      "(4096-item work() calls); %.2f s on %s. fir_work_only_msps: the same block's filter() alone on "
                      "2^24 samples in 4096-sample calls, no scheduler" % (a.cpu_log2n, isa, threads, secs, cpu_model()),
        }
    if dist is not None and not abandoned:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if abandoned:  # a hung pipeline leg: leave without joining it (the headline is printed)
        sys.stderr.flush()
        os._exit(0)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
