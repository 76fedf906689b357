#!/usr/bin/env python3
"""Headline benchmark: MSamples/s through the 127-tap fir_filter_ccf flowgraph (BASELINE
config C3: 2^28-sample complex-float stream, one MI355X per rank).

A step = one flowgraph run over the rank's N-sample shard: nop_source -> nop_head(N) ->
[HBM-resident hip_buffer ring, preloaded] -> gr::hip::fir_filter_ccf -> [hip_buffer] ->
null_sink, all inside one scheduler_hip GPU domain (include/nsr_flowgraph.h). Inputs are
resident in HBM before timing starts; the run ends only after the partition stream has
drained. With --gpus N (torchrun, one process per GPU) every rank streams its own
contiguous time shard x[rank*N, (rank+1)*N) with the 126-sample halo regenerated from the
counter-based source: weak scaling, no data-path collective.

Prints ONE JSON line (rank 0) with the roofline of the FIR kernel (HIP events around each
launch on the partition stream, algorithmic 16 B/sample) and the CPU baseline (the
scheduler_mt CPU path restated, timed on this host, rank 0 at N=1).

    python bench.py [--gpus N --steps K --warmup W] [--log2n 28] [--algo auto|mfma|direct]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_SAMPLE = 16  # algorithmic: read x (8 B) + write y (8 B) per output sample
FLOP_PER_SAMPLE = 508  # 127 taps x 2 (re, im) x FMA
METRIC = "MSamples/s through 127-tap fir_filter_ccf flowgraph; % HBM roofline at 1/8 GPU"


def firwin127():
    import scipy.signal as ss

    return ss.firwin(127, 0.2).astype(np.float32)  # C3 taps (tests/golden/fir127.npz)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(kernel, samples_per_launch):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_fir.json, produced
    by tools/pmc_summary.py from separate rocprofv3 --pmc passes, gfx950 FETCH_SIZE x2
    correction applied there), scaled to this launch size. kernel: the template name the
    plan reports (nsh_fir_plan_kernel), e.g. "k_fir_mfma9<5>"."""
    p = os.path.join(ROOT, "profiles", "pmc_fir.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return float(d[kernel]["hbm_bytes_per_sample"]) * samples_per_launch
    except (OSError, KeyError, ValueError, TypeError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--algo", default="auto", choices=["auto", "mfma", "mfma_x3", "mfma16", "direct"])
    ap.add_argument("--out-buf-mib", type=int, default=2048, help="FIR output hip_buffer (default: one launch per 2^28-sample step)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-log2n", type=int, default=28, help="CPU baseline sample (default: the full stream)")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    # one process per GPU; more ranks than GPUs (a rehearsal on a 1-GPU box) share devices
    device = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(device)
    dist = None
    backend = os.environ.get("NSH_BENCH_BACKEND", "nccl")  # nccl = RCCL; gloo only for rehearsals
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend=backend)

    from newsched_amd import nsh, nsr
    from oracle import oracle as orc  # checker only: tail parity + CPU-baseline inputs

    algo = {"auto": nsh.FIR_AUTO, "mfma": nsh.FIR_MFMA, "mfma16": nsh.FIR_MFMA16, "mfma_x3": nsh.FIR_MFMA_BF16X3,
            "direct": nsh.FIR_DIRECT}[a.algo]
    n = 1 << a.log2n
    taps = firwin127()
    first = rank * n  # this rank's time shard
    fb = nsr.FirBench(taps, n, device=device, algo=algo, first_index=first, out_buf_bytes=a.out_buf_mib << 20)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        fb.run()
    barrier()
    kms = 0.0
    samples = 0
    launches0 = fb.stats()["launches"]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        fb.run()
        st = fb.stats()  # HIP-event kernel time of this run (events re-armed at each start)
        kms += st["kernel_ms"]
        samples += st["samples"]
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = fb.stats()
    algo_used = {1: "direct", 2: "mfma", 3: "mfma16", 4: "mfma_x3"}.get(st["algo"], str(st["algo"]))
    kernel = st["kernel"]
    timed_launches = st["launches"] - launches0
    launches_per_run = timed_launches / a.steps
    per_launch_samples = samples / timed_launches
    avg_launch_ms = kms / timed_launches
    achieved = BYTES_PER_SAMPLE * per_launch_samples / (avg_launch_ms * 1e-3) / 1e9  # GB/s

    # parity on the measured path: the last 4096 outputs of the last run vs the oracle
    m = 4096
    y = fb.tail(m)
    lo = first + n - m - (taps.size - 1)
    xw = orc.synth(m + taps.size - 1, lo)
    y_ref = orc.fir_ccf(xw[taps.size - 1:], taps, hist=xw[: taps.size - 1])
    ok, err, scale = orc.tol_ok(y, y_ref)
    if dist is not None:  # every rank's shard tail must pass; report the worst error
        r = torch.tensor([0.0 if ok else 1.0, err], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(r, op=dist.ReduceOp.MAX)
        ok, err = r[0].item() == 0.0, float(r[1].item())

    value = world * n * a.steps / elapsed / 1e6  # MSamples/s, whole job
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: counter-based splitmix64 complex-float stream (BASELINE.md §2), HBM-resident before timing",
        "config": {
            "workload": "C3: 127-tap fir_filter_ccf (firwin(127,0.2) fp32 taps) over a 2^%d-sample complex-float stream per GPU, "
                        "nop_source->nop_head->[resident hip_buffer]->hip::fir_filter_ccf->[hip_buffer]->null_sink in scheduler_hip"
                        % a.log2n,
            "samples_per_gpu": n,
            "ntaps": int(taps.size),
            "fir_algo": algo_used,
            "fir_launches_per_step": launches_per_run,
            "samples_per_launch": int(per_launch_samples),
            "parallelism": "time-sharded replicas x%d (126-sample halo regenerated, no collective)" % world,
        },
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
        },
        "parity": {"check": "last 4096 outputs of the last step vs oracle (double accumulation), every rank",
                   "max_abs_err": err, "scale": scale, "ok": bool(ok)},
    }
    tr = load_pmc_traffic(kernel, per_launch_samples)
    if tr is not None:
        out["roofline"]["traffic"] = int(tr)

    if rank == 0 and world == 1 and not a.no_cpu:
        ncpu = 1 << a.cpu_log2n
        xs = orc.synth(1 << 20)  # vector_source data (repeated)
        secs = nsr.cpu_fir_run(taps, xs, ncpu, fixed_buf_size=32768)
        out["cpu_baseline"] = {
            "value": round(ncpu / secs / 1e6, 2),
            "unit": "MSamples/s",
            "cores": 4,
            "kind": "port",
            "sample": "2^%d samples through vector_source->head->fir_filter_ccf(127 taps, AVX-512 fp32)->null_sink, "
                      "scheduler_mt thread-per-block (4 threads; the FIR on one core), vmcircbuf 32768 B default buffers; "
                      "%.2f s on %s" % (a.cpu_log2n, secs, cpu_model()),
        }
    if dist is not None:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    fb.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
