"""Per-run host overhead of the C3 measurement flowgraph: wall time per fg run with HIP-event
timing on and stats() read every run (bench.py's loop), timing on without per-run stats, and
timing off; kernel time from the events. Usage: python tools/probe/run_overhead2.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch  # noqa: F401  (device init as in bench.py)

from newsched_amd import nsr

taps = ss.firwin(127, 0.2).astype(np.float32)
n = 1 << 28
res = {}
for name, timing, per_run_stats in (("timing+stats", True, True), ("timing", True, False), ("no_timing", False, False),
                                    ("timing+stats_2", True, True)):
    fb = nsr.FirBench(taps, n, out_buf_bytes=2048 << 20, timing=timing)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        fb.run()
    steps = 200
    k0 = fb.stats()["kernel_ms"]  # cumulative
    t0 = time.perf_counter()
    for _ in range(steps):
        fb.run()
        if per_run_stats:
            fb.stats()
    el = time.perf_counter() - t0
    kms = fb.stats()["kernel_ms"] - k0
    res[name] = {"us_per_run": round(el / steps * 1e6, 2), "kernel_us": round(kms / steps * 1e3, 2) if per_run_stats else None}
    fb.close() if hasattr(fb, "close") else None
print(json.dumps(res))
