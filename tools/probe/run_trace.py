"""Where a C3 flowgraph run's host overhead goes: steady-clock stamps at fixed points of each run
from a -DNSR_RUN_TRACE=1 build of libnewsched.so (NSR_LIB=that .so): run() entry (0), after
start() (1), the partition thread's NOTIFY (2), blocks started (3), FIR work() before / after its
launch (4 / 5), flush begin / end (6 / 7), FLUSHED at the monitor (8), run() return (9). Median
phase durations over 200 runs at 2^16 and 2^28 samples; `py` = previous return -> next entry.
Usage: NSR_LIB=build/abl/rt/libnewsched_rt.so python tools/probe/run_trace.py"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch  # noqa: F401

from newsched_amd import nsr

L = nsr.lib()
L.nsr_run_trace.argtypes = [C.POINTER(C.c_int64)]
h = ss.firwin(127, 0.2).astype(np.float32)
names = ["start", "wake", "blk_start", "to_launch", "launch", "to_flush", "flush", "to_flushed", "to_return"]
for log2n in (16, 28):
    fb = nsr.FirBench(h, 1 << log2n, out_buf_bytes=(2048 << 20) if log2n == 28 else (8 << 20))
    for _ in range(50):
        fb.run()
    rows, prev_end = [], None
    buf = (C.c_int64 * 16)()
    for _ in range(200):
        fb.run()
        L.nsr_run_trace(buf)
        t = np.array(buf[:10], dtype=np.int64)
        d = list(np.diff(t) / 1e3)
        d.append((t[0] - prev_end) / 1e3 if prev_end is not None else np.nan)
        prev_end = t[9]
        rows.append(d)
    a = np.array(rows)
    med = {n: round(float(np.nanmedian(a[:, i])), 1) for i, n in enumerate(names + ["py"])}
    med["total_run"] = round(float(np.median(a[:, :9].sum(axis=1))), 1)
    print(json.dumps({"log2n": log2n, "median_us": med}), flush=True)
    fb.close()
