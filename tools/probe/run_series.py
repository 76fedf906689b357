"""Per-run wall and kernel time of the C3 flowgraph for the first runs after creation (what
bench.py's warmup has to cover). Usage: python tools/probe/run_series.py [runs]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsr

torch.cuda.init()
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
h = ss.firwin(127, 0.2).astype(np.float32)
fb = nsr.FirBench(h, 1 << 28, out_buf_bytes=2048 << 20)
prev = fb.stats()["kernel_ms"]  # cumulative
for i in range(runs):
    t0 = time.perf_counter()
    fb.run()
    w = (time.perf_counter() - t0) * 1e6
    st = fb.stats()
    print("run %2d wall_us %7.1f kernel_us %7.1f launches %d" % (i, w, (st["kernel_ms"] - prev) * 1e3, st["launches"]), flush=True)
    prev = st["kernel_ms"]
