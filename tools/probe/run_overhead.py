"""Host overhead of one C3 flowgraph run (bench.py's step): wall time of fg->run() at a tiny
stream (2^16 samples, a few-us kernel), median over 300 runs.
Usage: python tools/probe/run_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsr

torch.cuda.init()
h = ss.firwin(127, 0.2).astype(np.float32)
for timing in (False, True):
    fb = nsr.FirBench(h, 1 << 16, timing=timing, out_buf_bytes=1 << 20)
    for _ in range(20):
        fb.run()
    w = []
    for _ in range(300):
        t0 = time.perf_counter()
        fb.run()
        w.append(time.perf_counter() - t0)
    w = np.array(w) * 1e6
    print("timing=%d run wall us: median %.1f p10 %.1f p90 %.1f" % (timing, np.median(w), np.percentile(w, 10),
                                                                   np.percentile(w, 90)), flush=True)
    fb.close()
