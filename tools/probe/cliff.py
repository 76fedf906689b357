"""Exact-path cost of the default FIR kernels: in k_fir_mfma12 (decim 1) a 2048-sample chunk whose
range exceeds the split's (a 2^40 spike among ~1 values) is filtered by the exact-fp32 matrix tile
and one holding a non-finite sample by the fp32 direct form, inside the same launch (k_fir_mfma11,
decim 2 / 4: the fp32 direct form for both). Times 2^28-sample launches with every
k-th chunk poisoned (k = inf, 256, 64, 16, 4, 1), HIP events, >= 1 s warm-up per case, and
checks a window around a poisoned chunk against the oracle.
Usage: python tools/probe/cliff.py [--log2n 28] [--decim 1|2|4]"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh
from oracle import oracle as orc

ap = argparse.ArgumentParser()
ap.add_argument("--log2n", type=int, default=28)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--decim", type=int, default=1)
ap.add_argument("--ks", default="0,256,64,16,4,1", help="every k-th chunk poisoned (0: none)")
ap.add_argument("--kinds", default="nan,spike")
a = ap.parse_args()
n = 1 << a.log2n
h = ss.firwin(127, 0.2).astype(np.float32)
D = a.decim
plan = nsh.FirPlan(h, D)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
y = torch.empty(n // D, dtype=torch.complex64, device="cuda")
s = torch.cuda.Stream()
res = {"kernel": plan.kernel, "decim": D, "log2n": a.log2n, "cases": []}
for kind in a.kinds.split(","):
    for k in [int(v) for v in a.ks.split(",")]:
        nsh.synth(x, n, 0)
        if k:
            v = float("nan") if kind == "nan" else 2.0 ** 40
            x.view(n // 2048, 2048)[::k, 7] = complex(v, 0.5)
        torch.cuda.synchronize()
        t0 = time.time()
        hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
        hout = torch.zeros_like(hin)
        while time.time() - t0 < 1.0:
            plan(x, hin, hout, y, n // D, stream=s)
            s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(a.reps):
                plan(x, hin, hout, y, n // D, stream=s)
            e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / a.reps * 1e3
        # parity on chunks 0..2 (chunk 0 poisoned when k > 0) against the oracle
        xs = x[: 3 * 2048].cpu().numpy()
        yr = orc.fir_ccf(xs, h, D)
        yy = y[: 3 * 2048 // D].cpu().numpy()
        fin = np.isfinite(yr.real) & np.isfinite(yr.imag)
        same_nf = bool(np.array_equal(fin, np.isfinite(yy.real) & np.isfinite(yy.imag)))
        ok, err, _ = orc.tol_ok(yy[fin], yr[fin])
        res["cases"].append({"kind": kind if k else "none", "every_kth_chunk": k, "exact_fraction": (1.0 / k) if k else 0.0,
                             "us": round(us, 1), "GSps_in": round(n / us / 1e3, 1),
                             "parity_ok": bool(ok and same_nf)})
        print(json.dumps(res["cases"][-1]), flush=True)
print(json.dumps(res))
