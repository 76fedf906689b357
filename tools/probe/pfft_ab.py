"""A/B N builds of libnsh_hip.so on C5's fused chain (nsh_fir_cascade_ccf, 4 x fir(firwin(127,
0.45), 2)) in one process: interleaved rounds, HIP events on one stream, >= 1 s warm-up; prints
each build's median launch time and whether its output equals the first build's.
Usage: python tools/probe/pfft_ab.py A.so B.so [...]   (env: LOG2N=28 ROUNDS=8)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import scipy.signal as ss
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
FP = C.POINTER(C.c_float)
for L in libs:
    L.nsh_fir_cascade_plan_create.argtypes = [C.c_int, C.POINTER(FP), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                              C.POINTER(C.c_void_p)]
    L.nsh_fir_cascade_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "8"))
h = ss.firwin(127, 0.45).astype(np.float32)
tp = (FP * 4)(*[h.ctypes.data_as(FP)] * 4)
nt = (C.c_int * 4)(*[127] * 4)
dc = (C.c_int * 4)(*[2] * 4)
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
s.synchronize()
n_out = n // 16
ys = [torch.zeros(n_out, dtype=torch.complex64, device="cuda") for _ in libs]
hs = [torch.zeros(1890, dtype=torch.complex64, device="cuda") for _ in libs]
plans = []
for L in libs:
    p = C.c_void_p()
    assert L.nsh_fir_cascade_plan_create(0, tp, nt, dc, 4, C.byref(p)) == 0
    plans.append(p)
run = [lambda L=L, p=p, y=y, hh=hh: L.nsh_fir_cascade_ccf(p, x.data_ptr(), None, hh.data_ptr(), y.data_ptr(), n_out,
                                                          C.c_void_p(s.cuda_stream)) for L, p, y, hh in zip(libs, plans, ys, hs)]
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.time()
while time.time() - t0 < 1.0:
    for r in run:
        assert r() == 0
s.synchronize()
t = [[] for _ in libs]
for _ in range(rounds):
    for i, r in enumerate(run):
        st.record(s)
        for _ in range(5):
            r()
        en.record(s)
        en.synchronize()
        t[i].append(st.elapsed_time(en) / 5 * 1e3)
for i, pth in enumerate(paths):
    same = bool(torch.equal(ys[i], ys[0]))
    rel = float((ys[i] - ys[0]).abs().max().item() / ys[0].abs().max().item())
    med = float(np.median(t[i]))
    print(json.dumps({"lib": pth, "median_us": round(med, 1), "min_us": round(min(t[i]), 1),
                      "GSps_input": round(n / med / 1e3, 1), "same_as_first": same, "max_rel_diff": rel}), flush=True)
