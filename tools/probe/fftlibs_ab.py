"""A/B N builds of libnsh_hip.so on fft1024 (forward) and the channelizer in one process
(interleaved rounds, HIP events, >= 1 s warm-up), 2^LOG2N samples; max relative difference of
each build's outputs to the first build's.
Usage: python tools/probe/fftlibs_ab.py A.so B.so [...]   (env: LOG2N=28 ROUNDS=6)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
for L in libs:
    L.nsh_fft1024_c2c.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    L.nsh_channelizer1024.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "6"))
s = torch.cuda.Stream()
sp = C.c_void_p(s.cuda_stream)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, sp) == 0
w = torch.from_numpy(np.exp(-0.5 * ((np.arange(1024) - 512) / 100.0) ** 2).astype(np.complex64)).cuda()
ys = [torch.empty_like(x) for _ in libs]
ops = {
    "fft1024": lambda L, y: L.nsh_fft1024_c2c(x.data_ptr(), y.data_ptr(), n // 1024, 0, sp),
    "chan1024": lambda L, y: L.nsh_channelizer1024(x.data_ptr(), y.data_ptr(), w.data_ptr(), n // 1024, sp),
}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, op in ops.items():
    t0 = time.time()
    while time.time() - t0 < 1.0:
        for L, y in zip(libs, ys):
            assert op(L, y) == 0
        s.synchronize()
    t = [[] for _ in libs]
    for _ in range(rounds):
        for i, (L, y) in enumerate(zip(libs, ys)):
            with torch.cuda.stream(s):
                e0.record(s)
                for _ in range(5):
                    op(L, y)
                e1.record(s)
            e1.synchronize()
            t[i].append(e0.elapsed_time(e1) / 5 * 1e3)
    for i, p in enumerate(paths):
        med = float(np.median(t[i]))
        rel = float((ys[i] - ys[0]).abs().max().item() / ys[0].abs().max().item())
        print(json.dumps({"op": name, "lib": p, "median_us": round(med, 1), "frac": round(16 * n / med / 1e3 / 8000, 4),
                          "max_rel_diff_vs_first": rel}), flush=True)
