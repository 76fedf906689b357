"""A/B/n of libnsh_hip.so builds on the fused channelizer (nsh_channelizer1024, BASELINE C4) and
fft1024 in one process: interleaved rounds, HIP events on one stream, 2^LOG2N samples; each build's
median / min launch time and whether its output equals the first build's.
Usage: python tools/probe/chan_libs_ab.py A.so B.so [C.so ...]   (env: LOG2N=28 ROUNDS=12 KIND=chan|fft)"""
import ctypes as C
import os
import sys

import numpy as np
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
for L in libs:
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
    L.nsh_fft1024_c2c.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    L.nsh_channelizer1024.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "12"))
kind = os.environ.get("KIND", "chan")
nf = n // 1024
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
b = np.arange(1024)
w = torch.from_numpy(((1 + 0.5 * np.cos(2 * np.pi * b / 1024)) / 1024).astype(np.complex64)).cuda()
ys = [torch.empty_like(x) for _ in libs]
if kind == "chan":
    run = [lambda L=L, y=y: L.nsh_channelizer1024(x.data_ptr(), y.data_ptr(), w.data_ptr(), nf, C.c_void_p(s.cuda_stream))
           for L, y in zip(libs, ys)]
else:
    run = [lambda L=L, y=y: L.nsh_fft1024_c2c(x.data_ptr(), y.data_ptr(), nf, 0, C.c_void_p(s.cuda_stream))
           for L, y in zip(libs, ys)]
s.synchronize()
for r in run:
    assert r() == 0
s.synchronize()
import time

t0 = time.time()
while time.time() - t0 < float(os.environ.get("WARM_S", "2")):  # clocks settle (2 s: see lib_abn.py)
    for r in run:
        r()
    s.synchronize()
t = [[] for _ in libs]
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(rounds):
    for i, r in enumerate(run):
        st.record(s)
        for _ in range(5):
            r()
        en.record(s)
        en.synchronize()
        t[i].append(st.elapsed_time(en) / 5 * 1e3)
for i in range(len(libs)):
    v = sorted(t[i])
    med = v[len(v) // 2]
    same = bool(torch.equal(ys[0], ys[i]))
    print(f"{kind} {paths[i]}: median {med:.1f} us min {v[0]:.1f} us -> {n / med / 1e3:.0f} GS/s, "
          f"{16 * n / med / 8e6 * 100:.2f} % of 8 TB/s; {'bit-identical' if same else 'DIFFERENT'}", flush=True)
