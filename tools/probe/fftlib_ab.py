"""A/B N builds of libnsh_hip.so on the 1024-point transforms in one process: the channelizer
(nsh_channelizer1024, BASELINE C4) and the forward fft1024, 2^LOG2N resident samples, interleaved
rounds of 10 launches, HIP events on one stream, >= 2 s warm-up. Prints each build's median / min
launch time, % of 8 TB/s at 16 B per sample, and its max error against numpy (double) on 64
frames relative to the largest output.
Usage: python tools/probe/fftlib_ab.py A.so B.so [...]   (env: LOG2N=28 ROUNDS=10 KIND=chan|fft)"""
import ctypes as C
import os
import statistics
import sys
import time

import numpy as np
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
for L in libs:
    L.nsh_channelizer1024.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    L.nsh_fft1024_c2c.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "10"))
kind = os.environ.get("KIND", "chan")
nf = n // 1024
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
wn = ((1.0 + 0.5 * np.cos(2 * np.pi * np.arange(1024) / 1024)) / 1024).astype(np.complex64)
w = torch.from_numpy(wn).cuda()
ys = [torch.empty_like(x) for _ in libs]


def run(i):
    if kind == "chan":
        return libs[i].nsh_channelizer1024(x.data_ptr(), ys[i].data_ptr(), w.data_ptr(), nf, C.c_void_p(s.cuda_stream))
    return libs[i].nsh_fft1024_c2c(x.data_ptr(), ys[i].data_ptr(), nf, 0, C.c_void_p(s.cuda_stream))


for i in range(len(libs)):
    assert run(i) == 0
s.synchronize()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for i in range(len(libs)):
        run(i)
    s.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = [[] for _ in libs]
for r in range(rounds):
    for i in (range(len(libs)) if r % 2 == 0 else reversed(range(len(libs)))):
        e0.record(s)
        for _ in range(10):
            run(i)
        e1.record(s)
        s.synchronize()
        ts[i].append(e0.elapsed_time(e1) / 10 * 1e3)
frames = [0, 1, 7, nf // 3, nf // 2 + 5, nf - 1] + list(range(100, 158))
xf = x.view(nf, 1024)[frames].cpu().numpy().astype(np.complex128)
ref = np.fft.fft(xf, axis=1)
if kind == "chan":
    ref = np.fft.ifft(ref * wn.astype(np.complex128), axis=1) * 1024
for i, p in enumerate(paths):
    med = statistics.median(ts[i])
    got = ys[i].view(nf, 1024)[frames].cpu().numpy()
    err = np.abs(got - ref).max() / np.abs(ref).max()
    d = (ys[i] - ys[0]).abs().max().item() / max(ys[0].abs().max().item(), 1e-30)
    print("%s %s: median %.1f us min %.1f us -> %.1f %% of 8 TB/s; err vs numpy %.2e; vs first build %.2e"
          % (p, kind, med, min(ts[i]), 16 * n / (med * 1e-6) / 8e12 * 100, err, d), flush=True)
