"""A/B two builds of libnsh_hip.so on the fused channelizer (nsh_channelizer1024, C4's W) over
2^LOG2N samples: median launch time each, max |difference| relative to max |y| between them,
and each against numpy (float64) on 8 frames.
Usage: python tools/probe/chan_v2_ab.py A.so B.so   (env: LOG2N=28 ROUNDS=8)"""
import ctypes as C
import os
import sys

import numpy as np
import torch

libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in sys.argv[1:3]]
for L in libs:
    L.nsh_channelizer1024.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "8"))
nf = n // 1024
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
b = np.arange(1024)
w = torch.from_numpy(((1 + 0.5 * np.cos(2 * np.pi * b / 1024)) / 1024).astype(np.complex64)).cuda()
ys = [torch.zeros(n, dtype=torch.complex64, device="cuda") for _ in libs]
run = [lambda L=L, y=y: L.nsh_channelizer1024(x.data_ptr(), y.data_ptr(), w.data_ptr(), nf, C.c_void_p(s.cuda_stream))
       for L, y in zip(libs, ys)]
for _ in range(20):
    for r in run:
        assert r() == 0
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t = [[] for _ in libs]
for _ in range(rounds):
    for i, r in enumerate(run):
        st.record(s)
        for _ in range(5):
            r()
        en.record(s)
        en.synchronize()
        t[i].append(st.elapsed_time(en) / 5 * 1e3)
xs = x.view(nf, 1024)[[0, 1, nf // 2, nf - 1]].cpu().numpy().astype(np.complex128)
ref = np.fft.ifft(np.fft.fft(xs, axis=1) * w.cpu().numpy().astype(np.complex128), axis=1) * 1024
for i, p in enumerate(sys.argv[1:3]):
    med = float(np.median(t[i]))
    y = ys[i].view(nf, 1024)[[0, 1, nf // 2, nf - 1]].cpu().numpy()
    err = float(np.abs(y - ref).max() / np.abs(ref).max())
    print("%s: median %.1f us = %.1f%% of 8 TB/s, rel err vs numpy %.2e" % (os.path.basename(p), med,
          16 * n / med / 1e3 / 80, err), flush=True)
d = float((ys[0] - ys[1]).abs().max().item() / ys[0].abs().max().item())
print("max |A - B| / max |A| = %.2e" % d)
e = ((ys[0] - ys[1]).abs().view(nf, 1024).amax(dim=1) / ys[0].abs().max()).cpu().numpy()
bad = np.nonzero(e > 1e-5)[0]
print("frames with |A - B| > 1e-5 max|A|: %d of %d; first %s; last %s" % (bad.size, nf, bad[:8].tolist(), bad[-8:].tolist()))
if bad.size:
    fb = int(bad[0])
    yb = ys[1].view(nf, 1024)[fb].cpu().numpy()
    ya = ys[0].view(nf, 1024)[fb].cpu().numpy()
    col = np.nonzero(np.abs(yb - ya) > 1e-5 * np.abs(ya).max())[0]
    print("frame", fb, "bad samples", col.size, col[:16].tolist())
