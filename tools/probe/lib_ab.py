"""A/B two builds of libnsh_hip.so in one process (interleaved rounds, HIP events on one
stream): FIR plans for decimation factors DECIMS (127 taps), then fft1024 and the fused
channelizer, over 2^LOG2N samples. Outputs of the two builds must be bit-identical.
Usage: python tools/probe/lib_ab.py A.so B.so   (env: DECIMS=1,2,4 LOG2N=28 ROUNDS=10)"""
import ctypes as C
import os
import sys

import numpy as np
import scipy.signal as ss
import torch

libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in sys.argv[1:3]]
for L in libs:
    L.nsh_fir_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.nsh_fir_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
    L.nsh_fir_plan_kernel.restype = C.c_char_p
    L.nsh_fir_plan_kernel.argtypes = [C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
    L.nsh_fft1024_c2c.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p]
    L.nsh_channelizer1024.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "10"))
h = ss.firwin(127, 0.2).astype(np.float32)
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
s.synchronize()
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
for D in [int(d) for d in os.environ.get("DECIMS", "1,2,4").split(",") if d]:
    n_out = n // D
    ys = [torch.zeros(n_out, dtype=torch.complex64, device="cuda") for _ in libs]
    plans = []
    for L in libs:
        p = C.c_void_p()
        assert L.nsh_fir_plan_create(0, h.ctypes.data, h.size, D, 2, C.byref(p)) == 0
        plans.append(p)
    run = [lambda L=L, p=p, y=y: L.nsh_fir_ccf(p, x.data_ptr(), hin.data_ptr(), hout.data_ptr(), y.data_ptr(), n_out,
                                               C.c_void_p(s.cuda_stream)) for L, p, y in zip(libs, plans, ys)]
    for r in run:
        assert r() == 0
    s.synchronize()
    same = bool(torch.equal(ys[0], ys[1]))
    t = [[], []]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for i, r in enumerate(run):
            st.record(s)
            for _ in range(5):
                r()
            en.record(s)
            en.synchronize()
            t[i].append(st.elapsed_time(en) / 5 * 1e3)
    names = [L.nsh_fir_plan_kernel(p).decode() for L, p in zip(libs, plans)]
    for i in range(2):
        v = sorted(t[i])
        med = v[len(v) // 2]
        gbs = (8 * n + 8 * n_out) / med / 1e3
        print(f"D={D} {sys.argv[1 + i]} {names[i]}: median {med:.1f} us min {v[0]:.1f} us -> {n / med / 1e3:.0f} GS/s input, "
              f"{gbs:.0f} GB/s ({gbs / 80:.1f}% of 8 TB/s)  bit-identical={same}", flush=True)


def ab(name, run, ys, nbytes):
    for r in run:
        assert r() == 0
    s.synchronize()
    same = bool(torch.equal(ys[0], ys[1]))
    t = [[], []]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for i, r in enumerate(run):
            st.record(s)
            for _ in range(5):
                r()
            en.record(s)
            en.synchronize()
            t[i].append(st.elapsed_time(en) / 5 * 1e3)
    for i in range(2):
        v = sorted(t[i])
        med = v[len(v) // 2]
        print(f"{name} {sys.argv[1 + i]}: median {med:.1f} us min {v[0]:.1f} us -> {n / med / 1e3:.0f} GS/s, "
              f"{nbytes / med / 1e3:.0f} GB/s ({nbytes / med / 1e3 / 80:.1f}% of 8 TB/s)  bit-identical={same}", flush=True)


nf = n // 1024
w = torch.from_numpy(((1 + 0.5 * np.cos(2 * np.pi * np.arange(1024) / 1024)) / 1024).astype(np.complex64)).cuda()
ys = [torch.zeros(n, dtype=torch.complex64, device="cuda") for _ in libs]
ab("fft1024", [lambda L=L, y=y: L.nsh_fft1024_c2c(x.data_ptr(), y.data_ptr(), nf, 0, C.c_void_p(s.cuda_stream))
               for L, y in zip(libs, ys)], ys, 16 * n)
ab("chan1024", [lambda L=L, y=y: L.nsh_channelizer1024(x.data_ptr(), y.data_ptr(), w.data_ptr(), nf, C.c_void_p(s.cuda_stream))
                for L, y in zip(libs, ys)], ys, 16 * n)
