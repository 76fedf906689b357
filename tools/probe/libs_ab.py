"""A/B N builds of libnsh_hip.so in one process (interleaved rounds, HIP events on one stream):
the default decim-1 FIR plan (127 taps, firwin(127, 0.2)) over 2^LOG2N samples; reports each
build's median launch time and whether its output equals the first build's.
Usage: python tools/probe/libs_ab.py A.so B.so [C.so ...]   (env: LOG2N=28 ROUNDS=10 DECIM=1)"""
import ctypes as C
import os
import sys

import numpy as np
import scipy.signal as ss
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
for L in libs:
    L.nsh_fir_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.nsh_fir_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
    L.nsh_fir_plan_kernel.restype = C.c_char_p
    L.nsh_fir_plan_kernel.argtypes = [C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
D = int(os.environ.get("DECIM", "1"))
rounds = int(os.environ.get("ROUNDS", "10"))
h = ss.firwin(127, 0.2).astype(np.float32)
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
s.synchronize()
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
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
for i, L in enumerate(libs):
    v = sorted(t[i])
    med = v[len(v) // 2]
    gbs = (8 * n + 8 * n_out) / med / 1e3
    same = bool(torch.equal(ys[0], ys[i]))
    print(f"{paths[i]} {L.nsh_fir_plan_kernel(plans[i]).decode()}: median {med:.1f} us min {v[0]:.1f} us "
          f"{gbs:.0f} GB/s ({gbs / 80:.1f}%)  same-as-first={same}", flush=True)
