"""A/B/n: several builds of libnsh_hip.so timed in one process (interleaved rounds, HIP events on
one stream) on one FIR plan (127 taps, firwin(127, 0.2) or C5's firwin(127, 0.45) chain), over
2^LOG2N resident samples. Prints each build's median / min launch time and whether its output is
bit-identical to the first build's (else the max |difference| relative to max |y|).
Usage: python tools/probe/lib_abn.py A.so B.so [C.so ...]
  env: DECIM=1 ALGO=2 (nsh_fir_algo; 2 = MFMA, 5 = MFMA_F32) LOG2N=28 ROUNDS=12 KIND=fir|casc
       INPUT=synth|spikeK (every K-th 2048-sample chunk holds a 2^40 spike: the exact path)"""
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
    L.nsh_fir_cascade_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]
    L.nsh_fir_cascade_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
    L.nsh_fir_cascade_kernel.restype = C.c_char_p
    L.nsh_fir_cascade_kernel.argtypes = [C.c_void_p]
    L.nsh_fir_cascade_hist_len.argtypes = [C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "12"))
D = int(os.environ.get("DECIM", "1"))
algo = int(os.environ.get("ALGO", "2"))
kind = os.environ.get("KIND", "fir")
inp = os.environ.get("INPUT", "synth")
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
s.synchronize()
if inp.startswith("spike"):
    k = int(inp[5:])
    x.view(-1, 2048)[::k, 7] = 2.0 ** 40
plans, names, hlen = [], [], 126
if kind == "casc":
    h = ss.firwin(127, 0.45).astype(np.float32)
    taps = [h] * 4
    arr = (C.c_void_p * 4)(*[t.ctypes.data for t in taps])
    nt = (C.c_int * 4)(*[127] * 4)
    dc = (C.c_int * 4)(*[2] * 4)
    D = 16
    for L in libs:
        p = C.c_void_p()
        assert L.nsh_fir_cascade_plan_create(0, arr, nt, dc, 4, C.byref(p)) == 0
        plans.append(p)
        names.append(L.nsh_fir_cascade_kernel(p).decode())
    hlen = libs[0].nsh_fir_cascade_hist_len(plans[0])
else:
    h = ss.firwin(127, 0.2).astype(np.float32)
    for L in libs:
        p = C.c_void_p()
        assert L.nsh_fir_plan_create(0, h.ctypes.data, h.size, D, algo, C.byref(p)) == 0
        plans.append(p)
        names.append(L.nsh_fir_plan_kernel(p).decode())
n_out = n // D
hin = torch.zeros(hlen, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
ys = [torch.zeros(n_out, dtype=torch.complex64, device="cuda") for _ in libs]
fn = "nsh_fir_cascade_ccf" if kind == "casc" else "nsh_fir_ccf"
run = [lambda L=L, p=p, y=y: getattr(L, fn)(p, x.data_ptr(), hin.data_ptr(), hout.data_ptr(), y.data_ptr(), n_out,
                                             C.c_void_p(s.cuda_stream)) for L, p, y in zip(libs, plans, ys)]
for r in run:
    assert r() == 0
s.synchronize()
t = [[] for _ in libs]
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
# clocks and power settle: every build in turn for at least WARM_S seconds (default 2; with 3 rounds
# only, the first two builds of a round ran ~1.5 % slower than the last two, profiles/r04r_*)
import time

t_w = time.perf_counter()
while time.perf_counter() - t_w < float(os.environ.get("WARM_S", "2")):
    for r in run:
        r()
    s.synchronize()
for _ in range(rounds):
    for i, r in enumerate(run):
        st.record(s)
        for _ in range(5):
            r()
        en.record(s)
        en.synchronize()
        t[i].append(st.elapsed_time(en) / 5 * 1e3)
ymax = float(ys[0].abs().max())
bpi = 8.5 if kind == "casc" else 8 + 8 / D
for i in range(len(libs)):
    v = sorted(t[i])
    med = v[len(v) // 2]
    same = bool(torch.equal(ys[0], ys[i]))
    diff = "bit-identical" if same else "max|d|/max|y| %.2e" % (float((ys[0] - ys[i]).abs().max()) / ymax)
    print(f"{paths[i]} {names[i]}: median {med:.1f} us min {v[0]:.1f} us -> {n / med / 1e3:.0f} GS/s input, "
          f"{bpi * n / med / 1e3:.0f} GB/s = {bpi * n / med / 8e6 * 100:.2f} % of 8 TB/s; {diff}", flush=True)
