"""Does the distance between a stream's input and output addresses move its rate (channel
camping)? nsh_copy and the 127-tap FIR (default plan) over 2^LOG2N complex samples from one input
buffer into ONE output allocation at several byte offsets -- same physical pages, only the
in/out address difference changes -- interleaved in one process after a 2 s warm-up, HIP events
over 5 launches per round. Usage: python tools/probe/offset_probe.py   env: LOG2N=28 ROUNDS=10"""
import ctypes as C
import os
import time

import numpy as np
import scipy.signal as ss
import torch

L = C.CDLL(os.path.abspath("newsched_amd/lib/libnsh_hip.so"))
L.nsh_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
L.nsh_fir_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
L.nsh_fir_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]

n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "10"))
nb = 8 * n
PAD = 8 << 20
offsets = [0, 4096, 3 * 4096, 64 * 1024 + 4096, 1 << 20, (1 << 20) + 4096 * 5, 4 << 20]
s = torch.cuda.Stream()
sp = C.c_void_p(s.cuda_stream)
x = torch.empty(nb // 8, dtype=torch.complex64, device="cuda")
yb = torch.empty((nb + PAD) // 8, dtype=torch.complex64, device="cuda")
print(f"x {x.data_ptr():#x}  y {yb.data_ptr():#x}  (y - x) mod 2 MiB = {(yb.data_ptr() - x.data_ptr()) % (2 << 20)}", flush=True)
assert L.nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, sp) == 0
h = ss.firwin(127, 0.2).astype(np.float32)
plan = C.c_void_p()
assert L.nsh_fir_plan_create(0, h.ctypes.data, h.size, 1, 0, C.byref(plan)) == 0
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
s.synchronize()


def leg(kind, off):
    y = yb.data_ptr() + off
    if kind == "copy":
        return lambda: L.nsh_copy(x.data_ptr(), y, nb, sp)
    return lambda: L.nsh_fir_ccf(plan, x.data_ptr(), hin.data_ptr(), hout.data_ptr(), y, n, sp)


for kind in ("copy", "fir"):
    legs = [(off, leg(kind, off)) for off in offsets]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for _, f in legs:
            assert f() == 0
        s.synchronize()
    t = {off: [] for off in offsets}
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for off, f in (legs if r % 2 == 0 else legs[::-1]):
            st.record(s)
            for _ in range(5):
                f()
            en.record(s)
            en.synchronize()
            t[off].append(st.elapsed_time(en) / 5 * 1e3)
    for off in offsets:
        v = sorted(t[off])
        med = v[len(v) // 2]
        print(f"{kind} out offset {off:>8} B: median {med:.1f} us min {v[0]:.1f} us -> {16 * n / med / 1e3:.0f} GB/s", flush=True)
