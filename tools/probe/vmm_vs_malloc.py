"""Does the allocation kind move the streaming rate? nsh_copy and the 127-tap FIR (default plan)
over 2^LOG2N complex samples, each on (a) torch's caching-allocator buffers (hipMalloc) and (b)
nsh_ring_alloc's VMM rings (hipMemCreate + two hipMemMap, as the flowgraph's hip_buffer edges),
interleaved in one process after a 2 s warm-up, HIP events over 5 launches per round.
Usage: python tools/probe/vmm_vs_malloc.py   env: LOG2N=28 ROUNDS=12"""
import ctypes as C
import os
import time

import numpy as np
import scipy.signal as ss
import torch

L = C.CDLL(os.path.abspath("newsched_amd/lib/libnsh_hip.so"))
L.nsh_ring_alloc.argtypes = [C.c_int, C.c_size_t, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_int)]
L.nsh_ring_free.argtypes = [C.c_void_p]
L.nsh_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
L.nsh_fir_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
L.nsh_fir_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]

n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "12"))
nb = 8 * n
s = torch.cuda.Stream()
sp = C.c_void_p(s.cuda_stream)

tx = torch.empty(n, dtype=torch.complex64, device="cuda")
ty = torch.empty(n, dtype=torch.complex64, device="cuda")
rings = []
for _ in range(2):
    b, a, dm = C.c_void_p(), C.c_size_t(), C.c_int()
    assert L.nsh_ring_alloc(0, nb, C.byref(b), C.byref(a), C.byref(dm)) == 0
    rings.append(b.value)
    print(f"ring {b.value:#x}: {a.value} B, double-mapped {dm.value}", flush=True)
rx, ry = rings
assert L.nsh_synth_cf32(tx.data_ptr(), n, 0, 0x6E736368, sp) == 0
assert L.nsh_copy(tx.data_ptr(), rx, nb, sp) == 0
h = ss.firwin(127, 0.2).astype(np.float32)
plan = C.c_void_p()
assert L.nsh_fir_plan_create(0, h.ctypes.data, h.size, 1, 0, C.byref(plan)) == 0
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
s.synchronize()

legs = {
    "copy malloc": lambda: L.nsh_copy(tx.data_ptr(), ty.data_ptr(), nb, sp),
    "copy vmm": lambda: L.nsh_copy(rx, ry, nb, sp),
    "fir malloc": lambda: L.nsh_fir_ccf(plan, tx.data_ptr(), hin.data_ptr(), hout.data_ptr(), ty.data_ptr(), n, sp),
    "fir vmm": lambda: L.nsh_fir_ccf(plan, rx, hin.data_ptr(), hout.data_ptr(), ry, n, sp),
}
t0 = time.perf_counter()
while time.perf_counter() - t0 < 2.0:
    for f in legs.values():
        assert f() == 0
    s.synchronize()
t = {k: [] for k in legs}
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
order = list(legs)
for r in range(rounds):
    for k in (order if r % 2 == 0 else order[::-1]):
        st.record(s)
        for _ in range(5):
            legs[k]()
        en.record(s)
        en.synchronize()
        t[k].append(st.elapsed_time(en) / 5 * 1e3)
y_m = ty.clone()
legs["fir vmm"]()
s.synchronize()
y_v = torch.empty_like(ty)
assert L.nsh_copy(ry, y_v.data_ptr(), nb, sp) == 0
legs["fir malloc"]()
s.synchronize()
print("fir outputs identical:", bool(torch.equal(ty, y_v)), flush=True)
for k in legs:
    v = sorted(t[k])
    med = v[len(v) // 2]
    print(f"{k}: median {med:.1f} us min {v[0]:.1f} us -> {16 * n / med / 1e3:.0f} GB/s", flush=True)
for b in rings:
    L.nsh_ring_free(b)
