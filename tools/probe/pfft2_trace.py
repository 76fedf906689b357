"""Phase timestamps of k_fir_pfft2<16> (a -DNSH_PFFT_TRACE=1 build): workgroup 0's first 64 frames,
per wave: t0 frame top, t1 exchange-1 stores issued (before B1), t2 after B1, t3 after the inverse
(waves 0..3 in their turn), t4 own products stored, t5 phase sum done (waves 8..15), t6 after B2.
Prints per-wave medians (cycles of s_memtime) and saves the raw array.
Usage: python tools/probe/pfft2_trace.py build/abl/pfft_trace.so   (env TRACE_OUT=trace.npy)"""
import ctypes as C
import json
import os
import sys

import numpy as np
import scipy.signal as ss
import torch

L = C.CDLL(os.path.abspath(sys.argv[1]), mode=C.RTLD_LOCAL)
FP = C.POINTER(C.c_float)
L.nsh_fir_cascade_plan_create.argtypes = [C.c_int, C.POINTER(FP), C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int,
                                          C.POINTER(C.c_void_p)]
L.nsh_fir_cascade_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << 28
h = ss.firwin(127, 0.45).astype(np.float32)
tp = (FP * 4)(*[h.ctypes.data_as(FP)] * 4)
nt = (C.c_int * 4)(*[127] * 4)
dc = (C.c_int * 4)(*[2] * 4)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert L.nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, None) == 0
y = torch.empty(n // 16, dtype=torch.complex64, device="cuda")
hh = torch.empty(1890, dtype=torch.complex64, device="cuda")
p = C.c_void_p()
assert L.nsh_fir_cascade_plan_create(0, tp, nt, dc, 4, C.byref(p)) == 0
for _ in range(200):
    assert L.nsh_fir_cascade_ccf(p, x.data_ptr(), None, hh.data_ptr(), y.data_ptr(), n // 16, None) == 0
buf = (C.c_ulonglong * (64 * 16 * 8))()
assert L.nsh_pfft_trace_copy(buf) == 0
raw = np.array(buf, dtype=np.int64).reshape(64, 16, 8)
np.save(os.environ.get("TRACE_OUT", "trace.npy"), raw)
t = raw[4:60].astype(np.float64)
t -= t[:, :, :1].min(axis=1, keepdims=True)  # relative to the frame's first wave at its top
res = {"frame_period": float(np.median(np.diff(raw[4:60, 0, 0])))}
names = ["top", "x1_stored", "after_B1", "after_inverse", "products", "sum_done", "after_B2"]
for k, nm in enumerate(names):
    res[nm] = [int(v) for v in np.median(t[:, :, k], axis=0)]
print(json.dumps(res))
