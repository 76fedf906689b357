"""Workgroup spans of k_fir_pfft<16> (a -DNSH_PFFT_TRACE=2 build): s_memtime at each workgroup's
start and at its last wave's exit, for one 2^28-input C5 launch after warm-up. Durations are
compared (not absolute times: the XCDs' clocks are not one counter). Prints the spread.
Usage: python tools/probe/pfft_wgspan.py build/abl/pfft_wg.so"""
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
res = []
for rep in range(5):
    for _ in range(200):
        assert L.nsh_fir_cascade_ccf(p, x.data_ptr(), None, hh.data_ptr(), y.data_ptr(), n // 16, None) == 0
    buf = (C.c_ulonglong * (64 * 16 * 8))()
    assert L.nsh_pfft_trace_copy(buf) == 0
    t = np.array(buf, dtype=np.int64)[:512].reshape(256, 2)
    d = (t[:, 1] - t[:, 0]).astype(np.float64)
    res.append({"min": float(d.min()), "median": float(np.median(d)), "max": float(d.max()),
                "max_over_median": float(d.max() / np.median(d)), "p90": float(np.percentile(d, 90)),
                "slowest_wgs": [int(i) for i in np.argsort(d)[-8:]]})
print(json.dumps(res))
