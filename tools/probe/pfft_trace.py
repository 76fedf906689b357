"""Phase timestamps of k_fir_pfft<16> (a -DNSH_PFFT_TRACE=1 build): workgroup 0's first 64 frames,
per wave: t0 loop top, t1 before B1, t2 after B1, t3 before B2, t4 after B2, t5 inverse done.
Prints the median per-phase cycles. Usage: python tools/probe/pfft_trace.py build/abl/pfft_trace.so"""
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
t = np.array(buf, dtype=np.int64).reshape(64, 16, 8)[4:60]  # steady frames
fr = t[1:, :, 0] - t[:-1, :, 0]            # frame period per wave
a = t[:, :, 1] - t[:, :, 0]                # phase A (window+FFT+MAC)
w1 = t[:, :, 2] - t[:, :, 1]               # wait at B1
b = t[:, :, 3] - t[:, :, 2]                # phase B
w2 = t[:, :, 4] - t[:, :, 3]               # wait at B2
ifw = np.array([t[i, (i + 4) % 4, 5] - t[i, (i + 4) % 4, 4] for i in range(t.shape[0])])  # inverse wave, after B2
res = {"frame_period": float(np.median(fr)), "A_median": float(np.median(a)), "A_max_per_frame": float(np.median(a.max(1))),
       "B1_wait_median": float(np.median(w1)), "B": float(np.median(b)), "B_max": float(np.median(b.max(1))),
       "B2_wait_median": float(np.median(w2)), "inverse": float(np.median(ifw)),
       "A_of_inverse_wave_next": float(np.median([t[i + 1, (i + 4) % 4, 1] - t[i, (i + 4) % 4, 4] for i in range(t.shape[0] - 1)]))}
print(json.dumps(res))
np.save(os.environ.get("TRACE_OUT", "trace.npy"), np.array(buf, dtype=np.int64).reshape(64, 16, 8))
