"""Is the 'first build of each round runs slow' effect of the A/B probes a property of the round
position or of the output buffer? One library, one FIR plan (C3, 2^28), four output buffers; rounds
time the buffers in order 0..3, then in order 3..0. Prints median per (buffer, order)."""
import ctypes as C
import os
import sys

import numpy as np
import scipy.signal as ss
import torch

L = C.CDLL(os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "newsched_amd/lib/libnsh_hip.so"))
L.nsh_fir_plan_create.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
L.nsh_fir_ccf.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_int64, C.c_void_p]
L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << 28
rounds = int(os.environ.get("ROUNDS", "10"))
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
assert L.nsh_synth_cf32(x.data_ptr(), n, 0, 0x6E736368, C.c_void_p(s.cuda_stream)) == 0
h = ss.firwin(127, 0.2).astype(np.float32)
p = C.c_void_p()
assert L.nsh_fir_plan_create(0, h.ctypes.data, 127, 1, 2, C.byref(p)) == 0
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
ys = [torch.empty(n, dtype=torch.complex64, device="cuda") for _ in range(4)]
print("output buffers (hex addresses):", [hex(y.data_ptr()) for y in ys], flush=True)
run = lambda y: L.nsh_fir_ccf(p, x.data_ptr(), hin.data_ptr(), hout.data_ptr(), y.data_ptr(), n, C.c_void_p(s.cuda_stream))
for y in ys:
    run(y)
s.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for order in ([0, 1, 2, 3], [3, 2, 1, 0]):
    t = {i: [] for i in order}
    for _ in range(rounds):
        for i in order:
            st.record(s)
            for _ in range(5):
                run(ys[i])
            en.record(s)
            en.synchronize()
            t[i].append(st.elapsed_time(en) / 5 * 1e3)
    for pos, i in enumerate(order):
        v = sorted(t[i])
        print(f"order {order} position {pos} buffer {i}: median {v[len(v) // 2]:.1f} us min {v[0]:.1f}", flush=True)
