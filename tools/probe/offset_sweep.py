"""Copy rate against the distance between input and output inside ONE allocation (tools/probe/
placement.py found whole pairs of separately allocated buffers that copy ~6 % faster than others,
the same pairs under hipMalloc and HIP-VMM: a property of where they landed, not of the virtual
addresses). One 2 * 2^LOG2N-sample + slack allocation; the input at its start, the output at
2^LOG2N samples + d bytes for each d; nsh_copy (k_copy_v4) timed with HIP events, interleaved over
ROUNDS rounds. KERNEL=fir / d2 / d4 times the 127-tap FIR (nsh_fir_ccf, AUTO: k_fir_mfma12 / k_fir_mfma13) and
KERNEL=map C2's fused multiply chain (k_map_c_v4) instead; the rate is quoted at 16 B / sample
(the decimators move 8 + 8/D).
Usage: python tools/probe/offset_sweep.py   (env: LOG2N=28 ROUNDS=4 KERNEL=copy|fir DS=d1,d2,...)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from newsched_amd import nsh  # noqa: E402

n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "4"))
ds = [int(v) for v in os.environ.get("DS", "0,256,4096,16384,65536,262144,1048576,2097152,4194304,8388608,"
                                                 "33554432,134217728").split(",")]
L = nsh.lib()
slack = max(ds) + (1 << 20)
buf = torch.empty(2 * n * 8 + slack, dtype=torch.uint8, device="cuda")
base = buf.data_ptr()
s = torch.cuda.Stream()
nsh.check(L.nsh_synth_cf32(C.c_void_p(base), n, 0, 7, C.c_void_p(s.cuda_stream)), "synth")
s.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
kernel = os.environ.get("KERNEL", "copy")
decim = {"fir": 1, "d2": 2, "d4": 4}.get(kernel, 0)
if decim:
    import scipy.signal as ss

    plan = nsh.FirPlan(ss.firwin(127, 0.2 if decim == 1 else 0.45).astype(np.float32), decim, nsh.FIR_AUTO)
    hout = torch.empty(126, dtype=torch.complex64, device="cuda")
elif kernel == "map":
    ks = [0.5 + 0.5j, 1j, 0.8 - 0.6j, 1.0]


def copy(d):
    if decim:
        plan(base, 0, hout, base + 8 * n + d, n // decim, stream=s)
        return
    if kernel == "map":
        nsh.mul_const_chain_cc(base, base + 8 * n + d, n, ks, stream=s)
        return
    nsh.check(L.nsh_copy(C.c_void_p(base), C.c_void_p(base + 8 * n + d), 8 * n, C.c_void_p(s.cuda_stream)), "copy")


t0 = time.time()
while time.time() - t0 < 1.5:
    copy(0)
    s.synchronize()
res = {d: [] for d in ds}
for r in range(rounds):
    for d in ds:
        e0.record(s)
        for _ in range(5):
            copy(d)
        e1.record(s)
        e1.synchronize()
        res[d].append(e0.elapsed_time(e1) / 5 * 1e3)
print("# base", hex(base), flush=True)
for d in ds:
    m = float(np.median(res[d]))
    print(json.dumps({"d_bytes": d, "median_us": round(m, 1), "pct": round(16.0 * n / (m * 1e-6) / 8e12 * 100, 2),
                      "runs": [round(x, 1) for x in res[d]]}), flush=True)
