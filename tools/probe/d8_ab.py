"""Single decimate-by-8 FIR (127 and 511 taps): the fp32 direct form k_fir_direct<8,2> (AUTO for
decim 8) vs the polyphase-FFT kernel (nsh_fir_cascade_ccf with one stage, k_fir_pfft<8,1>),
2^28 inputs, one process, HIP events, oracle parity on a tail window."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh
from oracle import oracle as orc

n = 1 << 28
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
s = torch.cuda.Stream()


def timed(fn, reps=10):
    t0 = time.time()
    while time.time() - t0 < 0.5:
        fn()
        s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for L in (127, 511):
    h = ss.firwin(L, 0.1).astype(np.float32)
    y1 = torch.empty(n // 8, dtype=torch.complex64, device="cuda")
    y2 = torch.empty_like(y1)
    hd = torch.zeros(L - 1, dtype=torch.complex64, device="cuda")
    hd2 = torch.zeros_like(hd)
    pd = nsh.FirPlan(h, 8)
    pc = nsh.FirCascadePlan([(h, 8)])
    hc = torch.zeros(pc.hist_len, dtype=torch.complex64, device="cuda")
    td = timed(lambda: pd(x, hd, hd2, y1, n // 8, stream=s))
    tc = timed(lambda: pc(x, None, hc, y2, n // 8, stream=s))
    m = 4096
    xs = orc.synth(8 * m + 8 * L, n - 8 * m - 8 * L)
    yr = orc.fir_ccf(xs, h, 8)[-m:]
    ok1 = orc.tol_ok(y1[-m:].cpu().numpy(), yr)[0]
    ok2 = orc.tol_ok(y2[-m:].cpu().numpy(), yr)[0]
    print(json.dumps({"ntaps": L, "direct_kernel": pd.kernel, "direct_us": round(td, 1), "direct_GSps_in": round(n / td / 1e3, 1),
                      "pfft_kernel": pc.kernel, "pfft_us": round(tc, 1), "pfft_GSps_in": round(n / tc / 1e3, 1),
                      "pfft_frac_9B": round(9 * n / tc / 1e3 / 8000, 4), "parity": [bool(ok1), bool(ok2)]}), flush=True)
