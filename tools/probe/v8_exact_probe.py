"""Diagnostic for k_fir_mfma8's exact path: per 2048-output chunk, NaN counts and error vs
the oracle for inputs with an inf, a NaN and a finite 2^60 spike."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh
from oracle import oracle as orc

h = ss.firwin(127, 0.2).astype(np.float32)
for name, pos, val, n in [("inf", 1000, complex(np.inf, 0.5), 50_000), ("nan", 5000, complex(np.nan, 0), 50_000),
                          ("spike", 1000, None, 50_000), ("inf-big", 1000, complex(np.inf, 0.5), 1 << 20)]:
    x = orc.synth(n, 9)
    if val is None:
        x[pos] *= np.float32(2.0 ** 60)
    else:
        x[pos] = np.complex64(val)
    p = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    dx = torch.from_numpy(x).cuda()
    hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
    hout = torch.zeros_like(hin)
    dy = torch.empty_like(dx)
    p(dx, hin, hout, dy, n)
    torch.cuda.synchronize()
    y = dy.cpu().numpy()
    ref = orc.fir_ccf(x, h)
    print(name, p.kernel, "nan(y)", int(np.isnan(y.real).sum()), "nan(ref)", int(np.isnan(ref.real).sum()))
    for c in range(min(4, n // 2048)):
        a, b = 2048 * c, 2048 * (c + 1)
        fin = np.isfinite(ref[a:b].real) & np.isfinite(y[a:b].real)
        err = np.abs(y[a:b][fin] - ref[a:b][fin])
        print("  chunk", c, "nan", int(np.isnan(y[a:b].real).sum()), "maxerr", float(err.max()) if err.size else None,
              "first-nan", (a + int(np.argmax(np.isnan(y[a:b].real)))) if np.isnan(y[a:b].real).any() else None)
