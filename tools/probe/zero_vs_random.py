"""Energy probe: the default FIR kernel on all-zero vs random input (same instructions, less
switching energy), interleaved, 2^28 samples; plus the copy kernel on both. If zeros run
markedly faster the kernel is held down by the chip's power management, not by issue or HBM."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh

n = 1 << int(os.environ.get("LOG2N", "28"))
h = ss.firwin(127, 0.2).astype(np.float32)
xr = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(xr, n, 0)
xz = torch.zeros_like(xr)
y = torch.empty_like(xr)
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
p = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {k: [] for k in ("fir_random", "fir_zero", "copy_random", "copy_zero")}
for _ in range(5):
    p(xr, hin, hout, y, n)
for rnd in range(int(os.environ.get("ROUNDS", "12"))):
    for k in res:
        x = xz if k.endswith("zero") else xr
        st.record()
        for _ in range(5):
            if k.startswith("fir"):
                p(x, hin, hout, y, n)
            else:
                nsh.copy(x, y, 8 * n)
        en.record()
        en.synchronize()
        res[k].append(st.elapsed_time(en) / 5 * 1e3)
for k, t in res.items():
    t = sorted(t)
    print(f"{k} ({p.kernel if k.startswith('fir') else 'k_copy_v4'}): median {t[len(t)//2]:.1f} us min {t[0]:.1f} us -> "
          f"{16 * n / t[len(t)//2] / 1e6:.0f} GB/s", flush=True)
