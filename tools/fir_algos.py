"""Time FIR algorithms (nsh_fir_ccf plans) in one process, interleaved rounds, HIP events:
127 taps firwin(127, 0.2) over 2^LOG2N samples. ALGOS = comma list of nsh algo names
(mfma, mfma_f32, direct, ...). Prints median/min launch time and % of the 8 TB/s roofline
(16 B per output sample), plus each algorithm's max error vs the first on a window."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh

n = 1 << int(os.environ.get("LOG2N", "28"))
names = os.environ.get("ALGOS", "mfma,mfma_f32").split(",")
ids = {"direct": nsh.FIR_DIRECT, "mfma": nsh.FIR_MFMA, "mfma16": nsh.FIR_MFMA16, "mfma_x3": nsh.FIR_MFMA_BF16X3,
       "mfma_f32": nsh.FIR_MFMA_F32}
h = ss.firwin(127, 0.2).astype(np.float32)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
plans = {a: nsh.FirPlan(h, 1, ids[a]) for a in names}
ys = {a: torch.empty_like(x) for a in names}
for a, p in plans.items():
    p(x, hin, hout, ys[a], n)
torch.cuda.synchronize()
y0 = ys[names[0]][:1 << 20]
for a in names:
    d = (ys[a][:1 << 20] - y0).abs().max().item()
    print(f"{a} ({plans[a].kernel}): max|y - y_{names[0]}| over 2^20 = {d:.3g}", flush=True)
res = {a: [] for a in names}
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(int(os.environ.get("ROUNDS", "10"))):
    for a, p in plans.items():
        st.record()
        for _ in range(5):
            p(x, hin, hout, ys[a], n)
        en.record()
        en.synchronize()
        res[a].append(st.elapsed_time(en) / 5 * 1e3)
for a in names:
    v = sorted(res[a])
    med = v[len(v) // 2]
    print(f"{a} ({plans[a].kernel}): median {med:.1f} us min {v[0]:.1f} us -> {n / med / 1e3:.0f} GS/s, "
          f"{16 * n / med / 1e3:.0f} GB/s ({16 * n / med / 1e3 / 80:.1f}% of 8 TB/s)", flush=True)
