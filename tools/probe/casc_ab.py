"""Time the fused two-stage decimator (nsh_fir_cascade2_ccf) against the same pair as two
nsh_fir_ccf(decim 2) launches, and the C5 chain (4 x fir(127, 2)) as 2 fused launches vs 4,
on 2^LOG2N input samples resident in HBM (interleaved rounds, torch events on the current
stream, which is the stream both paths launch on)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal
import torch

from newsched_amd import nsh

n = 1 << int(os.environ.get("LOG2N", "28"))
h = np.asarray(scipy.signal.firwin(127, 0.45), np.float32)
p1, p2 = nsh.FirPlan(h, 2, nsh.FIR_MFMA), nsh.FirPlan(h, 2, nsh.FIR_MFMA)
assert p1.cascade2_supported(p2)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
y1 = torch.empty(n // 2, dtype=torch.complex64, device="cuda")
y2 = torch.empty(n // 4, dtype=torch.complex64, device="cuda")
y2f = torch.empty(n // 4, dtype=torch.complex64, device="cuda")
y3 = torch.empty(n // 8, dtype=torch.complex64, device="cuda")
y4 = torch.empty(n // 16, dtype=torch.complex64, device="cuda")
y4f = torch.empty(n // 16, dtype=torch.complex64, device="cuda")
hz = [torch.zeros(126, dtype=torch.complex64, device="cuda") for _ in range(8)]


def sep2():
    p1(x, hz[0], hz[1], y1, n // 2)
    p2(y1, hz[2], hz[3], y2, n // 4)


def fused2():
    p1.cascade2(p2, x, hz[0], hz[1], hz[2], hz[3], y2f, n // 4)


def sep4():
    sep2()
    p1(y2, hz[4], hz[5], y3, n // 8)
    p2(y3, hz[6], hz[7], y4, n // 16)


def fused4():
    fused2()
    p1.cascade2(p2, y2f, hz[4], hz[5], hz[6], hz[7], y4f, n // 16)


runs = {"sep2": sep2, "fused2": fused2, "sep4": sep4, "fused4": fused4}
for f in runs.values():
    for _ in range(10):
        f()
torch.cuda.synchronize()
d2 = (y2f - y2).abs().max().item() / y2.abs().max().item()
d4 = (y4f - y4).abs().max().item() / y4.abs().max().item()
print(f"fused vs separate max rel diff: 2-stage {d2:.2e}, 4-stage {d4:.2e}", flush=True)
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {k: [] for k in runs}
for _ in range(int(os.environ.get("ROUNDS", "10"))):
    for k, f in runs.items():
        st.record()
        for _ in range(5):
            f()
        en.record()
        en.synchronize()
        res[k].append(st.elapsed_time(en) / 5 * 1e3)
for k, t in res.items():
    t = sorted(t)
    med = t[len(t) // 2]
    print(f"{k}: median {med:.1f} us (min {t[0]:.1f}) -> {n / med / 1e3:.0f} GS/s input", flush=True)
