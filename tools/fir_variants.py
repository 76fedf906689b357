"""A/B the MFMA FIR kernel variants in one process (interleaved rounds), 2^25-sample
launches (LOG2N): NSH_FIR_MFMA_VARIANT 0 = default (k_fir_mfma8 LEAN), 8 = k_fir_mfma8 per-sample tests, 6/7 = bf16x3 v2 depth 1/2, 20-22 = the
16-sample form. Checks each variant against the oracle on a window and against the first
variant over the whole output."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh
from oracle import oracle as orc

n = 1 << int(os.environ.get("LOG2N", "25"))
h = ss.firwin(127, 0.2).astype(np.float32)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
y = torch.empty_like(x)
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
plans = {}
# VARIANTS entries: "v" or "v:g" (g = NSH_FIR_WG_PER_CU for that plan)
for spec in os.environ.get("VARIANTS", "6,7,21").split(","):
    v, _, g = spec.partition(":")
    os.environ["NSH_FIR_MFMA_VARIANT"] = v
    if g:
        os.environ["NSH_FIR_WG_PER_CU"] = g
    plans[spec] = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    os.environ.pop("NSH_FIR_WG_PER_CU", None)
os.environ.pop("NSH_FIR_MFMA_VARIANT")
xs = x[:20000].cpu().numpy()
ref = orc.fir_ccf(xs, h)
for v, p in plans.items():
    p(x, hin, hout, y, n)
    torch.cuda.synchronize()
    ok, err, sc = orc.tol_ok(y[:20000].cpu().numpy(), ref)
    print(f"variant {v}: parity ok={ok} err={err:.3g}")
# full-length cross-check (all chunks/runs) against the first variant, at full and odd length
v0 = next(iter(plans))
for nn in (n, n - 12345):
    yr = torch.empty_like(y)
    plans[v0](x, hin, hout, yr, nn)
    for v, p in plans.items():
        y.zero_()
        p(x, hin, hout, y, nn)
        torch.cuda.synchronize()
        d = (y[:nn] - yr[:nn]).abs().max().item()
        tail_zero = bool((y[nn:] == 0).all().item())
        print(f"variant {v} n={nn}: max|y - y_v{v0}| = {d:.3g}  untouched tail ok={tail_zero}")
res = {v: [] for v in plans}
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rnd in range(int(os.environ.get("ROUNDS", "10"))):
    for v, p in plans.items():
        st.record()
        for _ in range(5):
            p(x, hin, hout, y, n)
        en.record()
        en.synchronize()
        res[v].append(st.elapsed_time(en) / 5)
for v, t in res.items():
    t = sorted(t)
    print(f"variant {v}: median {t[len(t)//2]*1e3:.1f} us  min {t[0]*1e3:.1f} us  -> {16*n/t[0]/1e6:.0f} GB/s ({16*n/t[0]/1e6/8000*100:.1f}% of 8 TB/s)")
