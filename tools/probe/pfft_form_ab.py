"""A/B of the C5 kernel forms in one process and one library: k_fir_pfft<16,1> (NSH_PFFT_FORM=1)
vs k_fir_pfft2<16> (NSH_PFFT_FORM=2), the form chosen at plan creation. 4 x fir(firwin(127, 0.45),
2) over 2^LOG2N resident inputs; interleaved rounds (order swapped every round), HIP events on one
stream, >= 1 s warm-up. Prints each form's median launch time, its HBM fraction at 8.5 B per input
sample, and the largest difference between the forms relative to max|y| (both are within fp32
transform rounding of the staged chain; the tests check each against the oracle).
Usage: python tools/probe/pfft_form_ab.py   (env: LOG2N=28 ROUNDS=10 FORMS=1,2)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh

n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "10"))
forms = [int(v) for v in os.environ.get("FORMS", "1,2").split(",")]
h = ss.firwin(127, 0.45).astype(np.float32)
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0, stream=s)
n_out = n // 16
plans, ys, hs = [], [], []
for fm in forms:
    os.environ["NSH_PFFT_FORM"] = str(fm)
    plans.append(nsh.FirCascadePlan([(h, 2)] * 4))
    ys.append(torch.zeros(n_out, dtype=torch.complex64, device="cuda"))
    hs.append(torch.zeros(1890, dtype=torch.complex64, device="cuda"))
os.environ.pop("NSH_PFFT_FORM")


def run(i):
    plans[i](x, None, hs[i], ys[i], n_out, stream=s)


st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.time()
while time.time() - t0 < 1.0:
    for i in range(len(forms)):
        run(i)
s.synchronize()
t = [[] for _ in forms]
for rd in range(rounds):
    order = range(len(forms)) if rd % 2 == 0 else reversed(range(len(forms)))
    for i in order:
        with torch.cuda.stream(s):
            st.record(s)
            for _ in range(5):
                run(i)
            en.record(s)
        en.synchronize()
        t[i].append(st.elapsed_time(en) / 5 * 1e3)
torch.cuda.synchronize()
ref = ys[0]
scale = ref.abs().max().item()
for i, fm in enumerate(forms):
    med = float(np.median(t[i]))
    d = (ys[i] - ref).abs().max().item() / scale
    print(json.dumps({"form": fm, "kernel": plans[i].kernel, "median_us": round(med, 1), "min_us": round(min(t[i]), 1),
                      "GSps_input": round(n / med / 1e3, 1), "hbm_frac_8.5B": round(8.5 * n / med / 1e3 / 8000, 4),
                      "max_rel_diff_vs_first": d, "hist_equal": bool(torch.equal(hs[i], hs[0]))}), flush=True)
