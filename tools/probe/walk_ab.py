"""Decimator walks A/B in one process: two plans of one libnsh_hip.so, created under different
NSH_DEC_WALK_MASK values (bit D: the lockstep walk k_fir_mfma13 + k_fir_exact13; clear: the
contiguous walk k_fir_mfma11), interleaved rounds of 10 calls each, HIP events around each
round on one stream (both kernels of a call inside). 127 taps firwin(127, 0.2), 2^LOG2N inputs.
Prints each plan's median / min per-call time, GB/s of (8 + 8/D) B per input sample, % of
8 TB/s, and the max |difference| of its output relative to the first plan's.
Usage: python tools/probe/walk_ab.py
  env: DECIM=4 LOG2N=28 ROUNDS=12 INPUT=synth|spikeK (every K-th 2048-input chunk holds a 2^40
       spike: the exact path) MASKS=0,16; a mask may carry ":W" (NSH_WALK_WGPC, workgroups per CU
       of the lockstep walk), e.g. MASKS=16:2,16:3"""
import os
import statistics
import sys
import time

import numpy as np
import scipy.signal as ss
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from newsched_amd import nsh  # noqa: E402

D = int(os.environ.get("DECIM", "4"))
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "12"))
inp = os.environ.get("INPUT", "synth")
masks = os.environ.get("MASKS", "0,16").split(",")
h = ss.firwin(127, 0.2).astype(np.float32)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
if inp.startswith("spike"):
    k = int(inp[5:])
    x.view(-1, 2048)[::k, 7] = 2.0 ** 40
plans = []
for m in masks:
    mask, _, wgpc = m.partition(":")
    os.environ["NSH_DEC_WALK_MASK"] = mask
    os.environ["NSH_WALK_WGPC"] = wgpc or "2"
    plans.append(nsh.FirPlan(h, D, nsh.FIR_MFMA))
n_out = n // D
s = torch.cuda.Stream()
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
ys = [torch.zeros(n_out, dtype=torch.complex64, device="cuda") for _ in plans]
for p, y in zip(plans, ys):
    p(x, hin, hout, y, n_out, stream=s)
s.synchronize()
t_w = time.perf_counter()
while time.perf_counter() - t_w < 2.0:
    for p, y in zip(plans, ys):
        p(x, hin, hout, y, n_out, stream=s)
    s.synchronize()
times = [[] for _ in plans]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    order = range(len(plans)) if r % 2 == 0 else reversed(range(len(plans)))
    for i in order:
        e0.record(s)
        for _ in range(10):
            plans[i](x, hin, hout, ys[i], n_out, stream=s)
        e1.record(s)
        s.synchronize()
        times[i].append(e0.elapsed_time(e1) / 10 * 1e3)
bpi = 8 + 8 / D
for p, m, t, y in zip(plans, masks, times, ys):
    med = statistics.median(t)
    gbs = bpi * n / (med * 1e-6) / 1e9
    d = (y - ys[0]).abs().max().item() / max(ys[0].abs().max().item(), 1e-30)
    print("mask %s %s: median %.1f us min %.1f us -> %.0f GS/s input, %.0f GB/s = %.2f %% of 8 TB/s; max|d|/max|y| %.2e"
          % (m, p.kernel, med, min(t), n / (med * 1e-6) / 1e9, gbs, gbs / 80.0, d), flush=True)
