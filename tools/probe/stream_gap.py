"""Per-step gap of the streaming C3 flowgraph (one run of K back-to-back 2^28-sample batches)
under three kernel-timing forms: the launch records its own events (default, nsh_time_next_launch),
two event records around each launch (NSH_FIR_TIMING=records), no timing. Each form in its own
process (the env var is read once); prints one JSON line per form.
Usage: python tools/probe/stream_gap.py [K] [ROUNDS]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 5

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, %r)
import numpy as np, scipy.signal as ss, torch
from newsched_amd import nsr
K, R, timing = %d, %d, %s
h = ss.firwin(127, 0.2).astype(np.float32)
n = 1 << 28
fb = nsr.FirBench(h, n, out_buf_bytes=2048 << 20, timing=timing)
fb.set_batches(K)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 1.5:
    fb.run()
steps, ks = [], []
for _ in range(R):
    s0 = fb.stats()
    torch.cuda.synchronize()
    t = time.perf_counter()
    fb.run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    s1 = fb.stats()
    steps.append(el / K * 1e6)
    if timing:
        ks.append((s1["kernel_ms"] - s0["kernel_ms"]) / (s1["launches"] - s0["launches"]) * 1e3)
r = {"step_us": sorted(steps)[len(steps) // 2]}
if ks:
    r["kernel_us"] = sorted(ks)[len(ks) // 2]
    r["gap_us"] = r["step_us"] - r["kernel_us"]
print(json.dumps(r))
'''

for mode in ("ext", "records", "off"):
    env = dict(os.environ)
    if mode == "records":
        env["NSH_FIR_TIMING"] = "records"
    code = CHILD % (ROOT, K, R, "False" if mode == "off" else "True")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:]
    print(json.dumps({"mode": mode, "K": K, "result": line}), flush=True)
