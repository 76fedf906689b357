"""Does a stream kernel's rate depend on where its buffers landed in HBM? (r04zs saw the same copy
code run 665-754 us per 2^28 samples depending on its output buffer.) Allocates NB buffers of
2^LOG2N complex samples (hipMalloc through torch, or HIP-VMM rings through nsh_ring_alloc with
KIND=vmm), then times nsh_copy (k_copy_v4) from every input buffer to every output buffer,
interleaved over ROUNDS rounds (HIP events, 5 launches each), and prints the median per (in, out)
pair, per output buffer and per input buffer -- a placement effect shows as a stable ranking of
buffers across rounds and across the partner buffer.
Usage: python tools/probe/placement.py   (env: NB=6 LOG2N=28 ROUNDS=4 KIND=malloc|vmm)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from newsched_amd import nsh  # noqa: E402

nb = int(os.environ.get("NB", "6"))
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "4"))
kind = os.environ.get("KIND", "malloc")
L = nsh.lib()
s = torch.cuda.Stream()
bufs, keep = [], []
for i in range(nb):
    if kind == "vmm":
        b, act, dm = C.c_void_p(), C.c_size_t(), C.c_int()
        nsh.check(L.nsh_ring_alloc(0, 8 * n, C.byref(b), C.byref(act), C.byref(dm)), "ring")
        bufs.append(b.value)
        keep.append(b)
    else:
        t = torch.empty(n, dtype=torch.complex64, device="cuda")
        keep.append(t)
        bufs.append(t.data_ptr())
    nsh.check(L.nsh_synth_cf32(C.c_void_p(bufs[-1]), n, 0, 7, C.c_void_p(s.cuda_stream)), "synth")
s.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def copy(i, o):
    nsh.check(L.nsh_copy(C.c_void_p(bufs[i]), C.c_void_p(bufs[o]), 8 * n, C.c_void_p(s.cuda_stream)), "copy")


t0 = time.time()
while time.time() - t0 < 1.5:  # clocks settle
    copy(0, 1)
    s.synchronize()
res = {}
for r in range(rounds):
    for i in range(nb):
        for o in range(nb):
            if i == o:
                continue
            e0.record(s)
            for _ in range(5):
                copy(i, o)
            e1.record(s)
            e1.synchronize()
            res.setdefault((i, o), []).append(e0.elapsed_time(e1) / 5 * 1e3)
med = {k: float(np.median(v)) for k, v in res.items()}
pct = lambda us: round(16.0 * n / (us * 1e-6) / 8e12 * 100, 2)
print("# kind", kind, "buffers", [hex(b) for b in bufs], flush=True)
for o in range(nb):
    row = [med[(i, o)] for i in range(nb) if i != o]
    print(json.dumps({"out": o, "median_us": round(float(np.median(row)), 1), "pct": pct(float(np.median(row))),
                      "per_in": [round(x, 1) for x in row]}), flush=True)
for i in range(nb):
    col = [med[(i, o)] for o in range(nb) if o != i]
    print(json.dumps({"in": i, "median_us": round(float(np.median(col)), 1), "pct": pct(float(np.median(col)))}),
          flush=True)
spread = [max(v) - min(v) for v in res.values()]
print(json.dumps({"round_to_round_spread_us_median": round(float(np.median(spread)), 1),
                  "all_pairs_min_us": round(min(med.values()), 1), "all_pairs_max_us": round(max(med.values()), 1)}))
if kind == "vmm":
    for b in keep:
        L.nsh_ring_free(b)
