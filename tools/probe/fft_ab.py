"""A/B the fft1024 / channelizer forms in one process (interleaved rounds): NSH_FFT_VARIANT
0 = register prefetch of the next frame (default), 1 = no prefetch, 3 workgroups per CU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from newsched_amd import nsh

n = 1 << int(os.environ.get("LOG2N", "28"))
nf = n // 1024
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
w = torch.from_numpy(((1 + 0.5 * np.cos(2 * np.pi * np.arange(1024) / 1024)) / 1024).astype(np.complex64)).cuda()
ys = {v: torch.empty_like(x) for v in "01"}
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for kind in ("fft", "chan"):
    res = {v: [] for v in "01"}
    def run(v):
        os.environ["NSH_FFT_VARIANT"] = v
        if kind == "fft":
            nsh.fft1024(x, ys[v], nf)
        else:
            nsh.channelizer1024(x, ys[v], w, nf)
    for v in "01":
        run(v)
    torch.cuda.synchronize()
    same = bool(torch.equal(ys["0"], ys["1"]))
    for _ in range(int(os.environ.get("ROUNDS", "12"))):
        for v in "01":
            run(v)
            st.record()
            for _ in range(5):
                run(v)
            en.record()
            en.synchronize()
            res[v].append(st.elapsed_time(en) / 5 * 1e3)
    for v, t in res.items():
        t = sorted(t)
        print(f"{kind} variant {v}: median {t[len(t)//2]:.1f} us min {t[0]:.1f} us -> {16 * n / t[len(t)//2] / 1e3:.0f} GB/s"
              f"  bit-identical={same}", flush=True)
