"""Kernel-level timing of libnsh_hip.so entry points (HIP events on the launch stream).
Usage: python tools/kbench.py [--n LOG2] [--reps R]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh


def timeit(fn, reps, stream):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        for _ in range(2):
            fn()
        st.record(stream)
        for _ in range(reps):
            fn()
        en.record(stream)
    en.synchronize()
    return st.elapsed_time(en) / reps  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=28)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n = 1 << a.n
    s = torch.cuda.Stream()
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    y = torch.empty_like(x)
    nsh.synth(x, n, 0, stream=s)
    hin = torch.zeros(160, dtype=torch.complex64, device="cuda")
    hout = torch.zeros_like(hin)
    res = {}
    h = ss.firwin(127, 0.2).astype(np.float32)
    for name, algo in [("fir_direct", nsh.FIR_DIRECT), ("fir_mfma", nsh.FIR_MFMA)]:
        p = nsh.FirPlan(h, 1, algo)
        ms = timeit(lambda: p(x, hin, hout, y, n, stream=s), a.reps, s)
        res[name] = {"ms": ms, "GS/s": n / ms / 1e6, "GB/s": 16 * n / ms / 1e6, "hbm_frac": 16 * n / ms / 1e6 / 8000}
    ms = timeit(lambda: nsh.copy(x, y, 8 * n, stream=s), a.reps, s)
    res["copy"] = {"ms": ms, "GB/s": 16 * n / ms / 1e6}
    ms = timeit(lambda: nsh.mul_const_chain_cc(x, y, n, [np.exp(0.1j), np.exp(0.2j), np.exp(0.3j), np.exp(0.4j)], stream=s), a.reps, s)
    res["mulchain4"] = {"ms": ms, "GS/s": n / ms / 1e6, "GB/s": 16 * n / ms / 1e6}
    z = torch.empty_like(x)
    ms = timeit(lambda: nsh.add_cc(x, y, z, n, stream=s), a.reps, s)
    res["add_cc"] = {"ms": ms, "GS/s": n / ms / 1e6, "GB/s": 24 * n / ms / 1e6}
    ms = timeit(lambda: nsh.fft1024(x, y, n // 1024, stream=s), a.reps, s)
    res["fft1024"] = {"ms": ms, "GS/s": n / ms / 1e6, "GB/s": 16 * n / ms / 1e6}
    w = torch.ones(1024, dtype=torch.complex64, device="cuda")
    ms = timeit(lambda: nsh.channelizer1024(x, y, w, n // 1024, stream=s), a.reps, s)
    res["chan1024"] = {"ms": ms, "GS/s": n / ms / 1e6, "GB/s": 16 * n / ms / 1e6}
    for dd in (2, 4):
        for nm, al in (("direct", nsh.FIR_DIRECT), ("mfma", nsh.FIR_MFMA)):
            p = nsh.FirPlan(ss.firwin(127, 0.45).astype(np.float32), dd, al)
            ms = timeit(lambda: p(x, hin, hout, y, n // dd, stream=s), a.reps, s)
            gbs = (8 + 8 / dd) * n / ms / 1e6
            res[f"fir_{nm}_d{dd}"] = {"ms": ms, "GS/s_in": n / ms / 1e6, "GB/s": gbs, "hbm_frac": gbs / 8000}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
