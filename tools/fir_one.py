"""Run one FIR configuration (and a calibration copy) repeatedly -- the workload for the
rocprofv3 --pmc passes in tools/pmc_fir.sh."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import scipy.signal as ss
import torch

from newsched_amd import nsh

ap = argparse.ArgumentParser()
ap.add_argument("--algo", default="mfma", choices=["mfma", "direct", "f32", "casc", "chan", "mul4"])
ap.add_argument("--log2n", type=int, default=25)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--decim", type=int, default=1)
a = ap.parse_args()
n = 1 << a.log2n
h = ss.firwin(127, 0.2).astype(np.float32)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
nsh.synth(x, n, 0)
y = torch.empty_like(x)
hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
hout = torch.zeros_like(hin)
if a.algo == "chan":  # C4's channelizer (nsh_channelizer1024), bench.py's weights
    import bench

    w = torch.from_numpy(bench.c4_weights()).cuda()
    for _ in range(a.reps):
        nsh.channelizer1024(x, y, w, n // 1024)

    class p:
        kernel = "k_chan1024"
elif a.algo == "mul4":  # C2's fused chain (nsh_mul_const_chain_cc)
    import bench

    for _ in range(a.reps):
        nsh.mul_const_chain_cc(x, y, n, bench.C2_KS)

    class p:
        kernel = "k_map_c_v4"
elif a.algo == "casc":  # C5's fused chain (nsh_fir_cascade_ccf): 4 x fir(firwin(127, 0.45), 2)
    p = nsh.FirCascadePlan([(ss.firwin(127, 0.45).astype(np.float32), 2)] * 4)
    hc = torch.zeros(p.hist_len, dtype=torch.complex64, device="cuda")
    for _ in range(a.reps):
        p(x, None, hc, y, n // 16)
else:
    p = nsh.FirPlan(h, a.decim, {"mfma": nsh.FIR_MFMA, "direct": nsh.FIR_DIRECT,
                                  "f32": nsh.FIR_MFMA_F32}[a.algo])
    for _ in range(a.reps):
        p(x, hin, hout, y, n // a.decim)
for _ in range(a.reps):
    nsh.copy(x, y, 8 * n)  # calibration: exactly 8n B read + 8n B written per launch
torch.cuda.synchronize()
print("done", n, a.algo, p.kernel)
