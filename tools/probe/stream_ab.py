"""A/B N builds of libnsh_hip.so on the stream kernels in one process (interleaved rounds, HIP
events on one stream): nsh_copy, the 4-stage multiply_const chain (C2 fused), add_cc over
2^LOG2N complex samples; reports each build's median per-launch time and GB/s and whether its
outputs equal the first build's.
Usage: python tools/probe/stream_ab.py A.so B.so [...]   (env: LOG2N=28 ROUNDS=8)"""
import ctypes as C
import os
import sys

import numpy as np
import torch

paths = sys.argv[1:]
libs = [C.CDLL(os.path.abspath(p), mode=C.RTLD_LOCAL) for p in paths]
for L in libs:
    L.nsh_copy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    L.nsh_mul_const_chain_cc.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_void_p]
    L.nsh_add_cc.argtypes = [C.c_void_p] * 3 + [C.c_int64, C.c_void_p]
    L.nsh_synth_cf32.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
n = 1 << int(os.environ.get("LOG2N", "28"))
rounds = int(os.environ.get("ROUNDS", "8"))
s = torch.cuda.Stream()
x = torch.empty(n, dtype=torch.complex64, device="cuda")
x2 = torch.empty(n, dtype=torch.complex64, device="cuda")
assert libs[0].nsh_synth_cf32(x.data_ptr(), n, 0, 1, C.c_void_p(s.cuda_stream)) == 0
assert libs[0].nsh_synth_cf32(x2.data_ptr(), n, 0, 2, C.c_void_p(s.cuda_stream)) == 0
k = np.array([0.5, 0.25, 1.5, -0.5, 0.75, 0.1, 1.0, 2.0], np.float32)
ops = {
    "copy": (16, lambda L, y: L.nsh_copy(x.data_ptr(), y.data_ptr(), n * 8, C.c_void_p(s.cuda_stream))),
    "mulc_chain4": (16, lambda L, y: L.nsh_mul_const_chain_cc(x.data_ptr(), y.data_ptr(), n, k.ctypes.data, 4,
                                                             C.c_void_p(s.cuda_stream))),
    "add_cc": (24, lambda L, y: L.nsh_add_cc(x.data_ptr(), x2.data_ptr(), y.data_ptr(), n, C.c_void_p(s.cuda_stream))),
}
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, (bps, fn) in ops.items():
    ys = [torch.zeros(n, dtype=torch.complex64, device="cuda") for _ in libs]
    # clocks settle: every build in turn for WARM_S seconds (default 2, as lib_abn.py); with 10
    # passes only, the builds' in-round position moved the copy by up to 10 % (profiles/r04zs_*)
    import time
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < float(os.environ.get("WARM_S", "2")):
        for L, y in zip(libs, ys):
            assert fn(L, y) == 0
        s.synchronize()
    t = [[] for _ in libs]
    for _ in range(rounds):
        for i, (L, y) in enumerate(zip(libs, ys)):
            st.record(s)
            for _ in range(5):
                fn(L, y)
            en.record(s)
            en.synchronize()
            t[i].append(st.elapsed_time(en) / 5 * 1e3)
    for i, pth in enumerate(paths):
        med = float(np.median(t[i]))
        print("%s %s: median %.1f us, %.0f GB/s (%.1f%%), same-as-first=%s" % (
            os.path.basename(pth), name, med, bps * n / med / 1e3, bps * n / med / 1e3 / 80, bool(torch.equal(ys[i], ys[0]))),
            flush=True)
