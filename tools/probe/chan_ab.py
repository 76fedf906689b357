"""A/B the channelizer dispatch shapes in one process: NSH_CHAN_VARIANT=0 (grid-stride k_chan1024)
vs K > 0 (k_chan1024x, XCD-ordered groups of 4K frames) -- the variant is read once per process, so
each runs in its own child; 2^28 samples, HIP events, >= 1 s warm-up, bit-identity via a digest."""
import json
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import time
    import numpy as np
    import torch
    from newsched_amd import nsh
    n = 1 << 28
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, 0)
    y = torch.empty_like(x)
    w = torch.from_numpy((np.exp(-0.5 * ((np.arange(1024) - 512) / 100.0) ** 2)).astype(np.complex64)).cuda()
    s = torch.cuda.Stream()
    t0 = time.time()
    while time.time() - t0 < 1.0:
        nsh.channelizer1024(x, y, w, n // 1024, stream=s)
        s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(10):
                nsh.channelizer1024(x, y, w, n // 1024, stream=s)
            e1.record(s)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 10 * 1e3)
    dig = float(y.view(torch.float32).double().abs().sum().item())
    us = sorted(ts)[2]
    print(json.dumps({"variant": os.environ.get("NSH_CHAN_VARIANT", "0"), "median_us": round(us, 1),
                      "GBs": round(16 * n / us / 1e3, 1), "frac": round(16 * n / us / 1e3 / 8000, 4), "digest": dig}), flush=True)
    sys.exit(0)
for rnd in range(2):
    for v in sys.argv[1:] or ["0", "1", "2", "4"]:
        env = dict(os.environ, NSH_CHAN_VARIANT=v)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True, text=True, timeout=200)
        print(r.stdout.strip() or r.stderr[-500:], flush=True)
