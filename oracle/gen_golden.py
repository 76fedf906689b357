"""Generate tests/golden/ fixtures with numpy/scipy (run in the build container only).

TEST INFRASTRUCTURE. The reference has no FIR/FFT blocks and cannot be built or imported
here, so the floating-point fixtures are produced from the published
algorithms the GNU Radio conventions name: scipy.signal.lfilter (FIR, zero initial state),
numpy.fft (FFT). The identity/copy vectors are the reference's own test vectors
(schedulers/mt/test/qa_scheduler_mt.cpp:17-39, :79-135; qa_block_grouping.cpp:15-66;
test/cuda/qa_scheduler_mt_cuda_copy.cpp:20-86), stored as generator rules + checksums.

    python oracle/gen_golden.py   # rewrites tests/golden/*.npz and manifest.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import scipy
import scipy.signal as ss

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
SEED = 0x6E736368
M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(M64)
    return z ^ (z >> np.uint64(31))


def synth(n: int, first: int = 0, seed: int = SEED) -> np.ndarray:
    """Independent numpy restatement of BASELINE.md §2 (checks the C oracle too)."""
    with np.errstate(over="ignore"):
        j = (np.arange(2 * n, dtype=np.uint64) + np.uint64(2 * first)) ^ np.uint64(seed)
        z = splitmix64(j)
    u = (z >> np.uint64(40)).astype(np.int64).astype(np.float32) * np.float32(1.0 / 8388608.0) - np.float32(1.0)
    return (u[0::2] + 1j * u[1::2]).astype(np.complex64)


def cmul32(a: np.ndarray, k) -> np.ndarray:
    """std::complex<float> product with each product rounded to fp32 (no FMA)."""
    ar, ai = a.real.astype(np.float32), a.imag.astype(np.float32)
    kr, ki = np.float32(np.real(k)), np.float32(np.imag(k))
    re = (ar * kr).astype(np.float32) - (ai * ki).astype(np.float32)
    im = (ar * ki).astype(np.float32) + (ai * kr).astype(np.float32)
    return (re.astype(np.float32) + 1j * im.astype(np.float32)).astype(np.complex64)


def lfilter_c(h32: np.ndarray, x: np.ndarray) -> np.ndarray:
    return ss.lfilter(h32.astype(np.float64), [1.0], x.astype(np.complex128))


def main() -> int:
    os.makedirs(OUT, exist_ok=True)
    files = {}

    # C3: 127-tap lowpass, firwin(127, 0.2) (Hamming), fp32 taps.
    h3 = ss.firwin(127, 0.2).astype(np.float32)
    x = synth(16384)
    y3 = lfilter_c(h3, x).astype(np.complex64)
    # second segment continuing the same stream (history across calls)
    x_b = synth(4096, first=16384)
    y3_b = lfilter_c(h3, np.concatenate([x, x_b]))[16384:].astype(np.complex64)
    np.savez(os.path.join(OUT, "fir127.npz"), taps=h3, x=x, y=y3, x_next=x_b, y_next=y3_b)
    files["fir127.npz"] = "C3 taps firwin(127,0.2) fp32; x=synth(16384); y=lfilter(h,1,x); next segment continues the stream"

    # C5 stage: firwin(127, 0.45), decimation 2 -> y_D[m] = y[2m]; 4-stage chain /16.
    h5 = ss.firwin(127, 0.45).astype(np.float32)
    xd = synth(16384)
    yd = lfilter_c(h5, xd)[::2].astype(np.complex64)
    chain = xd.astype(np.complex128)
    for _ in range(4):
        chain = ss.lfilter(h5.astype(np.float64), [1.0], chain)[::2].astype(np.complex64).astype(np.complex128)
    np.savez(os.path.join(OUT, "fir127_decim2.npz"), taps=h5, x=xd, y=yd, y_chain4=chain.astype(np.complex64))
    files["fir127_decim2.npz"] = "C5 taps firwin(127,0.45); decim 2: y[m]=lfilter(h,1,x)[2m]; y_chain4 = 4 stages, fp32 between stages"

    # C2: 4x multiply_const_cc, k_i = exp(j theta_i), theta = 0.1..0.4, each stage fp32-rounded.
    ks = np.exp(1j * np.array([0.1, 0.2, 0.3, 0.4])).astype(np.complex64)
    xm = synth(8192)
    ym = xm
    for k in ks:
        ym = cmul32(ym, k)
    np.savez(os.path.join(OUT, "mulchain4.npz"), k=ks, x=xm, y=ym)
    files["mulchain4.npz"] = "C2 k=exp(j*{0.1,0.2,0.3,0.4}); std::complex<float> products per stage"

    # C4: fft1024 -> multiply W -> ifft1024 (unnormalised).
    b = np.arange(1024)
    W = ((1.0 + 0.5 * np.cos(2 * np.pi * b / 1024)) / 1024.0).astype(np.complex64)
    xf = synth(8192)
    F = np.fft.fft(xf.astype(np.complex128).reshape(-1, 1024), axis=1)
    Fi = np.fft.ifft(xf.astype(np.complex128).reshape(-1, 1024), axis=1) * 1024
    yc = (np.fft.ifft(F * W.astype(np.complex128), axis=1) * 1024).reshape(-1)
    np.savez(os.path.join(OUT, "fft1024.npz"), x=xf, X=F.reshape(-1).astype(np.complex64),
             Xi=Fi.reshape(-1).astype(np.complex64), w=W, y_chan=yc.astype(np.complex64))
    files["fft1024.npz"] = "C4 numpy.fft.fft / 1024*ifft per 1024-frame; channelizer W[b]=(1+0.5cos(2 pi b/1024))/1024"

    # Reference test vectors (exact formulas; store prefixes + digests of the full vectors).
    def digest(a: np.ndarray) -> str:
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    fan = (2 * np.arange(1_000_000) + 1j * (2 * np.arange(1_000_000) + 1)).astype(np.complex64)
    cuda = (np.arange(102_400) - 1j * np.arange(102_400)).astype(np.complex64)
    refvec = {
        "TwoSinks": {"src": "schedulers/mt/test/qa_scheduler_mt.cpp:17-39", "input": [1.0, 2.0, 3.0, 4.0, 5.0],
                     "expect": "each sink == input"},
        "BlockFanout": {"src": "schedulers/mt/test/qa_scheduler_mt.cpp:79-135", "rule": "x[i]=(2i,2i+1), i<1e6",
                        "k": 1.0, "nblocks": [2, 8, 16], "fixed_buf_size": 8192, "sha256": digest(fan)},
        "BasicBlockGrouping": {"src": "schedulers/mt/test/qa_block_grouping.cpp:15-66", "rule": "x[i]=(2i,2i+1), i<1e6",
                               "k": 1.0, "ngroups": [2, 4, 8], "nblocks": [2, 8, 16], "sha256": digest(fan)},
        "CudaCopy": {"src": "schedulers/mt/test/cuda/qa_scheduler_mt_cuda_copy.cpp:20-86", "rule": "x[i]=(i,-i), i<102400",
                     "veclen": 1024, "fixed_buf_size": 32768, "sha256": digest(cuda)},
    }
    manifest = {
        "generator": "oracle/gen_golden.py",
        "numpy": np.__version__, "scipy": scipy.__version__,
        "seed": SEED, "synth": "x[i]=(u(2i),u(2i+1)), u(j)=((splitmix64(seed^j)>>40)*2^-23)-1",
        "tolerance": {"rel_normwise": 1e-5, "rel_elementwise": 1e-5, "abs_elementwise_frac_of_max": 1e-6},
        "files": files,
        "reference_vectors": refvec,
        "synth_prefix": [[float(v.real), float(v.imag)] for v in synth(8)],
    }
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", sorted(files), "to", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
