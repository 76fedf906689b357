"""Python face of the CPU ORACLE (oracle/nsh_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker. See nsh_oracle.c for what each function restates
(reference file:line) and which results are pinned by reference vectors vs. by
scipy/numpy fixtures ("parity unpinned" against the reference for FIR/FFT).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libnsh_oracle.so")
_lib = None

SEED = 0x6E736368


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = C.CDLL(_SO)
        vp, i64, u64, f, i = C.c_void_p, C.c_int64, C.c_uint64, C.c_float, C.c_int
        L.orc_synth_cf32.argtypes = [vp, i64, u64, u64]
        L.orc_copy.argtypes = [vp, vp, C.c_size_t]
        L.orc_mul_const_cc.argtypes = [vp, vp, i64, f, f]
        L.orc_mul_const_ff.argtypes = [vp, vp, i64, f]
        L.orc_mul_const_chain_cc.argtypes = [vp, vp, i64, vp, i]
        L.orc_add_cc.argtypes = [vp, vp, vp, i64]
        L.orc_mul_cc.argtypes = [vp, vp, vp, i64]
        L.orc_fir_ccf.argtypes = [vp, vp, vp, vp, i64, vp, i, i]
        L.orc_fft1024.argtypes = [vp, vp, i64, i]
        L.orc_channelizer1024.argtypes = [vp, vp, vp, i64]
        for fn in ("orc_synth_cf32", "orc_copy", "orc_mul_const_cc", "orc_mul_const_ff",
                   "orc_mul_const_chain_cc", "orc_add_cc", "orc_mul_cc", "orc_fir_ccf",
                   "orc_fft1024", "orc_channelizer1024"):
            getattr(L, fn).restype = None
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def c64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.complex64))


def synth(n: int, first_index: int = 0, seed: int = SEED) -> np.ndarray:
    y = np.empty(n, np.complex64)
    _load().orc_synth_cf32(_p(y), n, first_index, seed)
    return y


def mul_const_cc(x, k: complex) -> np.ndarray:
    x = c64(x)
    y = np.empty_like(x)
    _load().orc_mul_const_cc(_p(x), _p(y), x.size, float(k.real), float(k.imag))
    return y


def mul_const_ff(x, k: float) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(x, np.float32))
    y = np.empty_like(x)
    _load().orc_mul_const_ff(_p(x), _p(y), x.size, float(k))
    return y


def mul_const_chain_cc(x, ks) -> np.ndarray:
    x = c64(x)
    y = np.empty_like(x)
    k = np.asarray([v for kk in ks for v in (complex(kk).real, complex(kk).imag)], np.float32)
    _load().orc_mul_const_chain_cc(_p(x), _p(y), x.size, _p(k), len(ks))
    return y


def add_cc(a, b) -> np.ndarray:
    a, b = c64(a), c64(b)
    y = np.empty_like(a)
    _load().orc_add_cc(_p(a), _p(b), _p(y), a.size)
    return y


def mul_cc(a, b) -> np.ndarray:
    a, b = c64(a), c64(b)
    y = np.empty_like(a)
    _load().orc_mul_cc(_p(a), _p(b), _p(y), a.size)
    return y


def fir_ccf(x, taps, decim: int = 1, hist=None, return_hist: bool = False):
    """y[m] = sum_k h[k] x[m*decim - k]; len(x) must be a multiple of decim."""
    x = c64(x)
    h = np.ascontiguousarray(np.asarray(taps, np.float32))
    L = h.size
    n_out = x.size // decim
    y = np.empty(n_out, np.complex64)
    hist_a = c64(hist) if hist is not None else None
    hout = np.empty(max(L - 1, 1), np.complex64)
    _load().orc_fir_ccf(_p(x), _p(hist_a) if hist_a is not None else None, _p(hout), _p(y), n_out,
                        _p(h), L, decim)
    if return_hist:
        return y, hout[: L - 1]
    return y


def fft1024(x, inverse: bool = False) -> np.ndarray:
    x = c64(x)
    assert x.size % 1024 == 0
    y = np.empty_like(x)
    _load().orc_fft1024(_p(x), _p(y), x.size // 1024, 1 if inverse else 0)
    return y


def channelizer1024(x, w) -> np.ndarray:
    x, w = c64(x), c64(w)
    y = np.empty_like(x)
    _load().orc_channelizer1024(_p(x), _p(y), _p(w), x.size // 1024)
    return y


def tol_ok(y, y_ref, rel: float = 1e-5):
    """SURVEY.md §8c tolerance: max|y - y_ref| <= rel * max|y_ref| (norm-wise) and
    |y - y_ref| <= rel*|y_ref| + 0.1*rel*max|y_ref| per element. Returns (ok, max_abs_err,
    scale)."""
    y = np.asarray(y, np.complex128)
    r = np.asarray(y_ref, np.complex128)
    scale = float(np.max(np.abs(r))) if r.size else 0.0
    err = np.abs(y - r)
    maxerr = float(err.max()) if err.size else 0.0
    ok = maxerr <= rel * scale and bool(np.all(err <= rel * np.abs(r) + 0.1 * rel * scale))
    return ok, maxerr, scale
