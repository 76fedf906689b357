"""ctypes binding of libnsh_hip.so (include/nsh_hip.h) -- the MI355X kernel shim.

This module is the Python view of the C-ABI boundary; the C++17 newsched host links the
same library directly. It never falls back to a CPU implementation: if the in-tree
library is missing, `lib()` raises.

Device memory and streams on the Python side are torch tensors / torch streams (plumbing
only); every pointer handed to the shim is a raw device address.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
HIP_LIB = os.path.join(LIB_DIR, "libnsh_hip.so")
# NSH_HIP_LIB: another build of the library (A/B probes)
HIP_LIB = os.environ.get("NSH_HIP_LIB") or HIP_LIB

NSH_H2D, NSH_D2H, NSH_D2D, NSH_DEFAULT = 0, 1, 2, 3
FIR_AUTO, FIR_DIRECT, FIR_MFMA, FIR_MFMA16, FIR_MFMA_BF16X3, FIR_MFMA_F32, FIR_PFFT = 0, 1, 2, 3, 4, 5, 6

# name -> (restype, argtypes); mirrors include/nsh_hip.h exactly (tests check the header).
_vp, _i, _i64, _u64, _sz, _f = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_size_t, C.c_float
SIGNATURES = {
    "nsh_abi_version": (_i, []),
    "nsh_last_error": (C.c_char_p, []),
    "nsh_get_device_count": (_i, [C.POINTER(_i)]),
    "nsh_set_device": (_i, [_i]),
    "nsh_device_info": (_i, [_i, C.POINTER(_i), C.POINTER(_i), C.POINTER(_sz), C.c_char_p, _i]),
    "nsh_device_pci_id": (_i, [_i, C.c_char_p, _i]),
    "nsh_pointer_device": (_i, [_vp, C.POINTER(_i)]),
    "nsh_device_sync": (_i, []),
    "nsh_stream_create": (_i, [_i, C.POINTER(_vp)]),
    "nsh_stream_destroy": (_i, [_vp]),
    "nsh_stream_sync": (_i, [_vp]),
    "nsh_stream_query": (_i, [_vp]),
    "nsh_event_create": (_i, [C.POINTER(_vp)]),
    "nsh_event_destroy": (_i, [_vp]),
    "nsh_event_record": (_i, [_vp, _vp]),
    "nsh_event_query": (_i, [_vp]),
    "nsh_event_sync": (_i, [_vp]),
    "nsh_event_elapsed_ms": (_i, [_vp, _vp, C.POINTER(_f)]),
    "nsh_stream_wait_event": (_i, [_vp, _vp]),
    "nsh_time_next_launch": (_i, [_vp, _vp]),
    "nsh_timed_launches": (_i, [C.POINTER(_u64)]),
    "nsh_clock_sample": (_i, [_vp, _i64, _vp]),
    "nsh_malloc": (_i, [_i, _sz, C.POINTER(_vp)]),
    "nsh_free": (_i, [_vp]),
    "nsh_host_alloc": (_i, [_sz, C.POINTER(_vp)]),
    "nsh_host_free": (_i, [_vp]),
    "nsh_memcpy_async": (_i, [_vp, _vp, _sz, _i, _vp]),
    "nsh_memset_async": (_i, [_vp, _i, _sz, _vp]),
    "nsh_ring_alloc": (_i, [_i, _sz, C.POINTER(_vp), C.POINTER(_sz), C.POINTER(_i)]),
    "nsh_ring_free": (_i, [_vp]),
    "nsh_ipc_mem_export": (_i, [_vp, _vp]),
    "nsh_ipc_mem_open": (_i, [_i, _vp, C.POINTER(_vp)]),
    "nsh_ipc_mem_close": (_i, [_vp]),
    "nsh_copy": (_i, [_vp, _vp, _sz, _vp]),
    "nsh_mul_const_cc": (_i, [_vp, _vp, _i64, _f, _f, _vp]),
    "nsh_mul_const_ff": (_i, [_vp, _vp, _i64, _f, _vp]),
    "nsh_mul_const_chain_cc": (_i, [_vp, _vp, _i64, C.POINTER(_f), _i, _vp]),
    "nsh_add_cc": (_i, [_vp, _vp, _vp, _i64, _vp]),
    "nsh_mul_cc": (_i, [_vp, _vp, _vp, _i64, _vp]),
    "nsh_mul_const_vcc": (_i, [_vp, _vp, _vp, _i, _i64, _vp]),
    "nsh_synth_cf32": (_i, [_vp, _i64, _u64, _u64, _vp]),
    "nsh_fir_plan_create": (_i, [_i, C.POINTER(_f), _i, _i, _i, C.POINTER(_vp)]),
    "nsh_fir_plan_destroy": (_i, [_vp]),
    "nsh_fir_plan_algo": (_i, [_vp]),
    "nsh_fir_plan_kernel": (C.c_char_p, [_vp]),
    "nsh_fir_ccf": (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "nsh_fir_cascade_plan_create": (_i, [_i, C.POINTER(C.POINTER(_f)), C.POINTER(_i), C.POINTER(_i), _i,
                                         C.POINTER(_vp)]),
    "nsh_fir_cascade_plan_destroy": (_i, [_vp]),
    "nsh_fir_cascade_decim": (_i, [_vp]),
    "nsh_fir_cascade_hist_len": (_i, [_vp]),
    "nsh_fir_cascade_kernel": (C.c_char_p, [_vp]),
    "nsh_fir_cascade_ccf": (_i, [_vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "nsh_fft1024_c2c": (_i, [_vp, _vp, _i64, _i, _vp]),
    "nsh_channelizer1024": (_i, [_vp, _vp, _vp, _i64, _vp]),
}

_lib = None
_lock = threading.Lock()


class NshError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load the in-tree libnsh_hip.so (raises if it was not built -- no fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(HIP_LIB):
                raise NshError(f"{HIP_LIB} is missing: run `make hip` (or __graft_entry__.build())")
            L = C.CDLL(HIP_LIB, mode=C.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().nsh_last_error().decode(errors="replace")
        raise NshError(f"{what or 'nsh call'} failed (rc={rc}): {msg}")


def ptr(t) -> int:
    """Raw device address of a torch tensor (or an int passthrough)."""
    return t if isinstance(t, int) else t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def pointer_device(p) -> int:
    """The GPU whose device memory p points into, -1 for host memory / NULL (nsh_pointer_device)."""
    d = C.c_int(-2)
    check(lib().nsh_pointer_device(C.c_void_p(ptr(p)), C.byref(d)), "nsh_pointer_device")
    return d.value


# ---- thin typed wrappers over torch tensors (complex64 or float32 views) -------------
def copy(src, dst, nbytes: int, stream=None):
    check(lib().nsh_copy(ptr(src), ptr(dst), nbytes, stream_ptr(stream)), "nsh_copy")


def mul_const_cc(x, y, n: int, k: complex, stream=None):
    check(lib().nsh_mul_const_cc(ptr(x), ptr(y), n, float(k.real), float(k.imag), stream_ptr(stream)),
          "nsh_mul_const_cc")


def mul_const_ff(x, y, n: int, k: float, stream=None):
    check(lib().nsh_mul_const_ff(ptr(x), ptr(y), n, float(k), stream_ptr(stream)), "nsh_mul_const_ff")


def mul_const_chain_cc(x, y, n: int, ks, stream=None):
    arr = (C.c_float * (2 * len(ks)))(*[v for k in ks for v in (complex(k).real, complex(k).imag)])
    check(lib().nsh_mul_const_chain_cc(ptr(x), ptr(y), n, arr, len(ks), stream_ptr(stream)),
          "nsh_mul_const_chain_cc")


def add_cc(a, b, y, n: int, stream=None):
    check(lib().nsh_add_cc(ptr(a), ptr(b), ptr(y), n, stream_ptr(stream)), "nsh_add_cc")


def mul_cc(a, b, y, n: int, stream=None):
    check(lib().nsh_mul_cc(ptr(a), ptr(b), ptr(y), n, stream_ptr(stream)), "nsh_mul_cc")


def mul_const_vcc(x, y, k, vlen: int, nitems: int, stream=None):
    """y[i][j] = x[i][j] * k[j] over nitems items of vlen samples (k: device, vlen complex)."""
    check(lib().nsh_mul_const_vcc(ptr(x), ptr(y), ptr(k), vlen, nitems, stream_ptr(stream)), "nsh_mul_const_vcc")


class ClockSampler:
    """nsh_clock_sample on a side stream: start() before the work to observe, mhz() after it
    (waits for the sample). One wave sleeping between two counter reads, ~real_ms long."""

    def __init__(self, real_ms: float = 8.0):
        import torch

        self._ticks = max(1, int(real_ms * 1e5))  # 100 MHz real-time counter
        self._out = torch.zeros(2, dtype=torch.int64, device="cuda")
        self._s = torch.cuda.Stream()

    def start(self):
        check(lib().nsh_clock_sample(ptr(self._out), self._ticks, stream_ptr(self._s)), "nsh_clock_sample")

    def mhz(self) -> float:
        self._s.synchronize()
        cyc, ticks = (int(v) for v in self._out.cpu().tolist())
        return 100.0 * cyc / ticks if ticks > 0 else float("nan")


def synth(y, n: int, first_index: int = 0, seed: int = 0x6E736368, stream=None):
    check(lib().nsh_synth_cf32(ptr(y), n, first_index, seed, stream_ptr(stream)), "nsh_synth_cf32")


def fft1024(x, y, nframes: int, inverse: bool = False, stream=None):
    check(lib().nsh_fft1024_c2c(ptr(x), ptr(y), nframes, 1 if inverse else 0, stream_ptr(stream)),
          "nsh_fft1024_c2c")


def channelizer1024(x, y, w, nframes: int, stream=None):
    check(lib().nsh_channelizer1024(ptr(x), ptr(y), ptr(w), nframes, stream_ptr(stream)),
          "nsh_channelizer1024")


class FirPlan:
    """Device-resident FIR plan (taps uploaded/split once); see nsh_fir_ccf."""

    def __init__(self, taps, decim: int = 1, algo: int = FIR_AUTO, device: int = 0):
        import numpy as np

        t = np.ascontiguousarray(np.asarray(taps, dtype=np.float32))
        self.ntaps = int(t.size)
        self.decim = int(decim)
        h = C.c_void_p()
        arr = t.ctypes.data_as(C.POINTER(C.c_float))
        check(lib().nsh_fir_plan_create(device, arr, self.ntaps, self.decim, algo, C.byref(h)),
              "nsh_fir_plan_create")
        self._h = h
        self.algo = lib().nsh_fir_plan_algo(h)
        self.kernel = lib().nsh_fir_plan_kernel(h).decode()

    def __call__(self, x, hist_in, hist_out, y, n_out: int, stream=None):
        check(lib().nsh_fir_ccf(self._h, ptr(x), ptr(hist_in), ptr(hist_out), ptr(y), n_out,
                                stream_ptr(stream)), "nsh_fir_ccf")

    def close(self):
        if getattr(self, "_h", None):
            lib().nsh_fir_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FirCascadePlan:
    """A chain of fir_filter_ccf(taps_s, decim_s) stages as one pass; see nsh_fir_cascade_ccf."""

    def __init__(self, stages, device: int = 0):
        import numpy as np

        self._taps = [np.ascontiguousarray(np.asarray(t, dtype=np.float32)) for t, _ in stages]
        n = len(self._taps)
        tp = (C.POINTER(C.c_float) * n)(*[t.ctypes.data_as(C.POINTER(C.c_float)) for t in self._taps])
        nt = (C.c_int * n)(*[int(t.size) for t in self._taps])
        dc = (C.c_int * n)(*[int(d) for _, d in stages])
        h = C.c_void_p()
        check(lib().nsh_fir_cascade_plan_create(device, tp, nt, dc, n, C.byref(h)), "nsh_fir_cascade_plan_create")
        self._h = h
        self.decim = lib().nsh_fir_cascade_decim(h)
        self.hist_len = lib().nsh_fir_cascade_hist_len(h)
        self.kernel = lib().nsh_fir_cascade_kernel(h).decode()

    def __call__(self, x, hist_in, hist_out, y, n_out: int, stream=None):
        """n_out outputs from n_out * decim inputs; hist_in/hist_out: hist_len samples (or 0/None)."""
        check(lib().nsh_fir_cascade_ccf(self._h, ptr(x) if x is not None else None,
                                        ptr(hist_in) if hist_in is not None else None,
                                        ptr(hist_out) if hist_out is not None else None, ptr(y), n_out,
                                        stream_ptr(stream)), "nsh_fir_cascade_ccf")

    def close(self):
        if getattr(self, "_h", None):
            lib().nsh_fir_cascade_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
