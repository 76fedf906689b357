"""ctypes binding of libnewsched.so's flowgraph runners (include/nsr_flowgraph.h).

The flowgraphs are built and run by the C++ runtime (gr::flowgraph, scheduler_hip,
hip_buffer, gr::hip blocks); Python only passes POD arguments."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import nsh

RT_LIB = os.environ.get("NSR_LIB") or os.path.join(nsh.LIB_DIR, "libnewsched.so")  # NSR_LIB: probe builds
_lib = None

_vp, _i, _i64, _u64, _sz, _d = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_size_t, C.c_double
SIGNATURES = {
    "nsr_last_error": (C.c_char_p, []),
    "nsr_fir_bench_create": (_i, [_i, C.POINTER(C.c_float), _i, _i, _i64, _u64, _u64, _sz, _i, C.POINTER(_vp)]),
    "nsr_fir_bench_run": (_i, [_vp]),
    "nsr_fir_bench_runs": (_i, [_vp, _i64]),
    "nsr_fir_bench_set_batches": (_i, [_vp, _i64]),
    "nsr_fir_bench_set_timing_stride": (_i, [_vp, _i]),
    "nsr_fir_bench_stats": (_i, [_vp, C.POINTER(_d), C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_i)]),
    "nsr_fir_bench_kernel": (C.c_char_p, [_vp]),
    "nsr_fir_bench_tail": (_i, [_vp, _i64, C.POINTER(C.c_float)]),
    "nsr_fir_bench_destroy": (_i, [_vp]),
    "nsr_c5_create": (_i, [_i, _i, _i, C.POINTER(C.c_float), _i, _i, _i64, _u64, _u64, C.c_char_p, _u64,
                           C.c_char_p, _sz, C.POINTER(_vp)]),
    "nsr_c5_run": (_i, [_vp]),
    "nsr_c5_transport": (_i, [_vp, C.c_char_p, _i]),
    "nsr_c5_tail": (_i, [_vp, _i64, C.POINTER(C.c_float)]),
    "nsr_c5_destroy": (_i, [_vp]),
    "nsr_cpu_fir_run": (_i, [C.POINTER(C.c_float), _i, C.POINTER(C.c_float), _i64, _i64, _sz, C.POINTER(_d),
                             C.POINTER(_i)]),
    "nsr_rccl_library": (_i, [C.c_char_p, _i]),
    "nsr_rccl_self_test": (_i, [_i, _vp, _vp, _sz, _vp, _i]),
    "nsr_chain_bench_create": (_i, [_i, _i, C.POINTER(C.c_float), _i, _i, _i64, _u64, _u64, _sz, C.POINTER(_vp)]),
    "nsr_chain_bench_run": (_i, [_vp]),
    "nsr_chain_bench_set_batches": (_i, [_vp, _i64]),
    "nsr_chain_bench_stats": (_i, [_vp, C.POINTER(_d), C.POINTER(_u64), C.POINTER(_u64), C.c_char_p, _i,
                                   C.POINTER(_i)]),
    "nsr_chain_bench_tail": (_i, [_vp, _i64, C.POINTER(C.c_float)]),
    "nsr_chain_bench_destroy": (_i, [_vp]),
    "nsr_c1_run": (_i, [_i64, _sz, C.POINTER(_d), C.POINTER(_i)]),
    "nsr_cpu_fir_work_only": (_i, [C.POINTER(C.c_float), _i, C.POINTER(C.c_float), _i64, _i64, _i, C.POINTER(_d),
                                   C.c_char_p, _i]),
}

CHAIN_MUL_CONST_CC, CHAIN_CHANNELIZER, CHAIN_FIR = 1, 2, 3


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        nsh.lib()  # libnsh_hip.so first (RTLD_GLOBAL)
        if not os.path.exists(RT_LIB):
            raise nsh.NshError(f"{RT_LIB} is missing: run `make runtime` (or __graft_entry__.build())")
        L = C.CDLL(RT_LIB, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        raise nsh.NshError(f"{what} failed: {lib().nsr_last_error().decode(errors='replace')}")


def _f32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


class FirBench:
    """C3 measurement flowgraph (see nsr_fir_bench_create)."""

    def __init__(self, taps, n, device=0, algo=nsh.FIR_AUTO, first_index=0, seed=0x6E736368,
                 out_buf_bytes=256 << 20, timing=True):
        t = np.ascontiguousarray(np.asarray(taps, np.float32))
        self.ntaps, self.n = int(t.size), int(n)
        h = C.c_void_p()
        check(lib().nsr_fir_bench_create(device, _f32p(t), self.ntaps, algo, self.n, first_index, seed,
                                         out_buf_bytes, 1 if timing else 0, C.byref(h)), "nsr_fir_bench_create")
        self._h = h

    def set_timing_stride(self, stride: int):
        """Time every stride-th FIR launch (HIP events recorded by the launch itself)."""
        check(lib().nsr_fir_bench_set_timing_stride(self._h, int(stride)), "nsr_fir_bench_set_timing_stride")

    def set_batches(self, batches: int):
        """n-sample batches per run (one continuous stream of batches * n samples per run)."""
        check(lib().nsr_fir_bench_set_batches(self._h, int(batches)), "nsr_fir_bench_set_batches")

    def run(self, count: int = 1):
        """count back-to-back flowgraph runs (fg->run() each; a loop in C for count > 1: no
        Python between runs)."""
        if count == 1:
            check(lib().nsr_fir_bench_run(self._h), "nsr_fir_bench_run")
        else:
            check(lib().nsr_fir_bench_runs(self._h, int(count)), "nsr_fir_bench_runs")

    def stats(self):
        ms, la, sa, al = C.c_double(), C.c_uint64(), C.c_uint64(), C.c_int()
        check(lib().nsr_fir_bench_stats(self._h, C.byref(ms), C.byref(la), C.byref(sa), C.byref(al)),
              "nsr_fir_bench_stats")
        return {"kernel_ms": ms.value, "launches": la.value, "samples": sa.value, "algo": al.value,
                "kernel": lib().nsr_fir_bench_kernel(self._h).decode()}

    def tail(self, count):
        out = np.empty(count, np.complex64)
        check(lib().nsr_fir_bench_tail(self._h, count, _f32p(out.view(np.float32))), "nsr_fir_bench_tail")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().nsr_fir_bench_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ChainBench:
    """Measurement flowgraph of another single-GPU BASELINE config (see nsr_chain_bench_create):
    kind CHAIN_MUL_CONST_CC (params: complex constants), CHAIN_CHANNELIZER (params: 1024 complex
    weights), CHAIN_FIR (params: taps, with decim)."""

    def __init__(self, kind, params, n, device=0, decim=1, first_index=0, seed=0x6E736368, out_buf_bytes=256 << 20):
        if kind == CHAIN_FIR:
            p = np.ascontiguousarray(np.asarray(params, np.float32))
        else:
            p = np.ascontiguousarray(np.asarray(params, np.complex64)).view(np.float32)
        self.n = int(n)
        h = C.c_void_p()
        check(lib().nsr_chain_bench_create(device, kind, _f32p(p), int(p.size), int(decim), self.n, first_index, seed,
                                           out_buf_bytes, C.byref(h)), "nsr_chain_bench_create")
        self._h = h

    def set_batches(self, batches: int):
        check(lib().nsr_chain_bench_set_batches(self._h, int(batches)), "nsr_chain_bench_set_batches")

    def run(self):
        check(lib().nsr_chain_bench_run(self._h), "nsr_chain_bench_run")

    def stats(self):
        ms, la, sa, nb = C.c_double(), C.c_uint64(), C.c_uint64(), C.c_int()
        buf = C.create_string_buffer(256)
        check(lib().nsr_chain_bench_stats(self._h, C.byref(ms), C.byref(la), C.byref(sa), buf, 256, C.byref(nb)),
              "nsr_chain_bench_stats")
        return {"kernel_ms": ms.value, "launches": la.value, "samples": sa.value, "block": buf.value.decode(),
                "launching_blocks": nb.value}

    def tail(self, count):
        out = np.empty(count, np.complex64)
        check(lib().nsr_chain_bench_tail(self._h, count, _f32p(out.view(np.float32))), "nsr_chain_bench_tail")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().nsr_chain_bench_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def c1_run(n=1 << 20, fixed_buf_size=32768):
    """(seconds, threads) of one C1 run: null_source -> head(n) -> copy -> null_sink on scheduler_mt."""
    s, th = C.c_double(), C.c_int()
    check(lib().nsr_c1_run(int(n), fixed_buf_size, C.byref(s), C.byref(th)), "nsr_c1_run")
    return s.value, th.value


class C5Pipeline:
    """One process's share of the C5 decimating pipeline (see nsr_c5_create). Every process of
    one pipeline passes the same rendezvous_dir (a fresh directory on this node) and nonce."""

    def __init__(self, taps, n, group=0, n_groups=1, device=0, decim=2, first_index=0, seed=0x6E736368,
                 rendezvous_dir="", nonce=0, transport="auto", buf_bytes=64 << 20):
        t = np.ascontiguousarray(np.asarray(taps, np.float32))
        h = C.c_void_p()
        check(lib().nsr_c5_create(group, n_groups, device, _f32p(t), int(t.size), decim, int(n), first_index, seed,
                                  rendezvous_dir.encode(), int(nonce), transport.encode(), buf_bytes, C.byref(h)),
              "nsr_c5_create")
        self._h = h
        self.last = group == n_groups - 1

    def run(self):
        check(lib().nsr_c5_run(self._h), "nsr_c5_run")

    def transport(self):
        buf = C.create_string_buffer(512)
        check(lib().nsr_c5_transport(self._h, buf, 512), "nsr_c5_transport")
        return buf.value.decode()

    def tail(self, count):
        out = np.empty(count, np.complex64)
        check(lib().nsr_c5_tail(self._h, count, _f32p(out.view(np.float32))), "nsr_c5_tail")
        return out

    def close(self):
        if getattr(self, "_h", None):
            lib().nsr_c5_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cpu_fir_run(taps, x, n, fixed_buf_size=32768, with_threads=False):
    """Seconds of the CPU scheduler_mt FIR run (and the threads it used, with_threads=True)."""
    t = np.ascontiguousarray(np.asarray(taps, np.float32))
    xv = np.ascontiguousarray(np.asarray(x, np.complex64))
    s = C.c_double()
    th = C.c_int()
    check(lib().nsr_cpu_fir_run(_f32p(t), t.size, _f32p(xv.view(np.float32)), xv.size, int(n), fixed_buf_size,
                                C.byref(s), C.byref(th)), "nsr_cpu_fir_run")
    return (s.value, th.value) if with_threads else s.value


def cpu_fir_work_only(taps, x, n, chunk=4096):
    """(seconds, isa) of n FIR outputs in chunk-sample filter() calls, no scheduler."""
    t = np.ascontiguousarray(np.asarray(taps, np.float32))
    xv = np.ascontiguousarray(np.asarray(x, np.complex64))
    s = C.c_double()
    buf = C.create_string_buffer(64)
    check(lib().nsr_cpu_fir_work_only(_f32p(t), t.size, _f32p(xv.view(np.float32)), xv.size, int(n), int(chunk),
                                      C.byref(s), buf, 64), "nsr_cpu_fir_work_only")
    return s.value, buf.value.decode()


def rccl_library() -> str:
    """The librccl file this process's rccl crossings bound ("" if none)."""
    buf = C.create_string_buffer(1024)
    check(lib().nsr_rccl_library(buf, 1024), "nsr_rccl_library")
    return buf.value.decode()


def rccl_self_test(device, src_ptr, dst_ptr, nbytes, stream_ptr, peer=0):
    """One-process send/recv to self through the rccl transport's library table (see
    nsr_rccl_self_test); raises NshError with RCCL's text on any failure."""
    check(lib().nsr_rccl_self_test(int(device), C.c_void_p(src_ptr), C.c_void_p(dst_ptr), int(nbytes),
                                   C.c_void_p(stream_ptr), int(peer)), "nsr_rccl_self_test")
