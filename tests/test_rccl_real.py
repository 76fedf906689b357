"""The real librccl behind domain_adapter_remote's rccl transport, run on the box's one GPU.

The cross-GPU edge binds librccl by dlopen / dlsym (runtime/lib/domain_adapter_remote.cpp,
rccl_transport::lib) and so far met only the test double (tests/cpp/fake_rccl.hip). Here the
same table, with nothing substituted, runs a 1-rank communicator and a grouped ncclSend + ncclRecv
to self (domain_adapter_remote::rccl_self_test, nsr_rccl_self_test): the ncclUniqueId size, the
ncclCommInitRank argument order, ncclInt8 = 0 and the async-error query all meet the real library
before a multi-GPU run depends on them. The crossing this backs replaces the reference's in-process
buffer hand-off (/root/reference/runtime/include/gnuradio/domain_adapter_direct.hpp:156-172).

Each case runs in a child process under a time limit: a communicator that hangs must fail the
test, not the session."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

CHILD = r"""
import json, sys
import torch
sys.path.insert(0, %(root)r)
from newsched_amd import nsh, nsr
torch.cuda.set_device(0)
out = {}
n = %(nbytes)d
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
y = torch.zeros_like(x)
s = torch.cuda.Stream()
torch.cuda.synchronize()
out["ptr_dev_x"] = nsh.pointer_device(x.data_ptr())
case = %(case)r
try:
    if case == "self":
        nsr.rccl_self_test(0, x.data_ptr(), y.data_ptr(), n, s.cuda_stream)
        torch.cuda.synchronize()
        out["bit_exact"] = bool(torch.equal(x, y))
    elif case == "ring":
        # the crossings send from / land in hip_buffer rings: HIP-VMM memory mapped twice
        import ctypes as C
        L = nsh.lib()
        bases = []
        for _ in range(2):
            b, act, dm = C.c_void_p(), C.c_size_t(), C.c_int()
            nsh.check(L.nsh_ring_alloc(0, n, C.byref(b), C.byref(act), C.byref(dm)), "ring")
            bases.append((b.value, act.value, dm.value))
        out["ring_double_mapped"] = [r[2] for r in bases]
        out["ptr_dev_ring"] = [nsh.pointer_device(r[0]) for r in bases]
        # a span that crosses the wrap point of the source ring (read through its second mapping)
        src = bases[0][0] + bases[0][1] - n // 2
        nsh.check(L.nsh_memcpy_async(C.c_void_p(src), C.c_void_p(x.data_ptr()), n, nsh.NSH_D2D,
                                     C.c_void_p(s.cuda_stream)), "fill")
        s.synchronize()
        nsr.rccl_self_test(0, src, bases[1][0], n, s.cuda_stream)
        nsh.check(L.nsh_memcpy_async(C.c_void_p(y.data_ptr()), C.c_void_p(bases[1][0]), n, nsh.NSH_D2D,
                                     C.c_void_p(s.cuda_stream)), "read back")
        s.synchronize()
        out["bit_exact"] = bool(torch.equal(x, y))
        for r in bases:
            nsh.check(L.nsh_ring_free(C.c_void_p(r[0])), "ring free")
    elif case == "host_ptr":
        import numpy as np
        h = np.zeros(n, np.uint8)  # pageable host memory: refused before any RCCL call
        nsr.rccl_self_test(0, x.data_ptr(), h.ctypes.data, n, s.cuda_stream)
    elif case == "bad_peer":
        nsr.rccl_self_test(0, x.data_ptr(), y.data_ptr(), n, s.cuda_stream, peer=1)  # a 1-rank communicator
    out["error"] = None
except Exception as e:
    out["error"] = str(e)
out["library"] = nsr.rccl_library()
torch.cuda.synchronize()
print("RESULT " + json.dumps(out), flush=True)
"""


def run_case(case, nbytes=64 << 20, timeout=150):
    env = dict(os.environ)
    for k in ("NSH_RCCL_LIB", "NSH_REMOTE_TEST_RCCL"):
        env.pop(k, None)  # the real library, nothing substituted
    env.setdefault("NCCL_DEBUG", "WARN")
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "nbytes": nbytes, "case": case}], cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout, env=env)
    lines = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    assert p.returncode == 0 and lines, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    r = json.loads(lines[-1][7:])
    print(case, r)
    return r


@pytest.mark.gpu
def test_real_rccl_self_send_recv_bit_exact(torch_cuda):
    """64 MiB through a 1-rank communicator of the real librccl, send and receive to self in one
    group on a side stream: bit-exact, and the library bound is torch's already-loaded copy
    (RTLD_NOLOAD of soname librccl.so.1) or /opt/rocm's -- never the test double."""
    r = run_case("self")
    assert r["error"] is None, r
    assert r["bit_exact"], r
    assert r["ptr_dev_x"] == 0, r
    assert "librccl" in r["library"] and "fake" not in r["library"], r


@pytest.mark.gpu
def test_real_rccl_self_send_recv_vmm_rings(torch_cuda):
    """The same through the memory a crossing really moves: hip_buffer rings (one VMM allocation
    mapped twice), the source span straddling the ring's wrap point. Bit-exact."""
    r = run_case("ring")
    assert r["error"] is None, r
    assert r["bit_exact"], r


@pytest.mark.gpu
def test_real_rccl_wrong_pointer_is_an_error(torch_cuda):
    """A pageable host pointer where device memory belongs: a thrown error naming the buffer,
    raised before any RCCL call (no kernel touches it, so no GPU fault and no hang)."""
    r = run_case("host_ptr", nbytes=1 << 20)
    assert r["error"] and "not device memory" in r["error"], r


@pytest.mark.gpu
def test_real_rccl_own_error_codes_surface(torch_cuda):
    """An argument RCCL itself refuses (peer 1 in a 1-rank communicator): its return code reaches
    the caller as an exception carrying ncclGetErrorString's text, and the process stays healthy."""
    r = run_case("bad_peer", nbytes=1 << 20)
    assert r["error"] and "rccl_self_test" in r["error"], r
