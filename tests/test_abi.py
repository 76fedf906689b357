"""CPU: the C-ABI libraries build, load, and export every symbol their headers declare
(no compute calls -- there is no GPU in the build container)."""
import ctypes
import os
import shutil
import re
import subprocess

import pytest

from tests.conftest import ROOT


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nsh_\w+|nsr_\w+)\s*\(", txt)))


def exported(so):
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_hip_shim_exports_header():
    from newsched_amd import nsh

    syms = exported(nsh.HIP_LIB)
    missing = [s for s in declared("nsh_hip.h") if s not in syms]
    assert not missing, missing
    # the Python binding covers exactly the header
    assert sorted(nsh.SIGNATURES) == declared("nsh_hip.h")


def test_hip_shim_loads_and_reports():
    from newsched_amd import nsh

    L = nsh.lib()
    assert L.nsh_abi_version() == 1
    assert L.nsh_last_error() == b""


def test_hip_shim_is_gfx950_code_object(tmp_path):
    from newsched_amd import nsh

    # --offloading extracts the bundled code objects next to its input: run it on a copy
    lib = tmp_path / os.path.basename(nsh.HIP_LIB)
    shutil.copyfile(nsh.HIP_LIB, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_hip_shim_rejects_null_arguments_before_launch():
    """Argument errors come back as codes with a message, before any HIP call (so they are
    checkable here, without a GPU): a NULL plan to the FIR entry points."""
    from newsched_amd import nsh

    L = nsh.lib()
    one = ctypes.c_void_p(1)
    assert L.nsh_fir_ccf(None, one, None, one, one, 16, None) != 0
    assert b"null plan" in L.nsh_last_error()
    assert L.nsh_fir_cascade_ccf(None, one, None, one, one, 16, None) != 0
    assert b"null plan" in L.nsh_last_error()
    assert L.nsh_fir_plan_algo(None) == 0
    assert L.nsh_fir_ccf(None, one, None, one, one, 0, None) != 0  # plan checked first


def test_stream_and_fft_entry_points_reject_null():
    from newsched_amd import nsh

    L = nsh.lib()
    one = ctypes.c_void_p(16)
    assert L.nsh_copy(None, one, 64, None) != 0 and b"null" in L.nsh_last_error()
    assert L.nsh_mul_const_cc(one, None, 8, 1.0, 0.0, None) != 0
    assert L.nsh_add_cc(one, None, one, 8, None) != 0
    assert L.nsh_fft1024_c2c(None, one, 1, 0, None) != 0
    assert L.nsh_channelizer1024(one, ctypes.c_void_p(32), None, 1, None) != 0
    assert L.nsh_synth_cf32(None, 8, 0, 1, None) != 0
    assert L.nsh_copy(None, None, 0, None) == 0  # nothing to move: no error
