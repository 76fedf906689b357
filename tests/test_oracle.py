"""CPU: pin the oracle (oracle/nsh_oracle.c) against the golden fixtures and the
reference's own test vectors before anything is checked against it."""
import hashlib
import json
import os

import numpy as np

from oracle import oracle as orc
from tests.conftest import GOLDEN


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def test_synth_matches_manifest_and_numpy():
    m = manifest()
    x = orc.synth(8)
    np.testing.assert_array_equal(x, np.array([complex(a, b) for a, b in m["synth_prefix"]], np.complex64))
    # values lie on the 24-bit grid in [-1, 1)
    y = orc.synth(1 << 16, first_index=12345)
    v = np.concatenate([y.real, y.imag]).astype(np.float64)
    assert v.min() >= -1.0 and v.max() < 1.0
    assert np.all((v + 1.0) * 8388608.0 == np.round((v + 1.0) * 8388608.0))


def test_synth_segments_concatenate():
    a = orc.synth(1000)
    b = orc.synth(500, first_index=1000)
    np.testing.assert_array_equal(np.concatenate([a, b]), orc.synth(1500))


def test_fir_oracle_vs_lfilter(golden):
    g = golden("fir127.npz")
    y = orc.fir_ccf(g["x"], g["taps"])
    ok, err, scale = orc.tol_ok(y, g["y"])
    assert ok, (err, scale)
    assert err <= 1e-7 * scale  # double accumulation: agrees with lfilter to fp32 rounding


def test_fir_oracle_history_across_calls(golden):
    g = golden("fir127.npz")
    _, hist = orc.fir_ccf(g["x"], g["taps"], return_hist=True)
    y2 = orc.fir_ccf(g["x_next"], g["taps"], hist=hist)
    ok, err, scale = orc.tol_ok(y2, g["y_next"])
    assert ok, (err, scale)


def test_fir_oracle_decim(golden):
    g = golden("fir127_decim2.npz")
    y = orc.fir_ccf(g["x"], g["taps"], decim=2)
    ok, err, scale = orc.tol_ok(y, g["y"])
    assert ok, (err, scale)
    z = g["x"]
    for _ in range(4):
        z = orc.fir_ccf(z, g["taps"], decim=2)
    ok, err, scale = orc.tol_ok(z, g["y_chain4"])
    assert ok, (err, scale)


def test_fir_oracle_chunking_invariant():
    h = np.linspace(-0.3, 0.5, 37).astype(np.float32)
    x = orc.synth(3000)
    y_all = orc.fir_ccf(x, h)
    hist = np.zeros(36, np.complex64)
    parts = []
    for a, b in [(0, 1), (1, 40), (40, 41), (41, 1000), (1000, 3000)]:
        yp, hist = orc.fir_ccf(x[a:b], h, hist=hist, return_hist=True)
        parts.append(yp)
    np.testing.assert_array_equal(np.concatenate(parts), y_all)


def test_mulchain_oracle(golden):
    g = golden("mulchain4.npz")
    y = orc.mul_const_chain_cc(g["x"], list(g["k"]))
    np.testing.assert_array_equal(y, g["y"])  # per-stage fp32 products: bit-exact


def test_fft_oracle(golden):
    g = golden("fft1024.npz")
    ok, err, scale = orc.tol_ok(orc.fft1024(g["x"]), g["X"])
    assert ok, (err, scale)
    ok, err, scale = orc.tol_ok(orc.fft1024(g["x"], inverse=True), g["Xi"])
    assert ok, (err, scale)
    ok, err, scale = orc.tol_ok(orc.channelizer1024(g["x"], g["w"]), g["y_chan"])
    assert ok, (err, scale)


def test_reference_vectors_identity():
    """BlockFanout / BasicBlockGrouping (k = 1.0) and CudaCopy are exact identities."""
    m = manifest()["reference_vectors"]
    n = 1_000_000
    fan = (2 * np.arange(n) + 1j * (2 * np.arange(n) + 1)).astype(np.complex64)
    assert hashlib.sha256(fan.tobytes()).hexdigest() == m["BlockFanout"]["sha256"]
    np.testing.assert_array_equal(orc.mul_const_cc(fan, 1.0 + 0.0j), fan)
    cuda = (np.arange(102_400) - 1j * np.arange(102_400)).astype(np.complex64)
    assert hashlib.sha256(cuda.tobytes()).hexdigest() == m["CudaCopy"]["sha256"]
    out = np.empty_like(cuda)
    orc._load().orc_copy(orc._p(cuda), orc._p(out), cuda.nbytes)
    np.testing.assert_array_equal(out, cuda)


def test_add_mul_cc_oracle():
    a, b = orc.synth(1000), orc.synth(1000, first_index=7777)
    np.testing.assert_allclose(orc.add_cc(a, b), a + b, rtol=0, atol=0)
    p = orc.mul_cc(a, b)
    np.testing.assert_allclose(p, (a.astype(np.complex128) * b).astype(np.complex64), rtol=1e-6, atol=1e-7)
