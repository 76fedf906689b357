"""GPU parity: each kernel of libnsh_hip.so, called through the C-ABI, against the CPU
oracle on the same seeded inputs, plus golden fixtures and size-independent properties.

Tolerances: bit-exact for copy / identity multiplies / per-stage-rounded complex
products (same formula, no FMA); FIR and FFT within the north-star 1e-5 relative bound
(norm-wise max|dy| <= 1e-5 max|y_ref| and per element, oracle.tol_ok)."""
import os

import numpy as np
import pytest

from oracle import oracle as orc
from newsched_amd import nsh

pytestmark = pytest.mark.gpu


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


def test_synth_bit_exact(torch_cuda):
    torch = torch_cuda
    for n, first in [(1, 0), (1000, 0), (4097, 123456789)]:
        y = torch.empty(n, dtype=torch.complex64, device="cuda")
        nsh.synth(y, n, first)
        np.testing.assert_array_equal(host(y), orc.synth(n, first))


@pytest.mark.parametrize("nbytes", [8, 16, 24, 8 * 1023, 8 * (1 << 20) + 8])
@pytest.mark.parametrize("offset", [0, 8])
def test_copy_bit_exact(torch_cuda, nbytes, offset):
    torch = torch_cuda
    x = orc.synth(nbytes // 8 + 2)
    dx = dev(torch, x)
    dy = torch.zeros_like(dx)
    base_x = dx.data_ptr() + offset
    base_y = dy.data_ptr() + offset
    nsh.copy(base_x, base_y, nbytes)
    y = host(dy)
    o = offset // 8
    np.testing.assert_array_equal(y[o:o + nbytes // 8], x[o:o + nbytes // 8])
    assert np.all(y[:o] == 0) and np.all(y[o + nbytes // 8:] == 0)


def test_mul_const_identity_reference_vector(torch_cuda):
    """BlockFanout vector (qa_scheduler_mt.cpp:79-135): x=(2i,2i+1), k=1 -> identity."""
    torch = torch_cuda
    n = 1_000_000
    x = (2 * np.arange(n) + 1j * (2 * np.arange(n) + 1)).astype(np.complex64)
    dx = dev(torch, x)
    dy = torch.empty_like(dx)
    nsh.mul_const_cc(dx, dy, n, 1.0 + 0.0j)
    np.testing.assert_array_equal(host(dy), x)


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 262145])
@pytest.mark.parametrize("k", [0.5 - 0.25j, complex(np.exp(0.3j))])
def test_mul_const_cc_bit_exact(torch_cuda, n, k):
    torch = torch_cuda
    x = orc.synth(n, 99)
    dx = dev(torch, x)
    dy = torch.empty_like(dx)
    nsh.mul_const_cc(dx, dy, n, k)
    np.testing.assert_array_equal(host(dy), orc.mul_const_cc(x, np.complex64(k)))


def test_mul_const_cc_unaligned(torch_cuda):
    torch = torch_cuda
    n = 5001
    x = orc.synth(n + 1)
    dx = dev(torch, x)
    dy = torch.zeros_like(dx)
    nsh.mul_const_cc(dx.data_ptr() + 8, dy.data_ptr() + 8, n, 0.25 + 2j)
    np.testing.assert_array_equal(host(dy)[1:], orc.mul_const_cc(x[1:], np.complex64(0.25 + 2j)))


def test_mul_const_ff_bit_exact(torch_cuda):
    torch = torch_cuda
    x = orc.synth(4099).view(np.float32)
    dx = dev(torch, x)
    dy = torch.empty_like(dx)
    nsh.mul_const_ff(dx, dy, x.size, 1.7)
    np.testing.assert_array_equal(host(dy), orc.mul_const_ff(x, 1.7))


def test_mul_chain_golden(torch_cuda, golden):
    torch = torch_cuda
    g = golden("mulchain4.npz")
    dx = dev(torch, g["x"])
    dy = torch.empty_like(dx)
    nsh.mul_const_chain_cc(dx, dy, g["x"].size, list(g["k"]))
    np.testing.assert_array_equal(host(dy), g["y"])
    for m in (1, 2, 3, 7):
        ks = [complex(np.exp(0.1j * (i + 1))) for i in range(m)]
        nsh.mul_const_chain_cc(dx, dy, g["x"].size, ks)
        np.testing.assert_array_equal(host(dy), orc.mul_const_chain_cc(g["x"], [np.complex64(k) for k in ks]))


@pytest.mark.parametrize("n", [1, 777, 1 << 18])
def test_add_mul_cc_bit_exact(torch_cuda, n):
    torch = torch_cuda
    a, b = orc.synth(n, 1), orc.synth(n, 10 ** 6)
    da, db = dev(torch, a), dev(torch, b)
    dy = torch.empty_like(da)
    nsh.add_cc(da, db, dy, n)
    np.testing.assert_array_equal(host(dy), orc.add_cc(a, b))
    nsh.mul_cc(da, db, dy, n)
    np.testing.assert_array_equal(host(dy), orc.mul_cc(a, b))


@pytest.mark.parametrize("oa,ob,oy", [(1, 0, 0), (0, 1, 1), (1, 1, 0), (3, 2, 1)])
def test_add_mul_cc_mixed_alignment(torch_cuda, oa, ob, oy):
    """add_cc / multiply_cc / the 4-stage chain with each operand at its own sample offset (8-B
    but not 16-B aligned where odd), as two edges' read pointers and a write pointer of a flowgraph
    are; bit-exact against the oracle, guard samples around the output untouched."""
    torch = torch_cuda
    n = 12_345
    a, b = orc.synth(n, 3), orc.synth(n, 4)
    da = torch.zeros(n + 4, dtype=torch.complex64, device="cuda")
    db = torch.zeros(n + 4, dtype=torch.complex64, device="cuda")
    da[oa:oa + n] = dev(torch, a)
    db[ob:ob + n] = dev(torch, b)
    guard = complex(9.0, -9.0)
    for fn, ref in ((nsh.add_cc, orc.add_cc(a, b)), (nsh.mul_cc, orc.mul_cc(a, b))):
        dy = torch.full((n + 4,), guard, dtype=torch.complex64, device="cuda")
        fn(da.data_ptr() + 8 * oa, db.data_ptr() + 8 * ob, dy.data_ptr() + 8 * oy, n)
        y = host(dy)
        np.testing.assert_array_equal(y[oy:oy + n], ref)
        assert np.all(y[:oy] == guard) and np.all(y[oy + n:] == guard)
    ks = [complex(np.exp(0.1j * (i + 1))) for i in range(4)]
    dy = torch.full((n + 4,), guard, dtype=torch.complex64, device="cuda")
    nsh.mul_const_chain_cc(da.data_ptr() + 8 * oa, dy.data_ptr() + 8 * oy, n, ks)
    y = host(dy)
    np.testing.assert_array_equal(y[oy:oy + n], orc.mul_const_chain_cc(a, [np.complex64(k) for k in ks]))
    assert np.all(y[:oy] == guard) and np.all(y[oy + n:] == guard)


@pytest.mark.parametrize("vlen,nitems", [(1024, 37), (1, 1000), (3, 777), (1024, 0)])
def test_mul_const_vcc_bitexact(torch_cuda, vlen, nitems):
    """multiply_const_vcc: x[i][j] * k[j], each product rounded as the oracle's mul_cc."""
    torch = torch_cuda
    x = orc.synth(max(nitems * vlen, 1), 91)[: nitems * vlen]
    k = orc.synth(vlen, 92)
    dx, dk = dev(torch, x), dev(torch, k)
    dy = torch.zeros(max(nitems * vlen, 1), dtype=torch.complex64, device="cuda")
    nsh.mul_const_vcc(dx, dy, dk, vlen, nitems)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(dy)[: nitems * vlen], orc.mul_cc(x, np.tile(k, nitems)))


# "mfma" is the default matrix-core kernel (decim 1: per-chunk scaled fp16x2, k_fir_mfma12),
# "mfma_f32" the exact-fp32 matrix form (k_fir_f32mfma)
ALGOS = [("direct", nsh.FIR_DIRECT), ("mfma", nsh.FIR_MFMA), ("mfma_f32", nsh.FIR_MFMA_F32)]
MAX_TAPS = {"direct": 4096, "mfma": 161, "mfma_f32": 257}


def make_plan(name, taps, decim, algo):
    """FirPlan for an ALGOS entry."""
    return nsh.FirPlan(taps, decim, algo)


def run_fir(torch, plan, x, n_out, hist=None):
    L = plan.ntaps
    dx = dev(torch, x)
    hin = dev(torch, hist if hist is not None else np.zeros(max(L - 1, 1), np.complex64))
    hout = torch.zeros(max(L - 1, 1), dtype=torch.complex64, device="cuda")
    dy = torch.empty(max(n_out, 1), dtype=torch.complex64, device="cuda")
    plan(dx, hin, hout, dy, n_out)
    return host(dy)[:n_out], host(hout)[: L - 1]


@pytest.mark.parametrize("name,algo", ALGOS)
@pytest.mark.parametrize("decim", [1, 2, 4])
def test_fir_null_history_reads_zeros(torch_cuda, name, algo, decim):
    """hist_in = NULL is the stream start (zeros): bit-identical to an explicit zero history,
    for every kernel form and for calls shorter than the filter."""
    torch = torch_cuda
    if name != "direct" and name != "mfma" and decim > 1:
        pytest.skip("decimation: direct and mfma forms")
    h = np.hamming(127).astype(np.float32) / 70
    plan = make_plan(name, h, decim, algo)
    for n_out in (3, 40_001):
        x = orc.synth(n_out * decim, 8)
        y0, h0 = run_fir(torch, plan, x, n_out)
        dx = dev(torch, x)
        hout = torch.zeros(126, dtype=torch.complex64, device="cuda")
        dy = torch.empty(n_out, dtype=torch.complex64, device="cuda")
        plan(dx, 0, hout, dy, n_out)
        np.testing.assert_array_equal(host(dy), y0)
        np.testing.assert_array_equal(host(hout), h0)


@pytest.mark.parametrize("name,algo", ALGOS)
def test_fir127_golden(torch_cuda, golden, name, algo):
    torch = torch_cuda
    g = golden("fir127.npz")
    plan = make_plan(name, g["taps"], 1, algo)
    assert plan.algo == algo
    if name == "mfma":
        assert plan.kernel == "k_fir_mfma12<5>", plan.kernel
    y, hist = run_fir(torch, plan, g["x"], g["x"].size)
    ok, err, scale = orc.tol_ok(y, g["y"])
    assert ok, (name, err, scale)
    np.testing.assert_array_equal(hist, g["x"][-126:])
    y2, _ = run_fir(torch, plan, g["x_next"], g["x_next"].size, hist=hist)
    ok, err, scale = orc.tol_ok(y2, g["y_next"])
    assert ok, (name, err, scale)


@pytest.mark.parametrize("name,algo", ALGOS)
@pytest.mark.parametrize("ntaps", [1, 2, 16, 17, 31, 32, 33, 64, 127, 128, 145, 161])
@pytest.mark.parametrize("n", [1, 100, 2047, 2048, 2049, 70001])
def test_fir_vs_oracle_shapes(torch_cuda, name, algo, ntaps, n):
    if ntaps > MAX_TAPS[name]:
        pytest.skip(f"{name} supports ntaps <= {MAX_TAPS[name]}")
    torch = torch_cuda
    rng = np.random.default_rng(ntaps * 1000 + n)
    h = rng.standard_normal(ntaps).astype(np.float32) * 0.1
    x = orc.synth(n, 5 + n)
    hist = orc.synth(max(ntaps - 1, 1), 10 ** 7)[: ntaps - 1]
    plan = make_plan(name, h, 1, algo)
    y, hout = run_fir(torch, plan, x, n, hist=hist if ntaps > 1 else None)
    y_ref, h_ref = orc.fir_ccf(x, h, hist=hist if ntaps > 1 else None, return_hist=True)
    ok, err, scale = orc.tol_ok(y, y_ref)
    assert ok, (name, ntaps, n, err, scale)
    np.testing.assert_array_equal(hout, h_ref)


@pytest.mark.parametrize("decim", [2, 4, 8])
def test_fir_decim_vs_oracle(torch_cuda, decim):
    torch = torch_cuda
    h = np.hanning(127).astype(np.float32) / 64
    for n_out in (1, 513, 40001):
        x = orc.synth(n_out * decim, 3)
        hist = orc.synth(126, 4 * 10 ** 6)
        plan = nsh.FirPlan(h, decim, nsh.FIR_DIRECT)
        y, hout = run_fir(torch, plan, x, n_out, hist=hist)
        y_ref, h_ref = orc.fir_ccf(x, h, decim=decim, hist=hist, return_hist=True)
        ok, err, scale = orc.tol_ok(y, y_ref)
        assert ok, (decim, n_out, err, scale)
        np.testing.assert_array_equal(hout, h_ref)


@pytest.fixture(params=["v11", "v13"])
def dec_form(request, monkeypatch):
    """The polyphase MFMA kernels (fp16x2, per-chunk scale, exact forms): k_fir_mfma11 (contiguous
    walk, exact chunks inline) and k_fir_mfma13 (lockstep walk per XCD, exact chunks queued for
    k_fir_exact13), chosen at plan creation by NSH_DEC_WALK_MASK (bit D)."""
    monkeypatch.setenv("NSH_DEC_WALK_MASK", "0" if request.param == "v11" else "20")
    return request.param


def _dec_plan(h, decim, form):
    plan = nsh.FirPlan(h, decim, nsh.FIR_MFMA)
    assert plan.algo == nsh.FIR_MFMA
    want = {"v11": "k_fir_mfma11<", "v13": "k_fir_mfma13<"}[form]
    assert plan.kernel.startswith(want), plan.kernel
    return plan


@pytest.mark.parametrize("decim", [2, 4])
@pytest.mark.parametrize("ntaps", [1, 2, 15, 16, 17, 33, 64, 127, 128, 160])
@pytest.mark.parametrize("n_out", [1, 100, 1023, 1024, 1025, 33333])
def test_fir_decim_mfma_vs_oracle(torch_cuda, dec_form, decim, ntaps, n_out):
    """Polyphase MFMA forms: every phase/halo/tail shape against the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(ntaps * 7919 + n_out * decim)
    h = rng.standard_normal(ntaps).astype(np.float32) * 0.1
    x = orc.synth(n_out * decim, 11 + n_out)
    hist = orc.synth(max(ntaps - 1, 1), 5 * 10 ** 6)[: ntaps - 1]
    plan = _dec_plan(h, decim, dec_form)
    y, hout = run_fir(torch, plan, x, n_out, hist=hist if ntaps > 1 else None)
    y_ref, h_ref = orc.fir_ccf(x, h, decim=decim, hist=hist if ntaps > 1 else None, return_hist=True)
    ok, err, scale = orc.tol_ok(y, y_ref)
    assert ok, (decim, ntaps, n_out, err, scale)
    np.testing.assert_array_equal(hout, h_ref)


def test_fir_decim_auto_picks_mfma(torch_cuda):
    h = np.hanning(127).astype(np.float32)
    assert nsh.FirPlan(h, 2).algo == nsh.FIR_MFMA
    assert nsh.FirPlan(h, 4).algo == nsh.FIR_MFMA
    assert nsh.FirPlan(h, 8).algo == nsh.FIR_PFFT
    assert nsh.FirPlan(np.ones(2100, np.float32) / 2100, 8).algo == nsh.FIR_DIRECT  # 263 overlap rows > 256


@pytest.mark.parametrize("decim", [2, 4])
def test_fir_decim_mfma_edge_values(torch_cuda, dec_form, decim):
    """inf/NaN (pattern equal to the oracle's), a 2^60 spike, segments at 1e-30 / 1e30, zero
    chunks and an fp32-subnormal sample through the polyphase kernels; each region checked on
    its own scale. The fp16x2 form sends the chunks that need it through the exact path."""
    torch = torch_cuda
    h = _firwin127()
    n_out = 30_000
    x = orc.synth(n_out * decim, 40 + decim)
    seg = len(x) // 4
    x[:seg] *= np.float32(1e-30)
    x[3 * seg:] *= np.float32(1e30)
    x[seg + 5000] = np.complex64(complex(np.inf, 0.5))
    x[seg + 9000] = np.complex64(complex(np.nan, 0.0))
    x[2 * seg + 100] *= np.float32(2.0 ** 60)
    x[2 * seg + 6000:2 * seg + 10_000] = 0
    x[2 * seg + 12_000] = np.complex64(complex(1e-40, 0.0))
    y, _ = run_fir(torch, _dec_plan(h, decim, dec_form), x, n_out)
    ref = orc.fir_ccf(x, h, decim=decim)
    _assert_nonfinite_pattern(y, ref)
    before = lambda i: (i + decim - 1) // decim  # outputs [0, before(i)) do not see input i
    after = lambda i: (i + 126) // decim + 1     # outputs from after(i) on no longer see it
    regions = [(0, before(seg)), (after(seg), before(seg + 5000)), (after(seg + 9000), before(2 * seg + 100)),
               (after(2 * seg + 100), before(3 * seg)), (after(3 * seg), n_out)]
    for a, b in regions:
        ok, err, scale = orc.tol_ok(y[a:b], ref[a:b])
        assert ok, (decim, a, b, err, scale)


@pytest.mark.parametrize("decim", [2, 4])
@pytest.mark.parametrize("period", [1, 3, 64])
def test_fir_decim_mfma_periodic_exact_chunks(torch_cuda, dec_form, decim, period):
    """Every period-th 2048-input chunk holds a 2^40 spike (its range is beyond the fp16x2 split:
    the exact-fp32 tile), every (period+1)-th a NaN, over 2^20 + 37 inputs, called twice on one
    stream with the history handed on (k_fir_mfma13's exact queue alternates its two counter sets
    per call). The NaN pattern equals the oracle's; every chunk's finite outputs meet the tolerance
    on that chunk's own scale."""
    torch = torch_cuda
    h = _firwin127()
    n = (1 << 20) + 37 * decim
    x = orc.synth(n, 77 + period)
    x[100::2048 * period] *= np.float32(2.0 ** 40)
    x[1500::2048 * (period + 1)] = complex(np.nan, 0.25)
    plan = _dec_plan(h, decim, dec_form)
    half = (n // decim // 2) * decim
    y1, hy = run_fir(torch, plan, x[:half], half // decim)
    y2, _ = run_fir(torch, plan, x[half:], (n - half) // decim, hist=hy)
    y = np.concatenate([y1, y2])
    ref = orc.fir_ccf(x[: n // decim * decim], h, decim)
    _assert_nonfinite_pattern(y, ref)
    c = 2048 // decim
    for a in range(0, y.size, c):
        yy, rr = y[a:a + c], ref[a:a + c]
        fin = np.isfinite(rr.real) & np.isfinite(rr.imag)
        if fin.any():
            ok, err, scale = orc.tol_ok(yy[fin], rr[fin])
            assert ok, (a, err, scale)


def test_fir_decim4_walks_agree_full_stream(torch_cuda, monkeypatch):
    """D = 4 over 2^26 inputs: the lockstep walk (k_fir_mfma13) and the contiguous walk
    (k_fir_mfma11) within the split's rounding of each other everywhere, and the lockstep walk
    against the oracle on windows at XCD-range and chunk boundaries."""
    torch = torch_cuda
    h = _firwin127()
    n_in = 1 << 26
    n_out = n_in // 4
    dx = torch.empty(n_in, dtype=torch.complex64, device="cuda")
    nsh.synth(dx, n_in, 0)
    ys = {}
    for form, mask in (("v11", "0"), ("v13", "16")):
        monkeypatch.setenv("NSH_DEC_WALK_MASK", mask)
        plan = _dec_plan(h, 4, form)
        hout = torch.zeros(126, dtype=torch.complex64, device="cuda")
        y = torch.empty(n_out, dtype=torch.complex64, device="cuda")
        plan(dx, 0, hout, y, n_out)
        ys[form] = y
        plan.close()
    torch.cuda.synchronize()
    d = (ys["v11"] - ys["v13"]).abs().max().item()
    scale = ys["v11"].abs().max().item()
    assert d <= 1e-6 * scale, (d, scale)
    del dx
    chunks = n_out // 512
    per_x = (chunks + 7) // 8
    for o in (0, 512 * per_x - 300, 512 * 3 * per_x + 7, n_out - 1000):
        o = max(0, min(o, n_out - 1000))
        lo = 4 * o - 126
        xw = orc.synth(4 * 1000 + 126, max(lo, 0)) if lo >= 0 else np.concatenate(
            [np.zeros(-lo, np.complex64), orc.synth(4 * 1000 + 126 + lo, 0)])
        ref = orc.fir_ccf(xw[126:], h, 4, hist=xw[:126])
        ok, err, scale = orc.tol_ok(ys["v13"][o:o + 1000].cpu().numpy(), ref)
        assert ok, (o, err, scale)


def test_fir_decim2_golden_chain(torch_cuda, golden):
    torch = torch_cuda
    g = golden("fir127_decim2.npz")
    plan = nsh.FirPlan(g["taps"], 2)
    y, _ = run_fir(torch, plan, g["x"], g["x"].size // 2)
    ok, err, scale = orc.tol_ok(y, g["y"])
    assert ok, (err, scale)
    z = g["x"]
    for _ in range(4):
        z, _ = run_fir(torch, plan, z, z.size // 2)
    ok, err, scale = orc.tol_ok(z, g["y_chain4"])
    assert ok, (err, scale)


@pytest.mark.parametrize("name,algo", ALGOS)
def test_fir_chunked_stream_equals_one_shot(torch_cuda, name, algo):
    """Call-splitting invariance: the history hand-off makes any chunking exact for the
    direct form (tap order is position independent). The MFMA form sums each output in an
    order set by its phase within the call's 32-sample blocks, so chunking changes the
    rounding: equal within the 1e-5 bound, not bitwise."""
    torch = torch_cuda
    h = np.hamming(127).astype(np.float32) / 70
    x = orc.synth(300_000, 42)
    plan = make_plan(name, h, 1, algo)
    y_all, _ = run_fir(torch, plan, x, x.size)
    hist = np.zeros(126, np.complex64)
    parts = []
    for a, b in [(0, 5), (5, 4101), (4101, 4102), (4102, 150_000), (150_000, 300_000)]:
        yp, hist = run_fir(torch, plan, x[a:b], b - a, hist=hist)
        parts.append(yp)
    if algo == nsh.FIR_DIRECT:
        np.testing.assert_array_equal(np.concatenate(parts), y_all)
    else:
        ok, err, scale = orc.tol_ok(np.concatenate(parts), y_all)
        assert ok and err <= 1e-6 * scale, (err, scale)


@pytest.mark.parametrize("algo,decim,ntaps", [(nsh.FIR_DIRECT, 1, 127), (nsh.FIR_MFMA, 1, 127), (nsh.FIR_MFMA, 2, 127),
                                               (nsh.FIR_MFMA, 4, 127), (nsh.FIR_MFMA_F32, 1, 127), (nsh.FIR_AUTO, 8, 127),
                                               (nsh.FIR_AUTO, 16, 511), (nsh.FIR_MFMA, 1, 31)])
def test_fir_odd_sample_offsets(torch_cuda, algo, decim, ntaps):
    """Buffers as a flowgraph hands them over: hip_buffer read/write pointers advance by any item
    count, so a work() call's input, output and history pointers are 8-byte (one complex sample)
    but not 16-byte aligned as often as not. Every FIR form (16-B buffer loads, 8-B stores) over
    pointers at odd sample offsets into larger allocations, three calls with the history handed
    on, against the oracle; the guard samples around the output stay untouched."""
    torch = torch_cuda
    h = (np.hanning(ntaps + 2)[1:-1] / (ntaps / 2)).astype(np.float32)
    plan = nsh.FirPlan(h, decim, algo)
    sizes = [1, 2049, 70_001]  # outputs per call
    n_in = sum(sizes) * decim
    x = orc.synth(n_in, 7)
    dx = torch.zeros(n_in + 3, dtype=torch.complex64, device="cuda")
    dx[1:1 + n_in] = dev(torch, x)
    guard = complex(123.0, -77.0)
    dy = torch.full((sum(sizes) + 3,), guard, dtype=torch.complex64, device="cuda")
    hl = max(plan.ntaps - 1, 1)
    hs = [torch.zeros(hl + 1, dtype=torch.complex64, device="cuda") for _ in range(2)]
    pos, cur = 0, 0
    for i, m in enumerate(sizes):
        plan(dx[1 + pos * decim:], 0 if i == 0 else hs[cur][1:], hs[cur ^ 1][1:], dy[1 + pos:], m)
        cur ^= 1
        pos += m
    y = host(dy)
    assert y[0] == guard and np.all(y[1 + pos:] == guard)
    ok, err, scale = orc.tol_ok(y[1:1 + pos], orc.fir_ccf(x, h, decim))
    assert ok, (err, scale)


@pytest.mark.parametrize("name,algo", ALGOS)
def test_fir_linearity_large(torch_cuda, name, algo):
    """Size-independent property at 2^24 samples: FIR(a x1 + x2) == a FIR(x1) + FIR(x2)
    within fp32 rounding, and a windowed oracle check at the start, middle and end."""
    torch = torch_cuda
    n = 1 << 24
    h = np.asarray(__import__("scipy.signal", fromlist=["firwin"]).firwin(127, 0.2), np.float32)
    plan = make_plan(name, h, 1, algo)
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, 0)
    hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
    hout = torch.zeros_like(hin)
    y = torch.empty_like(x)
    plan(x, hin, hout, y, n)
    torch.cuda.synchronize()
    xs = x.cpu().numpy()
    ys = y.cpu().numpy()
    for a in (0, n // 2 - 5000, n - 10000):
        ref = orc.fir_ccf(xs[a:a + 10000], h, hist=xs[a - 126:a] if a > 0 else None)
        ok, err, scale = orc.tol_ok(ys[a:a + 10000], ref)
        assert ok, (name, a, err, scale)
    x2 = torch.empty_like(x)
    nsh.synth(x2, n, 1 << 30)
    y2 = torch.empty_like(x)
    plan(x2, hin, hout, y2, n)
    x3 = (0.5 * x + x2).contiguous()
    y3 = torch.empty_like(x)
    plan(x3, hin, hout, y3, n)
    torch.cuda.synchronize()
    lin = (0.5 * y + y2 - y3).abs().max().item()
    scale = y3.abs().max().item()
    assert lin <= 2e-6 * scale, (lin, scale)


def _firwin127():
    return np.asarray(__import__("scipy.signal", fromlist=["firwin"]).firwin(127, 0.2), np.float32)


def _assert_nonfinite_pattern(y, ref):
    for f in (np.isnan, np.isinf):
        for part in (np.real, np.imag):
            bad = np.nonzero(f(part(y)) != f(part(ref)))[0]
            assert bad.size == 0, (f.__name__, part.__name__, bad.size, bad[:8].tolist(), bad[-8:].tolist(),
                                   y[bad[:4]].tolist(), ref[bad[:4]].tolist())
    inf = np.isinf(y.real)
    np.testing.assert_array_equal(np.sign(y.real[inf]), np.sign(ref.real[inf]))
    inf = np.isinf(y.imag)
    np.testing.assert_array_equal(np.sign(y.imag[inf]), np.sign(ref.imag[inf]))


@pytest.fixture
def v8_form():
    """The decim-1 fp16x2 kernel: k_fir_mfma12 (one chunk per workgroup)."""
    return "v12"


def _v8_plan(h, form):
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    assert plan.kernel == "k_fir_mfma12<5>", plan.kernel
    return plan


def test_fir_mfma_nonfinite_inputs(torch_cuda, v8_form):
    """The fp16x2 kernels send chunks holding inf/NaN (and their successors, whose halo and scale
    include them) through the fp32 direct form in the same launch: the inf/NaN pattern of
    every output equals the oracle's (IEEE double), and finite outputs meet the tolerance."""
    torch = torch_cuda
    h = _firwin127()
    x = orc.synth(50_000, 9)
    x[1000] = np.complex64(complex(np.inf, 0.5))
    x[20_000] = np.complex64(complex(np.nan, 0.0))
    x[30_000] = np.complex64(complex(0.25, -np.inf))
    x[30_050] = np.complex64(complex(-np.inf, np.inf))
    y, _ = run_fir(torch, _v8_plan(h, v8_form), x, x.size)
    ref = orc.fir_ccf(x, h)
    _assert_nonfinite_pattern(y, ref)
    fin = np.isfinite(ref.real) & np.isfinite(ref.imag)
    ok, err, scale = orc.tol_ok(y[fin], ref[fin])
    assert ok, (err, scale)


def test_fir_mfma_wide_dynamic_range(torch_cuda, v8_form):
    """One sample 2^60 above the rest: the samples sharing its chunk (and the next one)
    would flush to zero in fp16 at the spike's scale, so those chunks take the exact path.
    Outputs away from the spike are checked against the oracle on their own scale."""
    torch = torch_cuda
    h = _firwin127()
    x = orc.synth(40_000, 21)
    x[10_000] *= np.float32(2.0 ** 60)
    y, _ = run_fir(torch, _v8_plan(h, v8_form), x, x.size)
    ref = orc.fir_ccf(x, h)
    for a, b in ((0, 10_000), (10_000, 10_127), (10_127, 40_000)):
        ok, err, scale = orc.tol_ok(y[a:b], ref[a:b])
        assert ok, (a, b, err, scale)


@pytest.mark.parametrize("decim", [1, 2, 4])
@pytest.mark.parametrize("ntaps", [127, 64, 9])
@pytest.mark.parametrize("kind", ["spike", "nan"])
def test_fir_mfma_exact_paths(torch_cuda, v8_form, ntaps, decim, kind):
    """Every 2048-sample chunk outside the fp16x2 split's range.
    'spike' (a finite 2^40 sample per chunk): k_fir_mfma12 (decim 1) and k_fir_mfma11 (decim 2, 4)
    compute such chunks with the exact-fp32 matrix tile of k_fir_f32mfma (fp32 products and sums;
    the decimators filter the chunk undecimated and keep every D-th output): within tolerance of
    the oracle on each chunk's own scale, and at decim 1 bit-identical to the NSH_FIR_MFMA_F32
    kernel when both use the same tap blocking (QF = 2Q - 1: 127 and 64 taps).
    'nan' (a NaN per chunk): every form computes such chunks with the fp32 direct form: the same
    NaN positions as k_fir_direct and every finite output bit-identical to it."""
    torch = torch_cuda
    h = (np.hamming(ntaps) / (ntaps / 2)).astype(np.float32)
    n = 9 * 2048 + 333
    x = orc.synth(n, 5)
    if kind == "spike":
        x[100::2048] *= np.float32(2.0 ** 40)
    else:
        x[100::2048] = complex(np.nan, 0.5)
    plan = nsh.FirPlan(h, decim, nsh.FIR_MFMA)
    if ntaps == 127:
        assert plan.kernel.startswith({1: "k_fir_mfma12",
                                       2: "k_fir_mfma13", 4: "k_fir_mfma13"}[decim]), plan.kernel
    y, hy = run_fir(torch, plan, x, n // decim)
    yd, hd = run_fir(torch, nsh.FirPlan(h, decim, nsh.FIR_DIRECT), x, n // decim)
    np.testing.assert_array_equal(hy.view(np.uint32), hd.view(np.uint32))
    if kind == "nan":
        nan = np.isnan(yd.real) | np.isnan(yd.imag)
        np.testing.assert_array_equal(np.isnan(y.real) | np.isnan(y.imag), nan)
        np.testing.assert_array_equal(y[~nan].view(np.uint32), yd[~nan].view(np.uint32))
        return
    if decim == 1:
        pf = nsh.FirPlan(h, 1, nsh.FIR_MFMA_F32)
        q12 = int(plan.kernel.split("<")[1].rstrip(">"))
        if pf.kernel == "k_fir_f32mfma<%d>" % (2 * q12 - 1):
            yf, _ = run_fir(torch, pf, x, n)
            np.testing.assert_array_equal(y.view(np.uint32), yf.view(np.uint32))
    ref = orc.fir_ccf(x[: n // decim * decim], h, decim)
    c = 2048 // decim
    for a in range(0, n // decim, c):   # each chunk on its own scale
        ok, err, scale = orc.tol_ok(y[a:a + c], ref[a:a + c])
        assert ok, (a, err, scale)


def test_fir_mfma12_exact_queue_streams(torch_cuda):
    """k_fir_mfma12 hands the chunks the split cannot carry to k_fir_exact12 through a queue per plan
    and stream. One plan on two streams, calls with and without such chunks interleaved, the second
    stream's queue grown by a longer call (1 chunk, then 2500): every call with exact chunks meets the
    tolerance per chunk, and every call without them is bit-identical to a fresh plan's output -- a
    queue left non-empty would have re-filtered stale chunks into it."""
    torch = torch_cuda
    h = _firwin127()
    plan = _v8_plan(h, "v12")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def call(x, stream):
        dx = dev(torch, x)
        hin = torch.zeros(126, dtype=torch.complex64, device="cuda")
        hout = torch.zeros_like(hin)
        dy = torch.full((x.size,), complex(7.0, 7.0), dtype=torch.complex64, device="cuda")
        torch.cuda.current_stream().synchronize()
        plan(dx, hin, hout, dy, x.size, stream=stream)
        stream.synchronize()
        return host(dy)

    def fresh(x):
        p = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
        y, _ = run_fir(torch, p, x, x.size)
        p.close()
        return y

    def check_exact(y, x):
        ref = orc.fir_ccf(x, h)
        for a in range(0, x.size, 2048):
            ok, err, scale = orc.tol_ok(y[a:a + 2048], ref[a:a + 2048])
            assert ok, (a, err, scale)

    xe = orc.synth(40 * 2048 + 5, 61)
    xe[300::4096] *= np.float32(2.0 ** 40)           # every other chunk on the exact-fp32 tile
    xe[7 * 2048 + 9] = complex(np.nan, 1.0)          # one chunk on the direct form
    xp = orc.synth(40 * 2048 + 5, 62)                # no exact chunk
    small = orc.synth(2048, 63)
    small[10] *= np.float32(2.0 ** 40)
    check_exact(call(small, s2), small)              # s2's queue: 1024 entries
    for stream in (s1, s2, s1):
        y = call(xe, stream)
        nan = np.isnan(y.real) | np.isnan(y.imag)
        ref = orc.fir_ccf(xe, h)
        np.testing.assert_array_equal(nan, np.isnan(ref.real) | np.isnan(ref.imag))
        ok_rows = ~(np.isnan(ref.real) | np.isnan(ref.imag))
        for a in range(0, xe.size, 2048):
            m = ok_rows[a:a + 2048]
            ok, err, scale = orc.tol_ok(y[a:a + 2048][m], ref[a:a + 2048][m])
            assert ok, (a, err, scale)
        np.testing.assert_array_equal(call(xp, stream).view(np.uint32), fresh(xp).view(np.uint32))
    big = orc.synth(2500 * 2048, 64)                 # grows s2's queue (2500 > 1024 entries)
    big[500::2048] *= np.float32(2.0 ** 40)
    check_exact(call(big, s2), big)
    np.testing.assert_array_equal(call(xp, s2).view(np.uint32), fresh(xp).view(np.uint32))
    plan.close()


@pytest.mark.parametrize("kind", ["nan", "spike"])
def test_fir_mfma12_exact_chunk_zero_from_history(torch_cuda, kind):
    """A history sample that sends chunk 0 to an exact form (inf/NaN: the direct form; a 2^40
    spike: the exact-fp32 tile): k_fir_exact12 re-reads chunk 0's halo from hist_in (the first kernel
    has already written hist_out by then, so the two must differ -- they may not alias). The
    non-finite pattern equals the direct form's and the oracle's; finite outputs meet the tolerance
    per chunk; hist_out is the last 126 inputs either way."""
    torch = torch_cuda
    h = _firwin127()
    n = 3 * 2048 + 17
    x = orc.synth(n, 71)
    hist = orc.synth(126, 72)
    if kind == "nan":
        hist[100] = complex(np.nan, 0.0)
    else:
        hist[100] *= np.float32(2.0 ** 40)
    y, hy = run_fir(torch, _v8_plan(h, "v12"), x, n, hist=hist)
    yd, hd = run_fir(torch, nsh.FirPlan(h, 1, nsh.FIR_DIRECT), x, n, hist=hist)
    np.testing.assert_array_equal(hy.view(np.uint32), x[-126:].view(np.uint32))
    ref = orc.fir_ccf(x, h, hist=hist)
    bad = ~(np.isfinite(ref.real) & np.isfinite(ref.imag))
    np.testing.assert_array_equal(~(np.isfinite(y.real) & np.isfinite(y.imag)), bad)
    np.testing.assert_array_equal(~(np.isfinite(yd.real) & np.isfinite(yd.imag)), bad)
    for a in range(0, n, 2048):
        m = ~bad[a:a + 2048]
        ok, err, scale = orc.tol_ok(y[a:a + 2048][m], ref[a:a + 2048][m])
        assert ok, (a, err, scale)


@pytest.mark.parametrize("decim", [1, 2, 4])
@pytest.mark.parametrize("ntaps", [127, 61])
def test_fir_mfma_exact_tile_mixed_stream(torch_cuda, ntaps, decim):
    """The exact-fp32 tile behind the default kernels (k_fir_mfma12 / k_fir_exact12, k_fir_mfma11,
    k_fir_mfma13 / k_fir_exact13) on a stream that
    mixes ordinary chunks, chunks holding a finite 2^35 spike (beyond the split's range: the tile)
    and chunks holding a sample 2^-35 below their maximum, cut into two calls at an unaligned point
    with the history handed over, the second call ending inside a chunk. The tile's fp32 products
    and sums carry no chunk-level scale, so every output meets the tolerance on its own block of
    2048 / D outputs (scale = that block's largest reference output)."""
    torch = torch_cuda
    h = (np.hamming(ntaps) / (ntaps / 2)).astype(np.float32)
    n_out = 23 * (2048 // decim) + 77
    x = orc.synth(n_out * decim, 41)
    rng = np.random.default_rng(5)
    for c in rng.choice(23, 7, replace=False):
        x[c * 2048 + int(rng.integers(0, 2048))] *= np.float32(2.0 ** 35)
    for c in rng.choice(23, 4, replace=False):
        x[c * 2048 + int(rng.integers(0, 2048))] *= np.float32(2.0 ** -35)
    plan = nsh.FirPlan(h, decim, nsh.FIR_MFMA)
    assert plan.kernel.startswith({1: "k_fir_mfma12", 2: "k_fir_mfma13", 4: "k_fir_mfma13"}[decim]), plan.kernel
    n1 = 9 * (2048 // decim) + 333  # first call: ends inside a chunk
    y1, h1 = run_fir(torch, plan, x[: n1 * decim], n1)
    y2, _ = run_fir(torch, plan, x[n1 * decim:], n_out - n1, hist=h1)
    y = np.concatenate([y1, y2])
    ref = orc.fir_ccf(x, h, decim)
    blk = 2048 // decim
    for a in range(0, n_out, blk):
        ok, err, scale = orc.tol_ok(y[a:a + blk], ref[a:a + blk])
        assert ok, (a, err, scale)


def test_fir_mfma_per_chunk_scale(torch_cuda, v8_form):
    """Segments at amplitudes 1e-30, 1 and 1e30 (each far outside fp16's range unscaled):
    the per-chunk power-of-two scale keeps every segment at fp32 accuracy, checked on the
    segment's own scale; chunks mixing two amplitudes take the exact path."""
    torch = torch_cuda
    h = _firwin127()
    seg = 20_480
    x = orc.synth(3 * seg, 33)
    x[:seg] *= np.float32(1e-30)
    x[2 * seg:] *= np.float32(1e30)
    y, _ = run_fir(torch, _v8_plan(h, v8_form), x, x.size)
    ref = orc.fir_ccf(x, h)
    for a, b in ((0, seg), (seg + 127, 2 * seg), (2 * seg + 127, 3 * seg)):
        ok, err, scale = orc.tol_ok(y[a:b], ref[a:b])
        assert ok, (a, b, err, scale)


def test_fir_mfma_tiny_and_zero_chunks(torch_cuda, v8_form):
    """All-zero chunks, an fp32-subnormal sample and a sample 2^-30 below its chunk maximum
    (fp16-subnormal after scaling: that chunk and its successor take the exact path), and
    a stream that ends inside a chunk: every output meets the tolerance, zeros stay zero."""
    torch = torch_cuda
    h = _firwin127()
    x = orc.synth(30_001, 77)
    x[2048:3 * 2048 + 100] = 0                       # zero chunks (and a zero halo)
    x[9000] = np.complex64(complex(1e-40, -3e-41))  # fp32 subnormal among O(1) samples
    x[15_000] = np.complex64(complex(2.0 ** -30, 0.0))
    y, _ = run_fir(torch, _v8_plan(h, v8_form), x, x.size)
    ref = orc.fir_ccf(x, h)
    ok, err, scale = orc.tol_ok(y, ref)
    assert ok, (err, scale)
    assert not np.any(y[2048 + 126:3 * 2048 + 100])


def test_fir_mfma_taps_far_below_max(torch_cuda):
    """Taps 2^-40 below the largest (and firwin's ~1e-18 taps at its sinc zeros) fall into
    fp16's subnormal range after scaling; the fp16x2 kernel still serves the plan and meets
    the tolerance (such a tap moves an output by <= 2^-39 max|h| sum|x|)."""
    torch = torch_cuda
    h = _firwin127()
    h[5] = np.float32(h.max() * 2.0 ** -40)
    x = orc.synth(30_000, 4)
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    assert plan.kernel == "k_fir_mfma12<5>", plan.kernel
    y, _ = run_fir(torch, plan, x, x.size)
    ok, err, scale = orc.tol_ok(y, orc.fir_ccf(x, h))
    assert ok, (err, scale)


def test_fir_plan_kernels():
    """Which kernel each algorithm runs (no silent fallback between the MFMA forms)."""
    h = _firwin127()
    assert nsh.FirPlan(h, 1, nsh.FIR_MFMA).kernel == "k_fir_mfma12<5>"
    assert nsh.FirPlan(h, 1, nsh.FIR_AUTO).kernel == "k_fir_mfma12<5>"
    assert nsh.FirPlan(h, 1, nsh.FIR_DIRECT).kernel == "k_fir_direct<1,8>"
    assert nsh.FirPlan(h, 2, nsh.FIR_MFMA).kernel == "k_fir_mfma13<2,5>"  # the lockstep walk at D = 2 too (r05zzg)
    assert nsh.FirPlan(h, 4, nsh.FIR_MFMA).kernel == "k_fir_mfma13<4,3>"  # the lockstep walk (round 5)
    for L in (1, 17, 33, 65, 97, 129, 161):
        assert nsh.FirPlan(np.ones(L, np.float32), 1, nsh.FIR_MFMA).kernel == "k_fir_mfma12<%d>" % ((L + 30) // 32 + 1)


def test_fir_retired_algorithms_fail_loudly():
    """The bf16x3 kernels retired in round 4 are refused at plan creation, never silently
    replaced by another kernel."""
    h = _firwin127()
    for algo in (nsh.FIR_MFMA_BF16X3, nsh.FIR_MFMA16):
        with pytest.raises(nsh.NshError, match="retired"):
            nsh.FirPlan(h, 1, algo)


def test_fft_golden(torch_cuda, golden):
    torch = torch_cuda
    g = golden("fft1024.npz")
    dx = dev(torch, g["x"])
    dy = torch.empty_like(dx)
    nf = g["x"].size // 1024
    nsh.fft1024(dx, dy, nf)
    ok, err, scale = orc.tol_ok(host(dy), g["X"])
    assert ok, (err, scale)
    nsh.fft1024(dx, dy, nf, inverse=True)
    ok, err, scale = orc.tol_ok(host(dy), g["Xi"])
    assert ok, (err, scale)
    dw = dev(torch, g["w"])
    nsh.channelizer1024(dx, dy, dw, nf)
    ok, err, scale = orc.tol_ok(host(dy), g["y_chan"])
    assert ok, (err, scale)


def test_fft_roundtrip_large(torch_cuda):
    """ifft(fft(x)) == 1024 x (size-independent property) at 2^22 samples."""
    torch = torch_cuda
    n = 1 << 22
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, 77)
    X = torch.empty_like(x)
    xr = torch.empty_like(x)
    nsh.fft1024(x, X, n // 1024)
    nsh.fft1024(X, xr, n // 1024, inverse=True)
    torch.cuda.synchronize()
    err = (xr / 1024 - x).abs().max().item()
    assert err <= 1e-5 * x.abs().max().item(), err
    sub = x[: 64 * 1024].cpu().numpy()
    ok, e, s = orc.tol_ok(X[: 64 * 1024].cpu().numpy(), orc.fft1024(sub))
    assert ok, (e, s)


@pytest.mark.parametrize("log2n", [27, 28])
def test_fft_chan_full_size_grid_walk(torch_cuda, log2n):
    """2^27 and 2^28 samples (C4's batch): more frames than one sweep of the grid-stride walk
    (fft1024: 24576 workgroups x 4 frames, channelizer: 16384 x 4), so workgroups walk 2-4 frame
    groups and the last sweep is partial. The frames around each sweep boundary and the last ones
    against the oracle; ifft(fft(x)) = 1024 x over the whole stream."""
    torch = torch_cuda
    n = 1 << log2n
    nf = n // 1024
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, 5 + log2n)
    X = torch.empty_like(x)
    nsh.fft1024(x, X, nf)
    xr = torch.empty_like(x)
    nsh.fft1024(X, xr, nf, inverse=True)
    rng = np.random.default_rng(log2n)
    w = (rng.standard_normal(1024) + 1j * rng.standard_normal(1024)).astype(np.complex64)
    y = torch.empty_like(x)
    nsh.channelizer1024(x, y, dev(torch, w), nf)
    torch.cuda.synchronize()
    err = (xr / 1024 - x).abs().max().item()
    assert err <= 1e-5 * x.abs().max().item(), err
    del xr
    frames = sorted({f for b in (98304, 196608, 65536, 131072, 196608, 262144) for f in (b - 1, b, b + 1)
                     if 0 <= f < nf} | {0, nf - 2, nf - 1})
    xs = np.concatenate([x[1024 * f:1024 * (f + 1)].cpu().numpy() for f in frames])
    Xs = np.concatenate([X[1024 * f:1024 * (f + 1)].cpu().numpy() for f in frames])
    ys = np.concatenate([y[1024 * f:1024 * (f + 1)].cpu().numpy() for f in frames])
    ok, e, s = orc.tol_ok(Xs, orc.fft1024(xs))
    assert ok, ("fft", e, s)
    ok, e, s = orc.tol_ok(ys, orc.channelizer1024(xs, w))
    assert ok, ("channelizer", e, s)


@pytest.mark.parametrize("ntaps", [1, 15, 16, 17, 127, 200, 257])
def test_fir_mfma_f32_exact_class(torch_cuda, ntaps):
    """The exact-fp32 matrix form (k_fir_f32mfma): fp32 products and sums, no split -- its
    error is the fp32 direct form's order-of-summation difference, far inside 1e-5, including
    at tap counts past the split forms' limit and across calls with history."""
    torch = torch_cuda
    rng = np.random.default_rng(ntaps)
    h = (rng.standard_normal(ntaps) * 0.1).astype(np.float32)
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA_F32)
    assert plan.kernel == "k_fir_f32mfma<%d>" % ((ntaps + 30) // 16), plan.kernel
    x = orc.synth(70_001, 31)
    hist = orc.synth(max(ntaps - 1, 1), 77)[: ntaps - 1]
    y, hout = run_fir(torch, plan, x, x.size, hist=hist if ntaps > 1 else None)
    y_ref, h_ref = orc.fir_ccf(x, h, hist=hist if ntaps > 1 else None, return_hist=True)
    ok, err, scale = orc.tol_ok(y, y_ref)
    assert ok, (ntaps, err, scale)
    np.testing.assert_array_equal(hout, h_ref)
    # the error class of exact fp32: no worse than twice the fp32 direct form's
    yd, _ = run_fir(torch, nsh.FirPlan(h, 1, nsh.FIR_DIRECT), x, x.size, hist=hist if ntaps > 1 else None)
    _, err_d, _ = orc.tol_ok(yd, y_ref)
    assert err <= max(2 * err_d, 1e-7 * scale), (err, err_d, scale)


def test_fir_mfma_f32_nonfinite_and_range(torch_cuda):
    """inf/NaN chunks take the fp32 direct form inside the launch (the zero-padded K would
    make inf*0 = NaN): the non-finite pattern equals the oracle's; 1e+-30 and subnormal
    samples need no scaling in fp32 and meet the tolerance."""
    torch = torch_cuda
    h = _firwin127()
    x = orc.synth(60_000, 13)
    x[1000] = np.complex64(complex(np.inf, 0.5))
    x[30_000] = np.complex64(complex(0.25, np.nan))
    x[40_000:41_000] *= np.float32(1e30)
    x[50_000:51_000] *= np.float32(1e-40)
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA_F32)
    y, _ = run_fir(torch, plan, x, x.size)
    ref = orc.fir_ccf(x, h)
    for part in ("real", "imag"):
        a, b = getattr(y, part), getattr(ref, part)
        np.testing.assert_array_equal(np.isnan(a), np.isnan(b))
        np.testing.assert_array_equal(np.isinf(a), np.isinf(b))
    fin = np.isfinite(ref)
    big = np.abs(ref[fin]).max()
    assert np.all(np.abs(y[fin] - ref[fin]) <= 1e-5 * np.abs(ref[fin]) + 1e-6 * big)


def test_fir_headline_full_size(torch_cuda):
    """BASELINE C3 at its full size: the default plan (k_fir_mfma12) over 2^28 samples, as
    bench.py runs it. Oracle windows at the stream's start and end, at chunk boundaries that are
    also XCD-range boundaries of the chunk remap (per_x chunks per XCD), and at random chunks;
    linearity FIR(0.5 x1 + x2) == 0.5 FIR(x1) + FIR(x2) over the whole stream; outputs are
    deterministic (a second run is bit-identical)."""
    torch = torch_cuda
    n = 1 << 28
    h = _firwin127()
    plan = nsh.FirPlan(h, 1)
    assert plan.kernel.startswith("k_fir_mfma12")
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    nsh.synth(x, n, 0)
    hout = torch.empty(126, dtype=torch.complex64, device="cuda")
    y = torch.empty_like(x)
    plan(x, 0, hout, y, n)  # null history: zeros before the stream
    torch.cuda.synchronize()
    nch = n // 2048
    per_x = (nch + 7) // 8
    rng = np.random.default_rng(28)
    starts = [0, n - 6000] + [per_x * 2048 * k - 3000 for k in range(1, 8)] + \
             [int(c) * 2048 - 100 for c in rng.integers(1, nch, 6)]
    for a in starts:
        m = 6000
        xs = x[a - 126 if a >= 126 else 0:a + m].cpu().numpy()
        hist = xs[:126] if a >= 126 else None
        ref = orc.fir_ccf(xs[126:] if a >= 126 else xs, h, hist=hist)
        ok, err, scale = orc.tol_ok(y[a:a + m].cpu().numpy(), ref)
        assert ok, (a, err, scale)
    y_again = torch.empty_like(x)
    plan(x, 0, hout, y_again, n)
    torch.cuda.synchronize()
    assert torch.equal(y, y_again)
    del y_again
    x2 = torch.empty_like(x)
    nsh.synth(x2, n, 1 << 30)
    y2 = torch.empty_like(x)
    plan(x2, 0, hout, y2, n)
    x3 = 0.5 * x + x2
    del x
    y3 = torch.empty_like(x3)
    plan(x3, 0, hout, y3, n)
    torch.cuda.synchronize()
    lin = (0.5 * y + y2 - y3).abs().max().item()
    scale = y3.abs().max().item()
    assert lin <= 2e-6 * scale, (lin, scale)


def test_time_next_launch_events(torch_cuda):
    """nsh_time_next_launch: the next FIR launch records the event pair itself (hipExtLaunchKernel);
    the elapsed time is positive and the setting is consumed by that one launch."""
    import ctypes as C
    torch = torch_cuda
    L = nsh.lib()
    h = _firwin127()
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    n = 1 << 22
    x = orc.synth(n, 3)
    dx, dy = dev(torch, x), torch.empty(n, dtype=torch.complex64, device="cuda")
    hout = torch.empty(126, dtype=torch.complex64, device="cuda")
    ev = [C.c_void_p(), C.c_void_p()]
    for e in ev:
        assert L.nsh_event_create(C.byref(e)) == 0
    assert L.nsh_time_next_launch(ev[0], ev[1]) == 0
    plan(dx, 0, hout, dy, n)
    torch.cuda.synchronize()
    ms = C.c_float()
    assert L.nsh_event_sync(ev[1]) == 0
    assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms)) == 0
    assert 0.0 < ms.value < 50.0, ms.value
    ok, err, _ = orc.tol_ok(host(dy)[:4096], orc.fir_ccf(x[:4096], h))
    assert ok, err
    plan(dx, 0, hout, dy, n)  # not timed: the events keep the first launch's times
    torch.cuda.synchronize()
    ms2 = C.c_float()
    assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms2)) == 0 and ms2.value == ms.value
    for e in ev:
        L.nsh_event_destroy(e)


def test_armed_timing_cleared_on_early_return(torch_cuda):
    """An event pair armed before a FIR call that launches nothing (n_out = 0) is dropped when the
    call returns (launch_events_guard): the next, unrelated FIR launch does not record
    it, so the events stay unrecorded."""
    import ctypes as C
    torch = torch_cuda
    L = nsh.lib()
    h = _firwin127()
    plan = nsh.FirPlan(h, 1, nsh.FIR_MFMA)
    n = 1 << 16
    dx = dev(torch, orc.synth(n, 5))
    dy = torch.empty(n, dtype=torch.complex64, device="cuda")
    hout = torch.empty(126, dtype=torch.complex64, device="cuda")
    ev = [C.c_void_p(), C.c_void_p()]
    for e in ev:
        assert L.nsh_event_create(C.byref(e)) == 0
    assert L.nsh_time_next_launch(ev[0], ev[1]) == 0
    plan(dx, 0, hout, dy, 0)  # nothing to do: returns before any launch
    plan(dx, 0, hout, dy, n)  # must not be timed
    torch.cuda.synchronize()
    ms = C.c_float()
    assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms)) != 0  # never recorded
    for e in ev:
        L.nsh_event_destroy(e)
    plan.close()


def test_pfft_plan_timed(torch_cuda):
    """A decim-16 plan (AUTO -> k_fir_pfft) records the armed pair with its own dispatch."""
    import ctypes as C
    import scipy.signal as ss
    torch = torch_cuda
    L = nsh.lib()
    h = ss.firwin(127, 0.03).astype(np.float32)
    plan = nsh.FirPlan(h, 16, nsh.FIR_AUTO)
    assert plan.kernel.startswith("k_fir_pfft"), plan.kernel
    n_out = 1 << 16
    x = orc.synth(16 * n_out, 9)
    dx = dev(torch, x)
    dy = torch.empty(n_out, dtype=torch.complex64, device="cuda")
    hout = torch.empty(126, dtype=torch.complex64, device="cuda")
    ev = [C.c_void_p(), C.c_void_p()]
    for e in ev:
        assert L.nsh_event_create(C.byref(e)) == 0
    assert L.nsh_time_next_launch(ev[0], ev[1]) == 0
    plan(dx, 0, hout, dy, n_out)
    torch.cuda.synchronize()
    ms = C.c_float()
    assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms)) == 0 and ms.value > 0
    ok, err, _ = orc.tol_ok(host(dy), orc.fir_ccf(x, h, 16))
    assert ok, err
    for e in ev:
        L.nsh_event_destroy(e)
    plan.close()


def test_timed_launches_counter_and_stream_kernels(torch_cuda):
    """nsh_timed_launches counts the launches that took an armed pair (scheduler_hip's kernel
    timing relies on it): an armed nsh_copy / nsh_mul_const_chain_cc / nsh_channelizer1024 records
    the pair (+1, positive elapsed time); a call that launches nothing (0 bytes) leaves the count
    and drops the pair when it returns, so the next, unarmed launch is not timed."""
    import ctypes as C
    torch = torch_cuda
    L = nsh.lib()

    def count():
        c = C.c_uint64()
        assert L.nsh_timed_launches(C.byref(c)) == 0
        return c.value

    n = 1 << 20
    x = dev(torch, orc.synth(n, 11))
    y = torch.empty_like(x)
    w = dev(torch, orc.synth(1024, 12))
    calls = [lambda: nsh.copy(x, y, 8 * n), lambda: nsh.mul_const_chain_cc(x, y, n, [0.5 + 0.5j, 1j]),
             lambda: nsh.channelizer1024(x, y, w, n // 1024), lambda: nsh.synth(y, n, 7)]
    for call in calls:
        ev = [C.c_void_p(), C.c_void_p()]
        for e in ev:
            assert L.nsh_event_create(C.byref(e)) == 0
        c0 = count()
        assert L.nsh_time_next_launch(ev[0], ev[1]) == 0
        call()
        assert count() == c0 + 1
        torch.cuda.synchronize()
        ms = C.c_float()
        assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms)) == 0 and ms.value > 0
        for e in ev:
            L.nsh_event_destroy(e)
    ev = [C.c_void_p(), C.c_void_p()]
    for e in ev:
        assert L.nsh_event_create(C.byref(e)) == 0
    c0 = count()
    assert L.nsh_time_next_launch(ev[0], ev[1]) == 0
    nsh.copy(x, y, 0)  # nothing to move: no launch, the pair is dropped on return
    nsh.copy(x, y, 8 * n)  # unarmed
    torch.cuda.synchronize()
    assert count() == c0
    ms = C.c_float()
    assert L.nsh_event_elapsed_ms(ev[0], ev[1], C.byref(ms)) != 0  # never recorded
    for e in ev:
        L.nsh_event_destroy(e)


def test_pointer_device(torch_cuda):
    """nsh_pointer_device (the rccl transport's span check): device memory -> its GPU (hipMalloc and
    a VMM double-mapped ring, both mappings), host memory (pageable, pinned) and NULL -> -1."""
    import ctypes as C
    torch = torch_cuda
    L = nsh.lib()
    t = torch.empty(1024, device="cuda")
    assert nsh.pointer_device(t.data_ptr()) == 0
    assert nsh.pointer_device(t.data_ptr() + 64) == 0
    h = np.zeros(1024, np.float32)
    assert nsh.pointer_device(h.ctypes.data) == -1
    p = torch.empty(1024).pin_memory()
    assert nsh.pointer_device(p.data_ptr()) == -1
    assert nsh.pointer_device(0) == -1
    b, act, dm = C.c_void_p(), C.c_size_t(), C.c_int()
    nsh.check(L.nsh_ring_alloc(0, 1 << 20, C.byref(b), C.byref(act), C.byref(dm)), "ring")
    assert nsh.pointer_device(b.value) == 0 and nsh.pointer_device(b.value + act.value + 8) == 0
    nsh.check(L.nsh_ring_free(b), "ring free")
