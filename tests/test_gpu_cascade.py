"""GPU parity for nsh_fir_cascade2_ccf (two decimate-by-2 FIRs fused in one launch, the form
scheduler_hip's fusion pass gives a fir_filter_ccf(h1, 2) -> fir_filter_ccf(h2, 2) pair) against
the oracle's two-call chain: every size shape (one chunk per workgroup, several, partial last
chunk), tap lengths across the supported range, history hand-off across calls, the golden
4-stage chain of the reference's decimator config, and the edge values the single-stage
decimator tests carry. Tolerance: the north-star 1e-5 (oracle.tol_ok) on the final outputs."""
import numpy as np
import pytest

from oracle import oracle as orc
from newsched_amd import nsh

pytestmark = [pytest.mark.gpu, pytest.mark.legacy]  # k_fir_casc2: make LEGACY=1


def _firwin(n, cutoff):
    return np.asarray(__import__("scipy.signal", fromlist=["firwin"]).firwin(n, cutoff), np.float32)


def _plans(h1, h2):
    p1, p2 = nsh.FirPlan(h1, 2, nsh.FIR_MFMA), nsh.FirPlan(h2, 2, nsh.FIR_MFMA)
    assert p1.cascade2_supported(p2)
    return p1, p2


def run_casc(torch, p1, p2, x, n_out, hist1=None, hist2=None):
    """-> (y, hist1_out, hist2_out) for 4 n_out inputs."""
    assert x.size == 4 * n_out
    dx = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    h1 = torch.from_numpy(np.zeros(p1.ntaps - 1, np.complex64) if hist1 is None else hist1).cuda()
    h2 = torch.from_numpy(np.zeros(p2.ntaps - 1, np.complex64) if hist2 is None else hist2).cuda()
    h1o, h2o = torch.zeros_like(h1), torch.zeros_like(h2)
    dy = torch.full((max(n_out, 1),), complex(7.0, 7.0), dtype=torch.complex64, device="cuda")
    p1.cascade2(p2, dx, h1, h1o, h2, h2o, dy, n_out)
    torch.cuda.synchronize()
    return dy.cpu().numpy()[:n_out], h1o.cpu().numpy(), h2o.cpu().numpy()


def ref_chain(x, h1, h2, hist1=None, hist2=None):
    y1, hh1 = orc.fir_ccf(x, h1, 2, hist=hist1, return_hist=True)
    y2, hh2 = orc.fir_ccf(y1, h2, 2, hist=hist2, return_hist=True)
    return y2, hh1, hh2, y1


@pytest.mark.parametrize("taps", [(127, 127), (33, 127), (127, 33), (160, 95), (64, 160)])
@pytest.mark.parametrize("n_out", [1, 5, 255, 256, 257, 512, 100_000, 1 << 20, (3 << 19) + 77])
def test_cascade2_vs_oracle_chain(torch_cuda, taps, n_out):
    torch = torch_cuda
    rng = np.random.default_rng(taps[0] * 131 + taps[1] + n_out)
    h1 = rng.standard_normal(taps[0]).astype(np.float32) / taps[0]
    h2 = rng.standard_normal(taps[1]).astype(np.float32) / taps[1]
    x = orc.synth(4 * n_out, n_out % 1000)
    p1, p2 = _plans(h1, h2)
    y, hh1, hh2 = run_casc(torch, p1, p2, x, n_out)
    ry, rh1, rh2, _ = ref_chain(x, h1, h2)
    ok, err, scale = orc.tol_ok(y, ry)
    assert ok, (taps, n_out, err, scale)
    np.testing.assert_array_equal(hh1, rh1)  # the input's tail: copied, bit-exact
    ok, err, scale = orc.tol_ok(hh2, rh2)    # stage 1's last outputs
    assert ok, ("hist2", err, scale)


def test_cascade2_stream_split_and_history(torch_cuda):
    """Call-splitting invariance through both histories (ping-pong in/out pairs), including
    calls shorter than either filter."""
    torch = torch_cuda
    h1, h2 = _firwin(127, 0.45), _firwin(127, 0.45)
    p1, p2 = _plans(h1, h2)
    n_total = 400_003
    x = orc.synth(4 * n_total, 17)
    ry, _, _, _ = ref_chain(x, h1, h2)
    cuts = [0, 1, 2, 40, 41, 300, 4096, 4097, 150_000, n_total]
    hist1 = np.zeros(126, np.complex64)
    hist2 = np.zeros(126, np.complex64)
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        y, hist1, hist2 = run_casc(torch, p1, p2, x[4 * a:4 * b], b - a, hist1, hist2)
        parts.append(y)
    ok, err, scale = orc.tol_ok(np.concatenate(parts), ry)
    assert ok, (err, scale)


def test_cascade2_nonzero_initial_history(torch_cuda):
    torch = torch_cuda
    h1, h2 = _firwin(95, 0.3), _firwin(127, 0.45)
    p1, p2 = _plans(h1, h2)
    hist1 = orc.synth(94, 5000)
    hist2 = orc.synth(126, 9000) * np.float32(0.01)
    for n_out in (3, 70_000):
        x = orc.synth(4 * n_out, 77)
        y, hh1, hh2 = run_casc(torch, p1, p2, x, n_out, hist1, hist2)
        ry, rh1, rh2, _ = ref_chain(x, h1, h2, hist1, hist2)
        ok, err, scale = orc.tol_ok(y, ry)
        assert ok, (n_out, err, scale)
        np.testing.assert_array_equal(hh1, rh1)
        ok, err, scale = orc.tol_ok(hh2, rh2)
        assert ok, (n_out, "hist2", err, scale)


def test_cascade2_null_histories(torch_cuda):
    """NULL hist1_in / hist2_in read as zeros: bit-identical to explicit zero histories."""
    torch = torch_cuda
    h = _firwin(127, 0.45)
    p1, p2 = _plans(h, h)
    for n_out in (2, 50_000):
        x = orc.synth(4 * n_out, 3)
        y0, a0, b0 = run_casc(torch, p1, p2, x, n_out)
        dx = torch.from_numpy(x).cuda()
        h1o = torch.zeros(126, dtype=torch.complex64, device="cuda")
        h2o = torch.zeros_like(h1o)
        dy = torch.empty(n_out, dtype=torch.complex64, device="cuda")
        p1.cascade2(p2, dx, 0, h1o, 0, h2o, dy, n_out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dy.cpu().numpy(), y0)
        np.testing.assert_array_equal(h1o.cpu().numpy(), a0)
        np.testing.assert_array_equal(h2o.cpu().numpy(), b0)


def test_cascade2_golden_chain4(torch_cuda, golden):
    """The reference's decimator config (4 x fir(127, decim 2)) as two fused
    launches, against the committed golden 4-stage output."""
    torch = torch_cuda
    g = golden("fir127_decim2.npz")
    p1, p2 = _plans(g["taps"], g["taps"])
    x = g["x"]
    n1 = x.size // 4
    z, _, _ = run_casc(torch, p1, p2, x[:4 * n1], n1)
    z, _, _ = run_casc(torch, p1, p2, z[:4 * (n1 // 4)], n1 // 4)
    ref = g["y_chain4"]
    ok, err, scale = orc.tol_ok(z, ref[:z.size])
    assert ok, (err, scale)


def test_cascade2_edge_values(torch_cuda):
    """inf/NaN (pattern equal to the oracle chain's), a 2^60 spike, segments at 1e-30 / 1e30,
    zero runs and an fp32-subnormal sample; each region checked on its own scale. Both
    stages send the chunks that need it through their exact fp32 paths."""
    torch = torch_cuda
    h = _firwin(127, 0.45)
    p1, p2 = _plans(h, h)
    n_out = 60_000
    x = orc.synth(4 * n_out, 91)
    seg = x.size // 4
    x[:seg] *= np.float32(1e-30)
    x[3 * seg:] *= np.float32(1e30)
    x[seg + 10_000] = np.complex64(complex(np.inf, 0.5))
    x[seg + 30_000] = np.complex64(complex(np.nan, 0.0))
    x[2 * seg + 100] *= np.float32(2.0 ** 60)
    x[2 * seg + 20_000:2 * seg + 40_000] = 0
    x[2 * seg + 50_000] = np.complex64(complex(1e-40, 0.0))
    y, _, _ = run_casc(torch, p1, p2, x, n_out)
    ry, _, _, _ = ref_chain(x, h, h)
    for f in (np.isnan, np.isinf):
        for part in (np.real, np.imag):
            bad = np.nonzero(f(part(y)) != f(part(ry)))[0]
            assert bad.size == 0, (f.__name__, part.__name__, bad[:8].tolist())
    # input i reaches outputs m with 4m - 378 <= i <= 4m (composite length 127 + 2*126)
    before = lambda i: (i + 3) // 4
    after = lambda i: (i + 378) // 4 + 1
    regions = [(0, before(seg)), (after(seg), before(seg + 10_000)), (after(seg + 30_000), before(2 * seg + 100)),
               (after(2 * seg + 100), before(3 * seg)), (after(3 * seg), n_out)]
    for a, b in regions:
        ok, err, scale = orc.tol_ok(y[a:b], ry[a:b])
        assert ok, (a, b, err, scale)


def test_cascade2_rejects_unsupported(torch_cuda):
    torch = torch_cuda
    h = _firwin(127, 0.45)
    ok2 = nsh.FirPlan(h, 2, nsh.FIR_MFMA)
    for other in (nsh.FirPlan(h, 4, nsh.FIR_MFMA), nsh.FirPlan(h, 2, nsh.FIR_DIRECT), nsh.FirPlan(h[:20], 2, nsh.FIR_MFMA)):
        assert not ok2.cascade2_supported(other)
        assert not other.cascade2_supported(ok2)
        z = torch.zeros(64, dtype=torch.complex64, device="cuda")
        with pytest.raises(nsh.NshError):
            ok2.cascade2(other, z, z, z[1:], z, z[1:], z, 4)
