"""GPU parity of the chirp-z transform (src/spectral/czt.c) and the cepstrum /
minimum-phase family (src/envelope/cepstrum.c, minphase.c) -- the FFT callers
SURVEY 8b lists -- through the reference's C API (host pointers) and the
batched device API.

Oracles: scipy.signal.czt / NumPy in f64 on the same f32 inputs, at the
reference harness tolerance (python/test_czt.py: rtol = atol = 2e-4) for the
harness's own cases, and normwise elsewhere; the compiled reference
(oracle/_ref) where its float chirps are accurate (N small).  The reference's
chirp angles are float products 0.5 n^2 * arg W, so its error grows with N (0.03
absolute at N = 257, useless at N = 4096, tests/test_oracle.py); the MI355X
chirps are tabulated in extended precision, so for large N the bar is f64
SciPy, not the reference."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _normwise(y, ref):
    return float(np.linalg.norm((y - ref).ravel()) / max(np.linalg.norm(ref.ravel()), 1e-30))


def _c64(z):
    return complex(np.complex64(z))


def _eff(z):
    """W or A as the transform uses it: argument of the float components, magnitude
    rounded to float (the reference's (float)hypot, czt.c:81-82)"""
    z = complex(np.complex64(z))
    return float(np.float32(abs(z))) * np.exp(1j * np.angle(z))


CASES = [(8, 8), (32, 32), (100, 64), (257, 300), (1000, 17), (4096, 4096), (3000, 5000), (1, 7), (9, 1),
         (40000, 1000)]


@pytest.mark.parametrize("n,m", CASES)
def test_czt_vs_scipy(amd, n, m):
    """DFT, zoom-arc and spiral parameters, complex and real input, against
    scipy.signal.czt in f64 (normwise <= 1e-5; P = next_pow2(N + M - 1) covers the
    fused, four-step and 2^16 FFT paths).  W and A are the float pairs the C API
    takes, with their magnitudes rounded to float as in the reference (_eff)."""
    from scipy.signal import czt
    rng = np.random.default_rng(n * 31 + m)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    params = [(np.exp(-2j * np.pi / max(n, 2)), 1.0), (np.exp(-2j * np.pi * 0.1 / m), np.exp(0.25j))]
    if max(n, m) <= 400:   # |W|^(k^2/2) = exp(2.5e-4 k^2) stays well inside float range
        params.append((1.0005 * np.exp(-0.03j), 0.999 * np.exp(0.1j)))
    for w, a in params:
        w, a = _c64(w), _c64(a)
        for xin in (x, x.real.astype(np.float32)):
            y = amd.czt(xin, m, w, a)
            ref = czt(xin.astype(np.complex128 if np.iscomplexobj(xin) else np.float64), m=m, w=_eff(w), a=_eff(a))
            assert np.all(np.isfinite(y))
            assert _normwise(y, ref) <= 1e-5, (n, m, w, a, _normwise(y, ref))


def test_czt_reference_harness_cases(amd, ref):
    """The reference's own checks through its C API: czt_tests.c:10-39 (impulse ->
    flat spectrum at DFT parameters, 1e-3) and python/test_czt.py (N = M = 32
    random complex; 800-1200 Hz zoom of a 1 kHz tone, M = 64) at rtol = atol = 2e-4
    vs scipy; and within 2x that bound of the compiled reference."""
    from scipy.signal import czt
    n = 8
    x = np.zeros(n, np.complex64)
    x[0] = 1
    ang = -2.0 * np.pi / n
    w = complex(np.float32(np.cos(ang)), np.float32(np.sin(ang)))
    assert np.allclose(amd.czt(x, n, w, 1.0 + 0j), 1.0, atol=1e-3)
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(32) + 1j * rng.standard_normal(32)).astype(np.complex64)
    w = _c64(np.exp(-2j * np.pi / 32))
    y, y_ref = amd.czt(x, 32, w, 1.0 + 0j), ref.czt(x, 32, w, 1.0 + 0j)
    s = czt(x.astype(np.complex128), m=32, w=w, a=1.0)
    np.testing.assert_allclose(y, s, rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(y, y_ref, rtol=4e-4, atol=4e-4)
    fs, f0 = 48000.0, 1000.0
    xr = np.cos(2 * np.pi * f0 * np.arange(32) / fs).astype(np.float32)
    st, W, A = amd.czt_params(800.0, 1200.0, 64, fs)
    assert st == 0 and (W, A) == ref.czt_params(800.0, 1200.0, 64, fs)[1:]
    y2 = amd.czt(xr, 64, W, A)
    np.testing.assert_allclose(y2, czt(xr.astype(np.float64), m=64, w=W, a=A), rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(y2, ref.czt(xr, 64, W, A), rtol=4e-4, atol=4e-4)


def test_czt_batched_device(vdev, amd):
    """The batched device plan equals one call per row (bit-identical) and the
    host API; complex and real rows; a batch large enough to be cut into chunks."""
    import torch
    n, m = 1500, 700
    w, a = _c64(np.exp(-2j * np.pi * 0.21 / m)), _c64(np.exp(0.4j))
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.complex(torch.randn(37, n, device="cuda", generator=g), torch.randn(37, n, device="cuda", generator=g))
    plan = vdev.CztPlan(n, m, w, a)
    y = plan(x)
    for r in (0, 11, 36):
        assert torch.equal(plan(x[r].contiguous()), y[r])
    np.testing.assert_array_equal(amd.czt(x[3].cpu().numpy(), m, w, a), y[3].cpu().numpy())
    xr = x.real.contiguous()
    yr = plan(xr)
    assert torch.equal(plan(xr[5].contiguous()), yr[5])
    np.testing.assert_array_equal(amd.czt(xr[5].cpu().numpy(), m, w, a), yr[5].cpu().numpy())
    big = vdev.CztPlan(300, 200, w, a)   # 512-point rows: 131072 rows per 256 MiB chunk
    xb = torch.randn(140000, 300, device="cuda", generator=g)
    yb = big(xb)
    for r in (0, 131071, 131072, 139999):
        assert torch.equal(big(xb[r].contiguous()), yb[r]), r
    with pytest.raises(vdev.VvError):
        plan(torch.zeros(2, n + 1, dtype=torch.complex64, device="cuda"))


CEPS_SIZES = [1, 2, 3, 16, 17, 64, 100, 1024, 4096, 8192, 48000, 1 << 15]


def _np_cepstrum(x):
    X = np.fft.fft(x.astype(np.float64))
    return np.real(np.fft.ifft(np.log(np.abs(X) + 1e-12)))


def _np_fold(c):
    n = len(c)
    C = np.zeros(n)
    if n:
        C[0] = c[0]
    C[1:n // 2] = 2 * c[1:n // 2]
    return C


@pytest.mark.parametrize("n", CEPS_SIZES)
def test_cepstrum_vs_numpy(amd, ref, n):
    """Real cepstrum (cepstrum.c:7-41) vs NumPy f64 on the same input: at least as
    close as the compiled reference (n <= 4096, where its O(n^2) C2C... is Kiss
    radix-2 or the naive DFT), and normwise <= 2e-5 everywhere."""
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    c = amd.cepstrum(x)
    c64 = _np_cepstrum(x)
    e = _normwise(c, c64)
    assert e <= 2e-5, e
    if n <= 4096:
        assert e <= max(2 * _normwise(ref.cepstrum(x), c64), 1e-6)


@pytest.mark.parametrize("n", CEPS_SIZES)
def test_minphase_vs_numpy(amd, ref, n):
    """icepstrum_minphase (cepstrum.c:43-78) and minphase_from_cepstrum
    (minphase.c:7-31) vs NumPy f64 of the same definitions, on a real signal's
    cepstrum (the use the reference's envelope_tests.c makes of them)."""
    rng = np.random.default_rng(n + 7)
    x = (rng.standard_normal(n) * np.exp(-np.arange(n) / max(n / 8, 1))).astype(np.float32)
    x[0] += 1.0
    c = (_np_cepstrum(x) * 0.5).astype(np.float32)
    H64 = np.exp(np.real(np.fft.fft(_np_fold(c.astype(np.float64)))))
    spec = amd.minphase_from_cepstrum(c)
    assert np.all(spec.imag == 0)
    assert _normwise(spec.real, H64) <= 2e-5
    xm = amd.icepstrum_minphase(c)
    x64 = np.real(np.fft.ifft(H64))
    assert _normwise(xm, x64) <= 2e-5
    if n <= 4096:
        assert _normwise(xm, x64) <= max(2 * _normwise(ref.icepstrum_minphase(c), x64), 1e-6)


def test_envelope_reference_known_answers(amd):
    """envelope_tests.c:9-23 through the C API: an impulse's cepstrum is ~0
    (c0 within 1e-3, the rest within 1e-2) and the minimum-phase inverse of that
    cepstrum starts at ~1 (1e-2); argument errors as the reference."""
    x = np.zeros(16, np.float32)
    x[0] = 1
    c = amd.cepstrum(x)
    assert abs(c[0]) < 1e-3 and np.all(np.abs(c[1:]) < 1e-2)
    assert abs(amd.icepstrum_minphase(c)[0] - 1.0) < 1e-2
    H = amd.minphase_from_cepstrum(c)
    np.testing.assert_allclose(H.real, 1.0, atol=1e-3)


def test_cepstrum_batched_device(vdev, amd):
    """Batched device rows equal the one-row host calls (same kernels)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(9)
    for n in (256, 1000, 8192):
        x = torch.randn(13, n, device="cuda", generator=g)
        c = vdev.cepstrum(x)
        np.testing.assert_array_equal(c[4].cpu().numpy(), amd.cepstrum(x[4].cpu().numpy()))
        cc = (0.1 * c).contiguous()
        xm = vdev.icepstrum_minphase(cc)
        np.testing.assert_array_equal(xm[7].cpu().numpy(), amd.icepstrum_minphase(cc[7].cpu().numpy()))
        sp = vdev.minphase_from_cepstrum(cc)
        np.testing.assert_array_equal(sp[12].cpu().numpy(), amd.minphase_from_cepstrum(cc[12].cpu().numpy()))


@pytest.mark.parametrize("n,m", [(8, 8), (100, 64), (257, 300), (1000, 17), (1500, 2000), (2049, 2048), (1, 1)])
def test_czt_fused_equals_unfused(vdev, knob, n, m):
    """P = next_pow2(N + M - 1) <= 4096 runs the one-pass kernel (k_czt_fused);
    knob CZT_UNFUSED=1 the chain of element-wise kernels and library FFTs.  The
    arithmetic is the same (the 1/P of the inverse folded into B is a power of
    two), so the rows must be bit-identical, complex and real input."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(n + 3 * m)
    plan = vdev.CztPlan(n, m, _c64(np.exp(-2j * np.pi * 0.13 / m)), _c64(np.exp(0.2j)))
    xc = torch.complex(torch.randn(41, n, device="cuda", generator=g), torch.randn(41, n, device="cuda", generator=g))
    for x in (xc, xc.real.contiguous()):
        knob("CZT_UNFUSED", "0")
        a = plan(x)
        knob("CZT_UNFUSED", "1")
        b = plan(x)            # the chain's P = 1024 FFTs as 16 x 16 x 4, the fused kernel's split
        knob("CZT_UNFUSED", "")
        torch.cuda.synchronize()
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [2, 16, 256, 1024, 4096])
def test_cepstrum_fused_vs_chain(vdev, knob, n):
    """Power-of-two n <= 4096 runs the one-pass kernels (k_ceps_fused);
    knob CEPS_UNFUSED=1 the element-wise chains around the library FFTs (the
    chain's cepstrum goes through R2C/C2R instead of the reference's C2C pair).
    Both are f32 computations of the same definitions: normwise within 2e-6 (the
    one-pass kernel is compiled separately, so its FMA contractions may differ)."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(23, n, device="cuda", generator=g)
    c = (0.1 * torch.randn(23, n, device="cuda", generator=g)).contiguous()
    knob("CEPS_UNFUSED", "0")
    a = (vdev.cepstrum(x), vdev.icepstrum_minphase(c), vdev.minphase_from_cepstrum(c))
    knob("CEPS_UNFUSED", "1")
    b = (vdev.cepstrum(x), vdev.icepstrum_minphase(c), vdev.minphase_from_cepstrum(c))
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert _normwise(u.cpu().numpy(), v.cpu().numpy()) <= 2e-6


def test_czt_cepstrum_golden(amd, golden):
    """The committed fixtures through the C API: CZT at the reference harness
    tolerance (rtol = atol = 2e-4) of both the f64 result and the reference's own
    output; the cepstrum family within 1e-5 of f64 (normwise)."""
    g = golden("czt_testpy_n32")
    y = amd.czt(g["x"], 32, complex(g["w"][0]), 1.0 + 0j)
    np.testing.assert_allclose(y, g["np64"], rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(y, g["kiss"], rtol=2e-4, atol=2e-4)
    g = golden("czt_zoom_n32_m64")
    y = amd.czt(g["x"], 64, complex(g["w"][0]), complex(g["a"][0]))
    np.testing.assert_allclose(y, g["np64"], rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(y, g["kiss"], rtol=2e-4, atol=2e-4)
    g = golden("cepstrum_n64")
    assert _normwise(amd.cepstrum(g["x"]), g["ceps_np64"]) <= 1e-5
    assert _normwise(amd.icepstrum_minphase(g["c"]), g["iceps_np64"]) <= 1e-5
    assert _normwise(amd.minphase_from_cepstrum(g["c"]), g["minph_np64"]) <= 1e-5
