"""Mixed-radix FFT (mixed_fft.hip) for 7-smooth lengths that are not powers of
two, n <= 4096 -- the lengths the reference sends through its O(n^2) DFT
(src/spectral/fft_kiss.c:76-92, :114-116).

Bars: the reference harness's per-bin tolerance against NumPy f64
(python/test_fft.py:37-38, rtol = atol = 5e-5), normwise within 4x the error of
SciPy's own f32 FFT, and at least as close to f64 as the reference (Kiss
restatement, elementwise) where the oracle runs fast; the device batched,
in-place and R2C/C2R entry points; and STFT frames of 400 / 480 samples.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import harness_or_normwise

from conftest import tolerances
from vvapi import C2C, R2C, C2R, FWD, BWD

pytestmark = pytest.mark.gpu

SMOOTH = [6, 12, 45, 96, 100, 343, 400, 480, 625, 960, 1000, 1536, 2000, 2187, 2401, 3000, 3125, 3969, 4000]


def _nw(y, ref):
    return float(np.max(np.abs(y - ref)) / np.max(np.abs(ref)))


@pytest.mark.parametrize("n", SMOOTH)
def test_mixed_c2c_vs_numpy(amd, orc, n):
    import scipy.fft
    r, a = tolerances()
    rng = np.random.default_rng(5000 + n)
    x = (rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)).astype(np.complex64)
    x64 = x.astype(np.complex128)
    for d, npf, spf in ((FWD, np.fft.fft, scipy.fft.fft), (BWD, np.fft.ifft, scipy.fft.ifft)):
        ref = npf(x64)
        y = amd.fft(x, C2C, d)
        np.testing.assert_allclose(y, ref, rtol=r, atol=a)
        assert _nw(y, ref) <= max(4 * _nw(spf(x), ref), 1e-6), (d, _nw(y, ref), _nw(spf(x), ref))
        if n <= 1000:
            k = orc.fft(x, C2C, d)
            assert np.all(np.abs(y - ref) <= np.abs(k - ref) + a + r * np.abs(ref))


@pytest.mark.parametrize("n", [6, 100, 400, 480, 1000, 2000, 3000, 4000])
def test_mixed_real_vs_numpy(amd, n):
    r, a = tolerances()
    rng = np.random.default_rng(6000 + n)
    xr = (rng.random(n) - 0.5).astype(np.float32)
    ref = np.fft.rfft(xr.astype(np.float64))
    X = amd.fft(xr, R2C)
    assert X.shape == (n // 2 + 1,) and X[-1].imag == 0.0
    np.testing.assert_allclose(X, ref, rtol=r, atol=a)
    Xin = ref.astype(np.complex64)
    y = amd.fft(Xin, C2R, BWD, n=n)
    np.testing.assert_allclose(y, np.fft.irfft(Xin.astype(np.complex128), n=n), rtol=r, atol=a)


@pytest.mark.parametrize("n,b", [(400, 37), (480, 1), (45, 1000), (4000, 9), (2187, 5), (960, 513)])
def test_mixed_batched_device(vdev, n, b):
    """Batched device plans, batches that leave slots of a workgroup idle,
    both directions and in place (in == out)."""
    import torch
    rng = np.random.default_rng(n * 7 + b)
    x = (rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)
    xd = torch.from_numpy(x).cuda()
    x64 = x.astype(np.complex128)
    yf = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xd).cpu().numpy()
    yb = vdev.FftPlan(n, vdev.C2C, vdev.BWD, batch=b)(xd).cpu().numpy()
    assert _nw(yf, np.fft.fft(x64, axis=1)) <= 2e-6
    assert _nw(yb, np.fft.ifft(x64, axis=1)) <= 2e-6
    xi = xd.clone()
    vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xi, out=xi)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(xi.cpu().numpy(), yf)


@pytest.mark.parametrize("n", [100, 400, 1000, 3000])
def test_mixed_matches_dft_kernel(vdev, knob, n):
    """The mixed-radix result agrees with the exact-angle f64 DFT kernel (n < 1025)
    or Bluestein (knob NO_MIXED=1 selects them) to f32 FFT accuracy."""
    import torch
    rng = np.random.default_rng(n + 11)
    b = 4
    x = torch.from_numpy((rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)).cuda()
    ym = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(x).cpu().numpy()
    knob("NO_MIXED", "1")
    yo = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(x).cpu().numpy()
    assert _nw(ym, yo) <= 2e-6


@pytest.mark.parametrize("nfft,hop", [(400, 160), (480, 120), (960, 240), (2000, 500)])
def test_stft_smooth_nfft(amd, orc, nfft, hop):
    """STFT magnitudes with speech-style non-power-of-two frames (the frame
    gather + mixed-radix FFT + |X| path) against NumPy f64 and the reference."""
    r, a = tolerances()
    rng = np.random.default_rng(nfft * 3 + hop)
    x = rng.uniform(-1, 1, 7 * nfft + 13).astype(np.float32)
    mag = amd.spectrogram(x, nfft, hop)
    ref = orc.spectrogram(x, nfft, hop)
    assert mag.shape == ref.shape
    w = orc.window(1, nfft).astype(np.float64)
    pad = np.concatenate([x.astype(np.float64), np.zeros(nfft)])
    np_mag = np.abs(np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(ref.shape[0])]) * w, axis=1))
    np.testing.assert_allclose(mag, np_mag, rtol=r, atol=a)
    assert np.all(np.abs(mag - np_mag) <= np.abs(ref - np_mag) + a + r * np_mag)


@pytest.mark.parametrize("nfft,hop,nch,n", [(400, 160, 3, 16000), (400, 160, 5, 4481), (480, 120, 2, 4801),
                                           (960, 240, 2, 9601), (960, 480, 3, 900), (2000, 500, 2, 1999),
                                           (45, 45, 1, 1000), (7, 3, 2, 50)])
def test_stft_smooth_device_kinds(vdev, nfft, hop, nch, n):
    """Multi-channel device STFT at smooth nfft, all three row kinds (magnitude,
    complex, power bins 0..nfft/2) from the one fused mixed-radix kernel,
    against NumPy f64 on the reference's frames (stft.c:112-144)."""
    import torch
    r, a = 5e-5, 5e-5
    rng = np.random.default_rng(nfft + n)
    x = rng.uniform(-1, 1, (nch, n)).astype(np.float32)
    st = vdev.Stft(nfft, hop)
    xd = torch.from_numpy(x).cuda()
    mag = st.spectrogram(xd).cpu().numpy()
    cpx = st.spectrogram(xd, complex_out=True).cpu().numpy()
    pw = st.power(xd).cpu().numpy()
    fr = st.frames(n)
    w = (0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(nfft - 1) * np.arange(nfft, dtype=np.float32)))
    for c in range(nch):
        pad = np.concatenate([x[c].astype(np.float64), np.zeros(nfft)])
        frames = np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w.astype(np.float64)
        X = np.fft.fft(frames, axis=1)
        np.testing.assert_allclose(cpx[c], X, rtol=r, atol=a)
        np.testing.assert_allclose(mag[c], np.abs(X), rtol=r, atol=a)
        np.testing.assert_allclose(pw[c], np.abs(X[:, :nfft // 2 + 1]) ** 2, rtol=2 * r, atol=2 * a * nfft)


LARGE = [4800, 11025, 16807, 24576 * 3, 44100, 48000, 88200, 96000,
         16000, 22050, 24000, 32000, 176400, 192000, 480000]


@pytest.mark.parametrize("n", LARGE)
def test_mixed_fourstep_c2c(amd, n):
    """7-smooth n > 4096: four-step over two mixed-radix passes.  Normwise
    within 4x SciPy's f32 FFT error against f64, both directions, round trip."""
    import scipy.fft
    rng = np.random.default_rng(n)
    x = (rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)).astype(np.complex64)
    for d, npf, spf in ((FWD, np.fft.fft, scipy.fft.fft), (BWD, np.fft.ifft, scipy.fft.ifft)):
        ref = npf(x.astype(np.complex128))
        y = amd.fft(x, C2C, d)
        harness_or_normwise(y, ref, spf(x), 4)
    assert _nw(amd.fft(amd.fft(x, C2C, FWD), C2C, BWD), x) <= 1e-5


@pytest.mark.parametrize("n", [4800, 48000, 96000])
def test_mixed_fourstep_real(amd, n):
    import scipy.fft
    rng = np.random.default_rng(n + 5)
    xr = (rng.random(n) - 0.5).astype(np.float32)
    ref = np.fft.rfft(xr.astype(np.float64))
    X = amd.fft(xr, R2C)
    assert X.shape == (n // 2 + 1,) and X[-1].imag == 0.0
    harness_or_normwise(X, ref, scipy.fft.rfft(xr), 4)
    assert _nw(amd.fft(X, C2R, BWD, n=n), xr) <= 1e-5


@pytest.mark.parametrize("n,b,chunk_mb", [(48000, 5, ""), (44100, 3, "1"), (4800, 33, "0")])
def test_mixed_fourstep_batched(vdev, knob, n, b, chunk_mb):
    """Batched device plans through the four-step (chunks of one transform
    with knob MIX_CHUNK_MB=1), in place, and against Bluestein
    (knob NO_MIXED=1) to f32 FFT accuracy."""
    import torch
    rng = np.random.default_rng(n + b)
    x = (rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)
    xd = torch.from_numpy(x).cuda()
    knob("MIX_CHUNK_MB", chunk_mb)
    yf = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xd).cpu().numpy()
    yb = vdev.FftPlan(n, vdev.C2C, vdev.BWD, batch=b)(xd).cpu().numpy()
    import scipy.fft
    x64 = x.astype(np.complex128)
    for i in range(b):
        harness_or_normwise(yf[i], np.fft.fft(x64[i]), scipy.fft.fft(x[i]), 4)
        harness_or_normwise(yb[i], np.fft.ifft(x64[i]), scipy.fft.ifft(x[i]), 4)
    xi = xd.clone()
    vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xi, out=xi)
    np.testing.assert_array_equal(xi.cpu().numpy(), yf)
    knob("NO_MIXED", "1")
    yo = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xd).cpu().numpy()
    assert _nw(yf, yo) <= 4e-6


@pytest.mark.parametrize("n", [400, 1000, 4800])
def test_mixed_real_batch_invariant(vdev, amd, n):
    """A row's R2C result does not depend on the batch it is computed in: the
    batched device plan's rows equal single-row host calls bit for bit."""
    import torch
    rng = np.random.default_rng(n + 77)
    x = (rng.random((5, n)) - 0.5).astype(np.float32)
    X = vdev.FftPlan(n, vdev.R2C, vdev.FWD, batch=5)(torch.from_numpy(x).cuda()).cpu().numpy()
    for i in (0, 3, 4):
        np.testing.assert_array_equal(X[i], amd.fft(x[i], R2C))


def test_round2_golden_gpu(amd, golden):
    """The committed round-2 fixtures through the C ABI: 400-point c2c and
    480-point r2c, and the 400/160 STFT, against NumPy f64 at the harness
    tolerance (rtol = atol = 5e-5), and at least as close as the reference's own
    O(n^2) f32 DFT; zero-phase FIR bit-identical to the reference."""
    r, a = tolerances()
    g = golden("fft_smooth_400_480")
    for key, y in (("c2c_fwd", amd.fft(g["x"], C2C, FWD)), ("c2c_bwd", amd.fft(g["x"], C2C, BWD)),
                   ("r2c", amd.fft(g["xr"], R2C))):
        ref, kiss = g[key + "_np64"], g[key + "_kiss"]
        np.testing.assert_allclose(y, ref, rtol=r, atol=a)
        assert np.all(np.abs(y - ref) <= np.abs(kiss - ref) + a + r * np.abs(ref))
    g = golden("stft_16000_n400_h160")
    mag = amd.spectrogram(g["x"], 400, 160)
    np.testing.assert_allclose(mag, g["np64"], rtol=r, atol=a)
    g = golden("filtfilt")
    assert np.array_equal(amd.filtfilt(g["h9"], g["xq"])[1], g["yq_kiss"])
    assert np.array_equal(amd.filtfilt(g["h257"], g["xg"])[1], g["yg_kiss"])


def _stft_f64(x, nfft, hop, frames):
    """f64 complex rows of stft.c:112-144's frames (zero-padded past the end)
    with the reference's float Hann table (window.c:25-36)."""
    w = (0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(nfft - 1) * np.arange(nfft, dtype=np.float32)))
    pad = np.concatenate([x.astype(np.float64), np.zeros(nfft)])
    fr = np.stack([pad[f * hop:f * hop + nfft] for f in range(frames)]) * w.astype(np.float64)
    return np.fft.fft(fr, axis=1)


def _power_close(pw, X, nfft, what):
    """Power rows |X|^2 (bins 0..nfft/2) against f64: the harness bound on |X|
    carried through the square, |p - |X|^2| <= 2 rtol |X|^2 + 2 atol max(|X|, 1)."""
    r, a = tolerances()
    h = np.abs(X[:, :nfft // 2 + 1])
    assert pw.shape == h.shape, (what, pw.shape, h.shape)
    err = np.abs(pw.astype(np.float64) - h ** 2)
    bound = 2 * r * h ** 2 + 2 * a * np.maximum(h, 1.0)
    worst = np.unravel_index(np.argmax(err / bound), err.shape)
    assert np.all(err <= bound), (what, worst, float(err[worst]), float(bound[worst]), float(pw[worst]),
                                  float(h[worst] ** 2))


def _per_bin(y, ref, what, r=None, a=None):
    r0, a0 = tolerances()
    np.testing.assert_allclose(y, ref, rtol=r or r0, atol=a or a0, err_msg=what)


@pytest.mark.parametrize("nfft,hop,nch,n", [(400, 160, 4, 48000), (480, 160, 3, 20011), (960, 320, 2, 30001),
                                           (320, 160, 2, 16000), (441, 220, 2, 44100), (600, 240, 3, 9999),
                                           (640, 320, 1, 32000), (720, 360, 2, 14401), (800, 200, 2, 8000),
                                           (900, 450, 2, 27000)])
def test_stft_speech_register_kernel(vdev, orc, knob, nfft, hop, nch, n):
    """The two-pass register kernel (k_stft_sq) at every length it serves:
    magnitude, complex and power rows of a multi-channel device STFT against
    NumPy f64 per bin at the harness tolerance (python/test_fft.py:37-38;
    power rows scale |X|'s bound by 2|X|), magnitudes at least as close to f64
    as the reference's own rows (the oracle: its f32 O(n^2) DFT,
    fft_kiss.c:76-92), and the generic kernel (knob STFT_SQ=0) as a third
    opinion."""
    import torch
    r, a = tolerances()
    rng = np.random.default_rng(nfft * 7 + n)
    x = rng.uniform(-1, 1, (nch, n)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    st = vdev.Stft(nfft, hop)

    def rows():
        return (st.spectrogram(xd).cpu().numpy(), st.spectrogram(xd, complex_out=True).cpu().numpy(),
                st.power(xd).cpu().numpy())

    mag, cpx, pw = rows()
    fr = st.frames(n)
    for c in range(nch):
        X = _stft_f64(x[c], nfft, hop, fr)
        _per_bin(cpx[c], X, f"complex rows ch {c}")
        _per_bin(mag[c], np.abs(X), f"magnitude rows ch {c}")
        _power_close(pw[c], X, nfft, f"power rows ch {c}")
    sel = slice(0, min(fr, 40))    # the oracle's f32 DFT is O(n^2): a bounded set of frames
    kiss = orc.spectrogram(x[0][: (sel.stop - 1) * hop + nfft], nfft, hop)[sel]
    X = np.abs(_stft_f64(x[0], nfft, hop, fr)[sel])
    assert np.all(np.abs(mag[0][sel] - X) <= np.abs(kiss - X) + a + r * X)
    knob("STFT_SQ", "0")
    for f, g in zip((mag, cpx, pw), rows()):
        assert f.shape == g.shape
        assert np.abs(f - g).max() <= 2e-6 * np.abs(g).max()


@pytest.mark.parametrize("n,b", [(400, 1001), (480, 7), (960, 130), (320, 33), (441, 65), (600, 9), (640, 64),
                                 (720, 5), (800, 100), (900, 17)])
@pytest.mark.parametrize("fwd", [True, False])
def test_c2c_register_kernel(vdev, orc, knob, n, b, fwd):
    """c2c rows through the register kernel, both directions, out of place and
    in place: per bin against NumPy f64 at the harness tolerance, at least as
    close to f64 as the reference (Kiss restatement, its O(n^2) DFT) on a
    sample of rows, and against the generic kernel (knob STFT_SQ=0)."""
    import torch
    r, a = tolerances()
    rng = np.random.default_rng(n + b)
    x = (rng.uniform(-0.5, 0.5, (b, n)) + 1j * rng.uniform(-0.5, 0.5, (b, n))).astype(np.complex64)
    xd = torch.from_numpy(x).cuda()
    d = FWD if fwd else BWD
    plan = vdev.FftPlan(n, vdev.C2C, vdev.FWD if fwd else vdev.BWD, batch=b)
    fast = plan(xd).cpu().numpy()
    inplace = xd.clone()
    plan(inplace, out=inplace)
    ref = np.fft.fft(x.astype(np.complex128), axis=1) if fwd else np.fft.ifft(x.astype(np.complex128), axis=1)
    _per_bin(fast, ref, "c2c rows")
    for i in sorted({0, b // 2, b - 1}):
        k = orc.fft(x[i], C2C, d)
        assert np.all(np.abs(fast[i] - ref[i]) <= np.abs(k - ref[i]) + a + r * np.abs(ref[i])), i
    np.testing.assert_array_equal(inplace.cpu().numpy(), fast)
    knob("STFT_SQ", "0")
    gen = plan(xd).cpu().numpy()
    assert np.abs(fast - gen).max() <= 2e-6 * np.abs(ref).max()


@pytest.mark.parametrize("n,b", [(400, 1001), (480, 3), (960, 77), (640, 12), (882, 31), (1200, 8), (1600, 40),
                                 (1800, 3), (1920, 5)])
def test_r2c_register_kernel(vdev, orc, knob, n, b):
    """Real rows whose n/2-point transform is a register length (the even/odd
    pair transform plus the split step): per bin against NumPy f64 at the
    harness tolerance, Im(Nyquist) = 0 exactly (fft_kiss.c:120-147), at least
    as close to f64 as the reference's R2C on a sample of rows, and against the
    generic kernel (knob STFT_SQ=0)."""
    import torch
    r, a = tolerances()
    rng = np.random.default_rng(3 * n + b)
    x = rng.uniform(-1, 1, (b, n)).astype(np.float32)
    xd = torch.from_numpy(x).cuda()
    plan = vdev.FftPlan(n, vdev.R2C, vdev.FWD, batch=b)
    fast = plan(xd).cpu().numpy()
    ref = np.fft.rfft(x.astype(np.float64), axis=1)
    assert fast.shape == ref.shape
    assert np.all(fast[:, -1].imag == 0.0) and np.all(fast[:, 0].imag == 0.0)
    _per_bin(fast, ref, "r2c rows")
    for i in sorted({0, b - 1}):
        k = orc.fft(x[i], R2C)
        assert np.all(np.abs(fast[i] - ref[i]) <= np.abs(k - ref[i]) + a + r * np.abs(ref[i])), i
    knob("STFT_SQ", "0")
    gen = plan(xd).cpu().numpy()
    assert np.abs(fast - gen).max() <= 2e-6 * np.abs(ref).max()


REGISTER_LENGTHS = (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)


@pytest.mark.parametrize("n", REGISTER_LENGTHS)
def test_register_golden(amd, vdev, golden, n):
    """tests/golden/register_n{n} (tests/golden/make_golden.py round3_sets, from
    the reference compiled in oracle/_ref): c2c both directions through the
    reference API, and the STFT's magnitude / complex / power rows through the
    reference API and the multi-channel device API, per bin against f64 at the
    harness tolerance and at least as close to f64 as the reference's own
    outputs in the fixture."""
    import torch
    r, a = tolerances()
    g = golden(f"register_n{n}")

    def not_worse(y, ref, kiss, what):
        _per_bin(y, ref, what)
        assert np.all(np.abs(y - ref) <= np.abs(kiss - ref) + a + r * np.abs(ref)), what

    not_worse(amd.fft(g["x"], C2C, FWD), g["c2c_fwd_np64"], g["c2c_fwd_kiss"], "c2c fwd")
    not_worse(amd.fft(g["x"], C2C, BWD), g["c2c_bwd_np64"], g["c2c_bwd_kiss"], "c2c bwd")
    hop = int(g["hop"][0])
    X = g["stft_cpx_np64"]
    mag_host = amd.spectrogram(g["sig"], n, hop)
    assert mag_host.shape == g["stft_mag_kiss"].shape
    not_worse(mag_host, np.abs(X), g["stft_mag_kiss"], "spectrogram (host API)")
    st = vdev.Stft(n, hop)
    sd = torch.from_numpy(np.stack([g["sig"], g["sig"][::-1].copy()])).cuda()
    mag = st.spectrogram(sd).cpu().numpy()[0]
    cpx = st.spectrogram(sd, complex_out=True).cpu().numpy()[0]
    pw = st.power(sd).cpu().numpy()[0]
    np.testing.assert_array_equal(mag, mag_host)
    not_worse(cpx, X, g["stft_cpx_kiss"], "complex rows")
    _power_close(pw, X, n, "power rows")
    half = np.abs(X[:, :n // 2 + 1])
    kiss_pw = np.abs(g["stft_cpx_kiss"][:, :n // 2 + 1].astype(np.complex128)) ** 2
    assert np.all(np.abs(pw - half ** 2) <= np.abs(kiss_pw - half ** 2) + 2 * (a + r * half) * np.maximum(half, 1.0))


def test_register_r2c_golden(amd, vdev, golden):
    """tests/golden/register_r2c: R2C at 400, 480 and twice every register
    length, through the reference API and a batched device plan (the fixture
    row among others must come out bit-identical)."""
    import torch
    r, a = tolerances()
    g = golden("register_r2c")
    for key in sorted(k for k in g if k.startswith("x")):
        n = int(key[1:])
        xr, ref, kiss = g[key], g[f"np64_{n}"], g[f"kiss{n}"]
        y = amd.fft(xr, R2C)
        _per_bin(y, ref, f"r2c {n}")
        assert y[-1].imag == 0.0
        assert np.all(np.abs(y - ref) <= np.abs(kiss - ref) + a + r * np.abs(ref)), n
        rows = np.random.default_rng(n).uniform(-1, 1, (6, n)).astype(np.float32)
        rows[4] = xr
        yb = vdev.FftPlan(n, vdev.R2C, vdev.FWD, batch=6)(torch.from_numpy(rows).cuda()).cpu().numpy()
        np.testing.assert_array_equal(yb[4], y)


@pytest.mark.parametrize("nfft,hop", [(4800, 1200), (8000, 2000), (6000, 1500)])
def test_stft_smooth_nfft_above_fused(vdev, nfft, hop):
    """7-smooth nfft > 4096 has no single-pass plan: the STFT takes the generic
    frame gather + four-step FFT path (a regression test: these once returned
    INTERNAL).  All three row kinds, normwise within 4x SciPy's own f32 FFT
    error against f64 on the reference's frames (stft.c:112-144)."""
    import scipy.fft
    import torch
    rng = np.random.default_rng(nfft)
    nch, n = 2, 5 * nfft + 77
    x = rng.uniform(-1, 1, (nch, n)).astype(np.float32)
    st = vdev.Stft(nfft, hop)
    xd = torch.from_numpy(x).cuda()
    mag = st.spectrogram(xd).cpu().numpy()
    cpx = st.spectrogram(xd, complex_out=True).cpu().numpy()
    pw = st.power(xd).cpu().numpy()
    fr = st.frames(n)
    w = (0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(nfft - 1) * np.arange(nfft, dtype=np.float32)))
    for c in range(nch):
        pad = np.concatenate([x[c], np.zeros(nfft, np.float32)])
        f32 = np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w
        X = np.fft.fft(f32.astype(np.float64), axis=1)
        X32 = scipy.fft.fft(f32, axis=1)
        harness_or_normwise(cpx[c], X, X32, 4)
        harness_or_normwise(mag[c], np.abs(X), np.abs(X32), 4)
        bound = max(4 * _nw(X32, X), 1e-6)
        assert _nw(pw[c], np.abs(X[:, :nfft // 2 + 1]) ** 2) <= 2 * bound
