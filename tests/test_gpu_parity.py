"""GPU parity tests (MI355X): the HIP backend through the C ABI vs the oracle.

Tolerances are the reference harness's own (python/test_fft.py:37-38,62:
rtol = atol = 5e-5, overridable with VV_PY_RTOL / VV_PY_ATOL), applied against
NumPy float64 on the same f32 inputs (the arbiter: the reference's Kiss itself
fails them at n >= 4096), plus a secondary check against the
oracle (Kiss restatement) within 2x that bound for n <= 1024, and the
reference's own known-answer tests restated.
"""
import numpy as np
import pytest

from conftest import tolerances
from vvapi import C2C, R2C, C2R, FWD, BWD, KISS, HIP, OK, ERR_UNSUPPORTED, FirState

pytestmark = pytest.mark.gpu

POW2 = [2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096]
NONPOW2 = [3, 5, 6, 7, 9, 10, 12, 15, 20, 24, 30, 48, 100, 200]   # gtest/test_fft.cpp:300-316


def close(y, ref, rtol=None, atol=None, factor=1.0):
    r, a = tolerances()
    r = (rtol if rtol is not None else r) * factor
    a = (atol if atol is not None else a) * factor
    np.testing.assert_allclose(y, ref, rtol=r, atol=a)


def kiss_check(y, kiss, f64, n):
    """Secondary check against the Kiss restatement: within 2x the
    harness bound for power-of-two n <= 1024 (its radix-2 path).  For other n the
    reference runs an f32 O(n^2) DFT whose own error exceeds that bound, so there we
    require ours to be at least as close to f64 as Kiss is (elementwise, + tolerance)."""
    r, a = tolerances()
    if n & (n - 1) == 0:
        if n <= 1024:
            close(y, kiss, factor=2.0)
        return
    assert np.all(np.abs(y - f64) <= np.abs(kiss - f64) + a + r * np.abs(f64))


# ---------------------------------------------------------------- FFT
def test_backend_is_hip(amd):
    L = amd.lib
    assert L.vv_dsp_fft_is_backend_available(HIP) == 1
    assert L.vv_dsp_fft_get_backend() == HIP
    assert L.vv_dsp_fft_is_backend_available(KISS) == 0   # no CPU backend inside the product


@pytest.mark.parametrize("n", POW2 + NONPOW2 + [1])
def test_c2c_vs_numpy(amd, orc, n):
    rng = np.random.default_rng(n)
    x = (rng.random(n) + 1j * rng.random(n)).astype(np.complex64)
    x64 = x.astype(np.complex128)
    yf = amd.fft(x, C2C, FWD)
    yb = amd.fft(x, C2C, BWD)
    close(yf, np.fft.fft(x64))
    close(yb, np.fft.ifft(x64))
    kiss_check(yf, orc.fft(x, C2C, FWD), np.fft.fft(x64), n)
    kiss_check(yb, orc.fft(x, C2C, BWD), np.fft.ifft(x64), n)


@pytest.mark.parametrize("n", POW2 + [8192] + NONPOW2 + [1, 33, 1000])
def test_r2c_c2r_vs_numpy(amd, orc, n):
    rng = np.random.default_rng(1000 + n)
    xr = rng.random(n).astype(np.float32)
    X = amd.fft(xr, R2C)
    close(X, np.fft.rfft(xr.astype(np.float64)))
    if n % 2 == 0 and n > 1:
        assert X[-1].imag == 0.0   # fft_kiss.c:141-143
    Xin = np.fft.rfft(xr.astype(np.float64)).astype(np.complex64)
    y = amd.fft(Xin, C2R, BWD, n=n)
    close(y, np.fft.irfft(Xin.astype(np.complex128), n=n))
    kiss_check(X, orc.fft(xr, R2C), np.fft.rfft(xr.astype(np.float64)), n)


def _normwise(y, ref):
    return float(np.max(np.abs(y - ref)) / np.max(np.abs(ref)))


def harness_or_normwise(y, ref, y32, factor, floor=1e-6):
    """The harness rule (python/test_fft.py:37-38: per bin, rtol = atol =
    VV_PY_RTOL / VV_PY_ATOL = 5e-5 against f64) wherever an f32 FFT can meet it:
    if SciPy's single-precision FFT of the same input `y32` passes it per bin,
    ours must too.  Where even SciPy's f32 FFT does not (large n: rounding error
    grows with log n and |X|), normwise within `factor` x SciPy's own error --
    the reference's Kiss fails both there."""
    r, a = tolerances()
    if np.allclose(y32, ref, rtol=r, atol=a):
        np.testing.assert_allclose(y, ref, rtol=r, atol=a)
        return "per-bin"
    assert _normwise(y, ref) <= max(factor * _normwise(y32, ref), floor), (_normwise(y, ref), _normwise(y32, ref))
    return "normwise"


@pytest.mark.parametrize("n", [8192, 16384, 1 << 16, 1 << 20])
def test_c2c_large_pow2(amd, n):
    """Power-of-two lengths above one workgroup's FFT (four-step path).  The
    reference's radix-2 Kiss covers every power of two (fft_kiss.c:27-74) but is
    itself outside the harness bound from n = 4096, so the bound
    here is normwise: within 4x the error of an f32 FFT (scipy.fft, single
    precision) against f64, and a round trip back to the input."""
    import scipy.fft
    rng = np.random.default_rng(n)
    x = (rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)).astype(np.complex64)
    ref = np.fft.fft(x.astype(np.complex128))
    y = amd.fft(x, C2C, FWD)
    harness_or_normwise(y, ref, scipy.fft.fft(x), 4)
    xb = amd.fft(y, C2C, BWD)
    assert _normwise(xb, x) <= 1e-5
    refb = np.fft.ifft(x.astype(np.complex128))
    harness_or_normwise(amd.fft(x, C2C, BWD), refb, scipy.fft.ifft(x), 4)


@pytest.mark.parametrize("n", [16384, 32768, 1 << 18])
def test_real_large_pow2(amd, n):
    import scipy.fft
    rng = np.random.default_rng(n + 7)
    xr = (rng.random(n) - 0.5).astype(np.float32)
    ref = np.fft.rfft(xr.astype(np.float64))
    X = amd.fft(xr, R2C)
    assert X.shape == (n // 2 + 1,) and X[-1].imag == 0.0
    harness_or_normwise(X, ref, scipy.fft.rfft(xr), 4)
    y = amd.fft(X, C2R, BWD, n=n)
    assert _normwise(y, xr) <= 1e-5


@pytest.mark.parametrize("n,b", [(1 << 15, 3), (1 << 16, 5), (1 << 17, 2)])
def test_real_large_pow2_batched(vdev, n, b):
    """Batched R2C / C2R above the fused kernels: the n/2-point four-step plus the
    split kernels (k_real_split_fwd / _inv, bins j and n/2 - j per thread), every
    row against NumPy f64 (normwise, 4x SciPy's f32 error) and round trip."""
    import scipy.fft
    import torch
    rng = np.random.default_rng(n + b)
    xr = (rng.random((b, n)) - 0.5).astype(np.float32)
    X = vdev.FftPlan(n, vdev.R2C, vdev.FWD, batch=b)(torch.from_numpy(xr).cuda())
    Xh = X.cpu().numpy()
    for i in range(b):
        ref = np.fft.rfft(xr[i].astype(np.float64))
        assert Xh[i, -1].imag == 0.0 and Xh[i, 0].imag == 0.0
        harness_or_normwise(Xh[i], ref, scipy.fft.rfft(xr[i]), 4)
    y = vdev.FftPlan(n, vdev.C2R, vdev.BWD, batch=b)(X).cpu().numpy()
    for i in range(b):
        assert _normwise(y[i], xr[i]) <= 1e-5, i


@pytest.mark.parametrize("n", [1025, 3000, 48000, 100003])
def test_c2c_bluestein(amd, orc, n):
    """Non-power-of-two lengths from 1025 on run Bluestein over the power-of-two
    kernels (the reference: an O(n^2) f32 DFT, fft_kiss.c:76-92).  Normwise
    within 8x an f32 FFT's error vs f64, and for the lengths the CPU oracle
    finishes quickly, at least as close to f64 as the reference's own result."""
    import scipy.fft
    rng = np.random.default_rng(n)
    x = (rng.random(n) - 0.5 + 1j * (rng.random(n) - 0.5)).astype(np.complex64)
    for d, npf, spf in ((FWD, np.fft.fft, scipy.fft.fft), (BWD, np.fft.ifft, scipy.fft.ifft)):
        ref = npf(x.astype(np.complex128))
        y = amd.fft(x, C2C, d)
        e = _normwise(y, ref)
        harness_or_normwise(y, ref, spf(x), 8, floor=2e-6)
        if n <= 3000:
            assert e <= _normwise(orc.fft(x, C2C, d), ref)
    assert _normwise(amd.fft(amd.fft(x, C2C, FWD), C2C, BWD), x) <= 1e-5


@pytest.mark.parametrize("n", [1500, 48000])
def test_real_bluestein(amd, n):
    import scipy.fft
    rng = np.random.default_rng(n + 3)
    xr = (rng.random(n) - 0.5).astype(np.float32)
    ref = np.fft.rfft(xr.astype(np.float64))
    X = amd.fft(xr, R2C)
    harness_or_normwise(X, ref, scipy.fft.rfft(xr), 8, floor=2e-6)
    assert _normwise(amd.fft(X, C2R, BWD, n=n), xr) <= 1e-5


def test_large_pow2_batched_device(vdev):
    import torch
    rng = np.random.default_rng(9)
    n, b = 16384, 3
    x = (rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)
    plan = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)
    y = plan(torch.from_numpy(x).cuda()).cpu().numpy()
    import scipy.fft
    for i in range(b):
        harness_or_normwise(y[i], np.fft.fft(x[i].astype(np.complex128)), scipy.fft.fft(x[i]), 4)


@pytest.mark.parametrize("n,b,chunk_mb", [(1 << 17, 5, "1"), (1 << 20, 2, "0"), (8192, 7, "")])
def test_large_pow2_chunked_batch(vdev, knob, n, b, chunk_mb):
    """Two-pass four-step over a batch, the batch split into Infinity-Cache
    sized chunks (knob FS_CHUNK_MB: 1 -> one transform per chunk, 0 -> the whole
    batch at once), both directions, against NumPy f64 per transform."""
    import torch
    rng = np.random.default_rng(n + b)
    x = (rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)
    xd = torch.from_numpy(x).cuda()
    knob("FS_CHUNK_MB", chunk_mb)
    yf = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xd).cpu().numpy()
    yb = vdev.FftPlan(n, vdev.C2C, vdev.BWD, batch=b)(xd).cpu().numpy()
    import scipy.fft
    x64 = x.astype(np.complex128)
    for i in range(b):
        harness_or_normwise(yf[i], np.fft.fft(x64[i]), scipy.fft.fft(x[i]), 4)
        harness_or_normwise(yb[i], np.fft.ifft(x64[i]), scipy.fft.ifft(x[i]), 4)


@pytest.mark.parametrize("n,b", [(48001, 3), (3001, 5), (100003, 2)])   # not 7-smooth: Bluestein
def test_bluestein_fused_equals_unfused(vdev, n, b):
    """The fused Bluestein chain (chirp pre-multiply in the columns pass, the
    product with V and the post-multiply in the rows passes) performs the same
    f32 operations as the separate-kernel chain: bit-identical outputs, for
    complex input both ways and for real input (R2C, n/2+1 bins), batched."""
    import torch
    rng = np.random.default_rng(n + b)
    xc = torch.from_numpy((rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)).cuda()
    xr = torch.from_numpy((rng.random((b, n)) - 0.5).astype(np.float32)).cuda()

    def run():
        return [vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)(xc).cpu().numpy(),
                vdev.FftPlan(n, vdev.C2C, vdev.BWD, batch=b)(xc).cpu().numpy(),
                vdev.FftPlan(n, vdev.R2C, vdev.FWD, batch=b)(xr).cpu().numpy()]
    fused = run()
    with vdev.knobs(BLUE_UNFUSED=1):
        unfused = run()
    for f, u in zip(fused, unfused):
        assert np.array_equal(f, u)
    assert fused[2].shape == (b, n // 2 + 1)
    ref = np.fft.fft(xc.cpu().numpy().astype(np.complex128), axis=1)
    assert _normwise(fused[0], ref) <= 2e-6


def test_impulse_known_answer(amd):
    """tests/fft_backend_tests.c:70-99 and spectral_tests.c:14-35 of the reference."""
    for n in (8, 16, 1024):
        x = np.zeros(n, np.complex64)
        x[0] = 1
        X = amd.fft(x, C2C, FWD)
        np.testing.assert_allclose(X, np.ones(n), atol=1e-5)
        xr = amd.fft(X, C2C, BWD)
        np.testing.assert_allclose(xr, x, atol=1e-5)


def test_r2c_c2r_sine_roundtrip(amd):
    """fft_backend_tests.c:156-238 / spectral_tests.c:37-66 (tol 1e-3)."""
    for n in (8, 16, 1024):
        i = np.arange(n, dtype=np.float32)
        xr = np.sin(np.float32(2.0) * np.float32(np.pi) * i / np.float32(n)).astype(np.float32)
        X = amd.fft(xr, R2C)
        y = amd.fft(X, C2R, BWD, n=n)
        np.testing.assert_allclose(y, xr, atol=1e-3)


@pytest.mark.parametrize("n", [16, 64, 128])
def test_backend_consistency_with_kiss(amd, orc, n):
    """gtest/test_fft.cpp:322-358: complex exponential at bin 1 vs Kiss, 1e-5 abs."""
    t = np.arange(n)
    x = np.exp(2j * np.pi * t / n).astype(np.complex64)
    np.testing.assert_allclose(amd.fft(x, C2C, FWD), orc.fft(x, C2C, FWD), atol=1e-5, rtol=0)


def test_golden_fft_testpy(amd, golden):
    for n in (16, 1024):
        g = golden(f"fft_testpy_n{n}")
        close(amd.fft(g["x"], C2C, FWD), g["c2c_fwd_np64"])
        close(amd.fft(g["x"], C2C, BWD), g["c2c_bwd_np64"])
        close(amd.fft(g["xr"], R2C), g["r2c_np64"])
        # the reference's own C2R fails this at n=1024 (1.22x); ours must pass
        close(amd.fft(g["X"], C2R, BWD, n=n), g["c2r_np64"])


def test_golden_batched_device(vdev, golden):
    import torch
    g = golden("fft_batch64_n1024")
    x = torch.from_numpy(g["x"]).cuda()
    plan = vdev.FftPlan(1024, vdev.C2C, vdev.FWD, batch=64)
    y = plan(x).cpu().numpy()
    close(y, g["np64"])
    close(y, g["kiss"], factor=2.0)


def test_device_plan_inplace_and_batch(vdev):
    import torch
    rng = np.random.default_rng(5)
    for n in (64, 1024, 4096, 100):
        b = 33
        x = (rng.uniform(-0.5, 0.5, (b, n)) + 1j * rng.uniform(-0.5, 0.5, (b, n))).astype(np.complex64)
        t = torch.from_numpy(x).cuda()
        plan = vdev.FftPlan(n, vdev.C2C, vdev.FWD, batch=b)
        plan(t, out=t)   # in place
        close(t.cpu().numpy(), np.fft.fft(x.astype(np.complex128), axis=1))


# ---------------------------------------------------------------- STFT
def test_golden_stft_spectrogram(amd, golden):
    g = golden("stft_48000_n1024_h256")
    mag = amd.spectrogram(g["x"], 1024, 256)
    assert mag.shape == g["kiss"].shape
    close(mag, g["np64"])
    close(mag, g["kiss"], factor=2.0)


@pytest.mark.parametrize("nfft,hop", [(1024, 256), (512, 128), (256, 1), (64, 64), (4096, 1024),
                                      (8192, 2048), (100, 30), (16, 5)])
def test_stft_vs_oracle(amd, orc, nfft, hop):
    rng = np.random.default_rng(nfft + hop)
    for n in (nfft // 2, nfft, 3 * nfft + 7):
        x = rng.uniform(-1, 1, n).astype(np.float32)
        mag = amd.spectrogram(x, nfft, hop)
        ref = orc.spectrogram(x, nfft, hop)
        assert mag.shape == ref.shape
        w = orc.window(1, nfft).astype(np.float64)
        fr = ref.shape[0]
        pad = np.concatenate([x.astype(np.float64), np.zeros(nfft, np.float64)])
        frames = np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)])
        np_mag = np.abs(np.fft.fft(frames * w, axis=1))
        if nfft <= 1024:
            close(mag, np_mag)
        else:   # per bin where an f32 FFT (SciPy, single precision) meets the harness rule
            import scipy.fft
            m32 = np.abs(scipy.fft.fft((frames * w).astype(np.float32).astype(np.complex64), axis=1))
            harness_or_normwise(mag, np_mag, m32, 4)


def test_stft_large_nfft(amd, orc):
    """nfft above the fused kernels (16384: frame gather + four-step FFT)."""
    nfft, hop = 16384, 4096
    x = np.random.default_rng(77).uniform(-1, 1, 3 * nfft + 11).astype(np.float32)
    mag = amd.spectrogram(x, nfft, hop)
    ref = orc.spectrogram(x, nfft, hop)
    assert mag.shape == ref.shape
    w = orc.window(1, nfft).astype(np.float64)
    pad = np.concatenate([x.astype(np.float64), np.zeros(nfft)])
    np_mag = np.abs(np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(ref.shape[0])]) * w, axis=1))
    assert _normwise(mag, np_mag) <= 2e-6


def test_stft_process_and_reconstruct(amd, orc):
    """spectral_tests.c:82-121: STFT/OLA roundtrip MSE < 1e-2; plus process vs Kiss."""
    import ctypes as C
    N, F, H = 256, 64, 32
    x = np.sin(np.float32(2 * np.pi) * np.arange(N, dtype=np.float32) / np.float32(32)).astype(np.float32)
    st, h = amd.stft_create(F, H, 1)
    assert st == OK
    try:
        y = np.zeros(N + F, np.float32)
        norm = np.zeros(N + F, np.float32)
        fp = lambda a, off=0: a[off:].ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        start = 0
        while start + F <= N + (F - H):
            frame = np.array([x[start + i] if start + i < N else 0 for i in range(F)], np.float32)
            spec = amd.stft_process(h, frame, F)
            w = orc.window(1, F)
            np.testing.assert_allclose(spec, orc.fft((frame * w).astype(np.complex64), C2C, FWD),
                                       rtol=1e-4, atol=1e-5)
            spec32 = np.ascontiguousarray(spec.view(np.float32))
            assert amd.lib.vv_dsp_stft_reconstruct(h, fp(spec32), fp(y, start), fp(norm, start)) == OK
            start += H
        y[norm > 1e-12] /= norm[norm > 1e-12]
        assert np.mean((x - y[:N]) ** 2) < 1e-2
    finally:
        amd.lib.vv_dsp_stft_destroy(h)


def _pr_signal():
    """tests/gtest/test_stft.cpp:452-471: 512/128 Hann, a three-tone signal of
    4 * 512 samples computed in double and rounded to float."""
    F, H = 512, 128
    i = np.arange(4 * F, dtype=np.float64)
    x = (0.5 * np.sin(2.0 * np.pi * 5.0 * i / F) + 0.3 * np.sin(2.0 * np.pi * 13.0 * i / F)
         + 0.2 * np.sin(2.0 * np.pi * 23.0 * i / F)).astype(np.float32)
    return x, F, H


def _pr_check(x, y, norm, F):
    """test_stft.cpp:494-519: normalise where norm > 1e-10, then over [F, len - F)
    max |error| < 1e-3 and RMS error < 1e-5 (float arithmetic, as the test)."""
    y = y.copy()
    m = norm > np.float32(1e-10)
    y[m] /= norm[m]
    e = np.abs(x[F:len(x) - F] - y[F:len(x) - F]).astype(np.float32)
    rms = float(np.sqrt(np.sum(e * e, dtype=np.float32) / np.float32(len(e))))
    assert float(e.max()) < 1e-3, e.max()
    assert rms < 1e-5, rms
    return float(e.max()), rms


def test_stft_perfect_reconstruction_reference_api(amd):
    """The reference's known answer for perfect reconstruction
    (tests/gtest/test_stft.cpp:452-519) through the reference API on the HIP
    backend: vv_dsp_stft_process and vv_dsp_stft_reconstruct frame by frame,
    every frame with frame_start + 512 <= len."""
    import ctypes as C
    x, F, H = _pr_signal()
    st, h = amd.stft_create(F, H, 1)
    assert st == OK
    try:
        y = np.zeros(len(x), np.float32)
        norm = np.zeros(len(x), np.float32)
        fp = lambda a, off=0: a[off:].ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
        start = 0
        while start + F <= len(x):
            spec = np.ascontiguousarray(amd.stft_process(h, np.ascontiguousarray(x[start:start + F]), F).view(np.float32))
            assert amd.lib.vv_dsp_stft_reconstruct(h, fp(spec), fp(y, start), fp(norm, start)) == OK
            start += H
        _pr_check(x, y, norm, F)
    finally:
        amd.lib.vv_dsp_stft_destroy(h)


@pytest.mark.parametrize("nfft,hop,reps", [(512, 128, 1), (1024, 256, 64), (1024, 512, 16)])
def test_stft_perfect_reconstruction_batched(vdev, nfft, hop, reps):
    """The same known answer through the batched device path: all frames of
    the signal by vv_dsp_stft_process_device, then ONE fused inverse FFT +
    window + overlap-add launch (k_istft for nfft 1024, the generic OLA
    otherwise); also at 1024/256 and 1024/512 Hann over a longer multi-tone
    signal (the reference's tones scaled to the frame length)."""
    import torch
    if nfft == 512:
        x, F, H = _pr_signal()
    else:
        F, H = nfft, hop
        i = np.arange(reps * F, dtype=np.float64)
        x = (0.5 * np.sin(2.0 * np.pi * 5.0 * i / F) + 0.3 * np.sin(2.0 * np.pi * 13.0 * i / F)
             + 0.2 * np.sin(2.0 * np.pi * 23.0 * i / F)).astype(np.float32)
    count = (len(x) - F) // H + 1
    frames = np.stack([x[f * H:f * H + F] for f in range(count)])
    st = vdev.Stft(F, H)
    spec = st.process(torch.from_numpy(frames).cuda())
    y = torch.zeros(len(x), device="cuda")
    norm = torch.zeros(len(x), device="cuda")
    st.reconstruct(spec, y, norm)
    _pr_check(x, y.cpu().numpy(), norm.cpu().numpy(), F)


@pytest.mark.parametrize("hop,count", [(256, 37), (256, 700), (128, 300), (512, 9), (1024, 5), (256, 1)])
def test_stft_reconstruct_device_batched(vdev, orc, hop, count):
    """vv_dsp_stft_reconstruct (stft.c:95-110) applied to `count` frames at `hop`:
    the fused inverse-FFT + window + overlap-add kernel against the oracle's
    frame-by-frame loop, with non-zero accumulators and a general (non-Hermitian)
    spectrum.  The window-norm sums take the same values in the same order."""
    import ctypes as C
    import torch
    nfft = 1024
    rng = np.random.default_rng(hop + count)
    spec = (rng.uniform(-1, 1, (count, nfft)) + 1j * rng.uniform(-1, 1, (count, nfft))).astype(np.complex64)
    length = (count - 1) * hop + nfft
    acc0 = rng.uniform(-1, 1, length).astype(np.float32)
    nrm0 = rng.uniform(0, 1, length).astype(np.float32)
    st = vdev.Stft(nfft, hop)
    acc = torch.from_numpy(acc0.copy()).cuda()
    nrm = torch.from_numpy(nrm0.copy()).cuda()
    st.reconstruct(torch.from_numpy(spec).cuda(), acc, nrm)
    acc_only = torch.from_numpy(acc0.copy()).cuda()
    st.reconstruct(torch.from_numpy(spec).cuda(), acc_only)
    w = orc.window(1, nfft)
    ra, rn = acc0.copy(), nrm0.copy()
    fp = lambda a, off=0: a[off:].ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    for f in range(count):
        row = np.ascontiguousarray(spec[f].view(np.float32))
        assert orc.lib.orc_stft_reconstruct(fp(w), nfft, fp(row), fp(ra, f * hop), fp(rn, f * hop)) == 0
    np.testing.assert_allclose(acc.cpu().numpy(), ra, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(acc_only.cpu().numpy(), ra, rtol=1e-5, atol=1e-6)
    assert np.array_equal(nrm.cpu().numpy(), rn)


def test_stft_multichannel_equals_single(vdev):
    import torch
    rng = np.random.default_rng(9)
    sig = torch.from_numpy(rng.uniform(-1, 1, (5, 20000)).astype(np.float32)).cuda()
    st = vdev.Stft(1024, 256)
    multi = st.spectrogram(sig)
    for c in range(5):
        single = st.spectrogram(sig[c].contiguous())
        assert torch.equal(multi[c], single)
    spec = st.spectrogram(sig, complex_out=True)
    torch.testing.assert_close(spec.abs(), multi, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("nch,n", [(1, 48000 + 333), (3, 20000), (5, 1280), (4, 700), (7, 480000),
                                   (50, 480000 + 333), (2, 9 * 48000 + 4)])
def test_stft_ring_equals_span(vdev, knob, nch, n):
    """hop % 256 == 0 on the LDS-DMA path runs the ring-span kernel (VAR 3: each
    wave walks a contiguous run of pairs and DMAs only the 2*hop new samples of
    each span).  Rows must be bit-identical to the whole-span kernel (VAR 0,
    knob STFT_RING=0) in all three output kinds: runs cross channel boundaries
    (50 ch: 16-pair runs over 938-pair channels), start at tail pairs, and end
    on odd frame counts."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(nch * 7 + n)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    for hop in (256, 512):
        st = vdev.Stft(1024, hop)
        kinds = (lambda: st.spectrogram(sig), lambda: st.spectrogram(sig, complex_out=True), lambda: st.power(sig))
        for kind, f in enumerate(kinds):
            knob("STFT_RING", "1")
            ring = f()
            knob("STFT_RING", "0")
            span = f()
            torch.cuda.synchronize()
            assert torch.equal(ring, span), (hop, kind)
            del ring, span


# ---------------------------------------------------------------- FIR
def test_golden_fir_direct_bitexact(amd, golden):
    g = golden("fir_257_n16384")
    y = amd.fir_apply(g["h"], g["x"])
    assert np.array_equal(y, g["kiss"])   # same summation order as fir.c:170-186


def test_golden_fir_fft(amd, golden):
    g = golden("fir_257_n16384")
    y = amd.fir_apply(g["h"], g["x"], fft=True)
    np.testing.assert_allclose(y, g["np64"], rtol=3e-3, atol=3e-3)   # python/test_filters.py:32-33
    np.testing.assert_allclose(y, g["np64"], rtol=1e-5, atol=2e-6)
    g = golden("firfft_257_n1500")
    np.testing.assert_allclose(amd.fir_apply(g["h"], g["x"], fft=True), g["np64"], rtol=1e-5, atol=2e-6)


def test_fir_streaming_state_matches_reference(amd, orc):
    """vv_dsp_fir_apply across calls: history ring continues exactly (bit-exact)."""
    import ctypes as C
    rng = np.random.default_rng(3)
    h = orc.fir_design_lowpass(33, 0.2, 1)
    x = rng.standard_normal(5000).astype(np.float32)
    st = FirState()
    assert amd.lib.vv_dsp_fir_state_init(C.byref(st), 33) == OK
    try:
        chunks = [x[:7], x[7:40], x[40:41], x[41:3000], x[3000:]]
        y = np.concatenate([amd.fir_apply(h, c, state=st) for c in chunks])
    finally:
        amd.lib.vv_dsp_fir_state_free(C.byref(st))
    assert np.array_equal(y, orc.fir_apply(h, x))


@pytest.mark.parametrize("taps", [1, 2, 7, 64, 257, 1025, 5000])
def test_fir_fft_sizes(amd, orc, taps):
    rng = np.random.default_rng(taps)
    h = rng.standard_normal(taps).astype(np.float32) / np.sqrt(taps)
    for n in (1, 100, 20000):
        x = rng.standard_normal(n).astype(np.float32)
        y = amd.fir_apply(h, x, fft=True)
        ref = np.convolve(x.astype(np.float64), h.astype(np.float64))[:n]
        np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5)


def test_fir_filter_tests_impulse(amd):
    """filter_tests.c:17-39: fir_apply_fft on a minimal state ({0}, num_taps only)."""
    import ctypes as C
    h = amd.fir_design_lowpass(7, 0.3, 2)
    x = np.zeros(32, np.float32)
    x[0] = 1
    st = FirState()
    st.num_taps = 7
    y = np.zeros(32, np.float32)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    assert amd.lib.vv_dsp_fir_apply_fft(C.byref(st), fp(h), fp(x), fp(y), 32) == OK
    assert np.sum(y.astype(np.float64) ** 2) > 0
    np.testing.assert_allclose(y[:7], h, atol=1e-6)


def test_fir_multichannel_device(vdev, orc):
    import torch
    rng = np.random.default_rng(4)
    h = orc.fir_design_lowpass(257, 0.25, 2)
    x = rng.uniform(-1, 1, (3, 50000)).astype(np.float32)
    plan = vdev.FirPlan(torch.from_numpy(h))
    y = plan(torch.from_numpy(x).cuda()).cpu().numpy()
    yd = plan(torch.from_numpy(x).cuda(), direct=True).cpu().numpy()
    for c in range(3):
        assert np.array_equal(yd[c], orc.fir_apply(h, x[c]))
        np.testing.assert_allclose(y[c], yd[c], rtol=1e-5, atol=3e-6)


# ---------------------------------------------------------------- Hilbert / DCT
def test_golden_hilbert(amd, golden):
    for n in (1024, 255):
        g = golden(f"hilbert_n{n}")
        z = amd.hilbert(g["x"])
        np.testing.assert_allclose(z, g["np64"], rtol=1e-5, atol=1e-5)


def test_hilbert_sine_known_answer(amd):
    """hilbert_tests.c:16-48: bin-centred sine, real part within 1e-3, imag = -cos."""
    N, fs, k = 256, 1000.0, 31
    f0 = k * fs / N
    x = np.sin(2 * np.pi * f0 * np.arange(N) / fs).astype(np.float32)
    z = amd.hilbert(x)
    assert np.max(np.abs(z.real - x)) < 1e-3
    np.testing.assert_allclose(z.imag, -np.cos(2 * np.pi * f0 * np.arange(N) / fs), atol=1e-4)


@pytest.mark.parametrize("n", [4, 7, 8, 63, 64, 257, 1024, 4096])
def test_hilbert_sizes(amd, n):
    import scipy.signal
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    np.testing.assert_allclose(amd.hilbert(x), scipy.signal.hilbert(x.astype(np.float64)), rtol=1e-4, atol=2e-5)


def test_golden_dct(amd, golden):
    for n in (64, 1024):
        g = golden(f"dct2_n{n}")
        y = amd.dct(g["x"], 2, False)
        np.testing.assert_allclose(y, g["np64"], rtol=1e-4, atol=1e-4)
        xi = amd.dct(y, 2, True)
        np.testing.assert_allclose(xi, g["x"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n", [1, 2, 7, 8, 40, 63, 64, 256, 257, 400, 1000, 1024, 4800, 8192, 16384])
def test_dct_types_vs_formula(amd, n):
    import scipy.fft
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    x64 = x.astype(np.float64)
    tol = dict(rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(n) / 8))
    np.testing.assert_allclose(amd.dct(x, 2), scipy.fft.dct(x64, 2) / 2, **tol)
    np.testing.assert_allclose(amd.dct(x, 2, True), scipy.fft.idct(2 * x64, 2), **tol)
    np.testing.assert_allclose(amd.dct(x, 3, True), scipy.fft.idct(2 * x64, 2), **tol)
    np.testing.assert_allclose(amd.dct(x, 4), scipy.fft.dct(x64, 4) / 2, **tol)
    np.testing.assert_allclose(amd.dct(x, 4, True), scipy.fft.dct(x64, 4) / n, **tol)
    kk = np.arange(n)[:, None]
    nn = np.arange(n)[None, :]
    y3 = x64[0] + 2 * (np.cos(np.pi * kk * (nn + 0.5) / n)[:, 1:] @ x64[1:]) if n > 1 else x64[:1]
    np.testing.assert_allclose(amd.dct(x, 3), y3, **tol)


def test_dct_roundtrip_known_answer(amd):
    """dct_tests.c:11-50: DCT-II -> inverse and DCT-IV involution at n=8, 1e-5."""
    n = 8
    x = np.sin(np.float32(2 * np.pi) * np.arange(n, dtype=np.float32) / np.float32(n)).astype(np.float32)
    np.testing.assert_allclose(amd.dct(amd.dct(x, 2), 2, True), x, atol=1e-5)
    x4 = np.cos(2 * np.pi * (np.arange(n) + 0.3) / n).astype(np.float32)
    np.testing.assert_allclose(amd.dct(amd.dct(x4, 4), 4, True), x4, atol=1e-5)


# ---------------------------------------------------------------- mel / MFCC
MEL = [(512, 26, 16000.0, 0.0, 8000.0), (1024, 40, 48000.0, 20.0, 20000.0), (2048, 128, 44100.0, 0.0, 22050.0)]


def test_mfcc_reference_tests(amd):
    """tests/mfcc_tests.c of the reference, restated."""
    for hz in (0.0, 100.0, 1000.0, 4000.0, 8000.0):
        assert abs(amd.mel_to_hz(amd.hz_to_mel(hz)) - hz) <= 1e-3 * max(1.0, hz)
    assert amd.hz_to_mel(-100.0) == 0.0 and amd.mel_to_hz(-100.0) == 0.0
    st, fb = amd.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0)
    assert st == OK and fb.shape == (26, 257) and (fb > 0).any()
    power = (1.0 / (1.0 + np.arange(257, dtype=np.float32))).astype(np.float32)[None, :]
    m = amd.mfcc_pipeline(power, 512, 26, 13, 16000.0, 0.0, 8000.0, 22.0, 1e-10)
    assert m.shape == (1, 13) and np.isfinite(m).all()


@pytest.mark.parametrize("args", MEL)
def test_log_mel_and_mfcc_vs_oracle(amd, orc, args):
    n_fft, n_mels = args[0], args[1]
    st, fb = orc.mel_filterbank(*args)
    assert st == 0
    rng = np.random.default_rng(n_mels)
    power = ((rng.random((37, n_fft // 2 + 1)) ** 2) * 10).astype(np.float32)
    lm, lm_o = amd.log_mel(power, fb, 1e-10), orc.log_mel(power, fb, 1e-10)
    # the filterbank sums are bit-identical (same order, no FMA); logf may differ by an ulp
    np.testing.assert_allclose(lm, lm_o, rtol=1e-6, atol=1e-6)
    for lifter in (0.0, 22.0):
        m, m_o = amd.mfcc(lm_o, 13, lifter), orc.mfcc(lm_o, 13, lifter)
        # DCT-II: the reference accumulates cosf terms in f32 (dct.c:21-30), ours uses a
        # table rounded from double: normwise agreement at the harness tolerance
        assert _normwise(m, m_o) <= 5e-5, _normwise(m, m_o)
    p = amd.mfcc_pipeline(power, n_fft, n_mels, 13, args[2], args[3], args[4], 22.0, 1e-10)
    assert _normwise(p, orc.mfcc(lm_o, 13, 22.0)) <= 5e-5


def test_stft_power_to_mfcc_device(vdev, orc):
    """Device pipeline: multi-channel power spectrogram (STFT mode 2) -> fused
    log-mel + MFCC, against the oracle chain on NumPy f64 power spectra."""
    import torch
    nfft, hop, nch, n = 1024, 256, 3, 48000 + 333
    g = torch.Generator(device="cuda").manual_seed(8)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    pw = st.power(sig)
    fr = st.frames(n)
    assert pw.shape == (nch, fr, nfft // 2 + 1)
    x = sig.cpu().numpy().astype(np.float64)
    w = orc.window(1, nfft).astype(np.float64)
    ref_pw = []
    for c in range(nch):
        pad = np.concatenate([x[c], np.zeros(nfft)])
        F = np.fft.rfft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)
        ref_pw.append(np.abs(F) ** 2)
    ref_pw = np.stack(ref_pw)
    assert _normwise(pw.cpu().numpy(), ref_pw) <= 1e-5
    # fused log-mel + MFCC on the device (vv_dsp_mfcc_process_device / vv_dsp_log_mel_device)
    plan = vdev.Mfcc(nfft, 40, 13, 48000.0, 20.0, 20000.0, lifter=22.0, eps=1e-10)
    rows = nch * fr
    mf = plan(pw).reshape(rows, 13)
    lmd = plan.log_mel(pw).reshape(rows, 40)
    torch.cuda.synchronize()
    del plan
    _, fb = orc.mel_filterbank(nfft, 40, 48000.0, 20.0, 20000.0)
    lm_ref = orc.log_mel(ref_pw.reshape(rows, -1).astype(np.float32), fb, 1e-10)
    np.testing.assert_allclose(lmd.cpu().numpy(), lm_ref, rtol=1e-4, atol=1e-4)
    assert _normwise(mf.cpu().numpy(), orc.mfcc(lm_ref, 13, 22.0)) <= 1e-4


@pytest.mark.parametrize("nfft,hop,n,off", [(1024, 256, 48000 + 333, 0), (1024, 256, 48000 + 333, 1),
                                            (1024, 256, 48128, 0), (1024, 256, 48000, 1), (1024, 128, 48000, 2),
                                            (1024, 512, 20000, 3), (1024, 100, 9999, 0), (1024, 768, 30001, 0),
                                            (1024, 256, 1024 + 256, 0), (1024, 256, 700, 1),
                                            (256, 64, 10000, 1), (2048, 512, 30000, 0), (4096, 1024, 40000, 2)])
def test_stft_power_rows(vdev, orc, nfft, hop, n, off):
    """Power spectrogram (STFT mode 2, bins 0..nfft/2) per bin against NumPy f64
    on the same f32 input, and against the magnitude kernel squared.  `off`
    shifts the output by whole floats, so rows lose 16 B alignment (the
    staged dword-store path for nfft = 1024 needs only 4 B); odd frame counts
    exercise the pair whose second frame does not exist."""
    import torch
    nch = 3
    g = torch.Generator(device="cuda").manual_seed(nfft + hop + n)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr, nh = st.frames(n), nfft // 2 + 1
    buf = torch.full((off + nch * fr * nh + 64,), -7.0, device="cuda")
    out = buf[off:off + nch * fr * nh].view(nch, fr, nh)
    pw = st.power(sig, out=out)
    mag = st.spectrogram(sig)
    torch.cuda.synchronize()
    b = buf.cpu().numpy()
    assert np.all(b[:off] == -7.0) and np.all(b[off + nch * fr * nh:] == -7.0), "stores outside the rows"
    x = sig.cpu().numpy().astype(np.float64)
    w = orc.window(1, nfft).astype(np.float64)
    pw = pw.cpu().numpy()
    for c in range(nch):
        pad = np.concatenate([x[c], np.zeros(nfft + hop)])
        ref = np.abs(np.fft.rfft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)) ** 2
        scale = np.max(ref, axis=1, keepdims=True)
        # |X|^2 carries twice the relative error of |X|: 2 x VV_PY_RTOL/ATOL (python/test_fft.py:37-38)
        assert np.all(np.abs(pw[c] - ref) <= 1e-4 * np.abs(ref) + 1e-4 * scale), (c, np.max(np.abs(pw[c] - ref)))
    m2 = mag.cpu().numpy()[:, :, :nh].astype(np.float64) ** 2
    assert _normwise(pw, m2) <= 1e-5


@pytest.mark.parametrize("nfft,hop,n,off", [(1024, 256, 48128, 0), (1024, 256, 48000, 1), (1024, 512, 20000, 3),
                                            (1024, 256, 1280, 0), (1024, 256, 700, 1), (1024, 100, 9999, 0),
                                            (1024, 768, 30001, 2), (512, 128, 10000, 1), (2048, 512, 30000, 0)])
def test_stft_complex_rows(vdev, orc, nfft, hop, n, off):
    """Complex STFT rows (vv_dsp_stft_process batched over frames, full nfft bins,
    stft.c:74-92) per bin against NumPy f64 at the harness tolerance, with guard
    regions around the rows (odd frame counts: the pair without a second frame)."""
    import torch
    nch = 3
    g = torch.Generator(device="cuda").manual_seed(nfft * 3 + hop + n)
    sig = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr = st.frames(n)
    buf = torch.full((off + nch * fr * nfft + 64,), complex(-7.0, 3.0), dtype=torch.complex64, device="cuda")
    out = buf[off:off + nch * fr * nfft].view(nch, fr, nfft)
    y = st.spectrogram(sig, out=out, complex_out=True)
    torch.cuda.synchronize()
    b = buf.cpu().numpy()
    assert np.all(b[:off] == complex(-7.0, 3.0)) and np.all(b[off + nch * fr * nfft:] == complex(-7.0, 3.0))
    x = sig.cpu().numpy().astype(np.float64)
    w = orc.window(1, nfft).astype(np.float64)
    y = y.cpu().numpy()
    r, a = tolerances()
    for c in range(nch):
        pad = np.concatenate([x[c], np.zeros(nfft + hop)])
        ref = np.fft.fft(np.stack([pad[f * hop:f * hop + nfft] for f in range(fr)]) * w, axis=1)
        np.testing.assert_allclose(y[c], ref, rtol=r, atol=4 * a)


@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("nfft,hop,n", [(1024, 256, 48000 + 333), (1024, 256, 96000), (512, 128, 20001)])
def test_stft_frames_range(vdev, nfft, hop, n, kind):
    """vv_dsp_stft_frames_range_device: frame-range shards of one long signal
    (SURVEY 8e, config 3 sharded across GPUs).  Even frame0 (the frame_shard
    layout): rows bit-identical to the whole-signal call.  Odd frame0: the pair
    partners change, so within f32 rounding.  Ranges past the last frame fail."""
    import torch
    import vvdsp_dist
    g = torch.Generator(device="cuda").manual_seed(n + kind)
    sig = torch.rand(2, n, device="cuda", generator=g) * 2 - 1
    st = vdev.Stft(nfft, hop)
    fr = st.frames(n)
    full = {0: lambda: st.spectrogram(sig), 1: lambda: st.spectrogram(sig, complex_out=True),
            2: lambda: st.power(sig)}[kind]().cpu()
    for world in (1, 3, 8):
        parts = [st.frames_range(sig, lo, hi - lo, kind).cpu()
                 for lo, hi in (vvdsp_dist.frame_shard(fr, world, r) for r in range(world)) if hi > lo]
        assert torch.equal(torch.cat(parts, 1), full), world
    for lo, cnt in ((1, 5), (fr - 3, 3), (7, fr - 7)):
        y = st.frames_range(sig, lo, cnt, kind).cpu().numpy()
        ref = full[:, lo:lo + cnt].numpy()
        assert _normwise(y, ref) <= 2e-6, (lo, cnt)
    with pytest.raises(vdev.VvError, match="status 3"):   # VV_DSP_ERROR_OUT_OF_RANGE
        st.frames_range(sig, fr - 2, 3, kind)
    assert st.frames_range(sig, fr, 0, kind).shape[1] == 0


def test_golden_mel(amd, golden):
    g = golden("mel_512_26")
    st, fb = amd.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0)
    assert st == OK and np.array_equal(fb, g["fb"])   # host setup: bit-identical
    np.testing.assert_allclose(amd.log_mel(g["power"], fb, 1e-10), g["log_mel_kiss"], rtol=1e-6, atol=1e-6)
    assert _normwise(amd.mfcc(g["log_mel_kiss"], 13, 22.0), g["mfcc_kiss"]) <= 5e-5
    assert _normwise(amd.mfcc_pipeline(g["power"], 512, 26, 13, 16000.0, 0.0, 8000.0, 22.0, 1e-10),
                     g["mfcc_kiss"]) <= 5e-5


# ---------------------------------------------------------------- batched single-pass Hilbert / DCT-II
@pytest.mark.parametrize("n", [2, 8, 16, 32, 64, 128, 256, 1024, 2048, 4096, 8192])
def test_hilbert_batched_device(vdev, n):
    """vv_dsp_hilbert_analytic over a batch of rows (two rows per complex FFT,
    odd batch -> last row alone) vs scipy.signal.hilbert in f64."""
    import scipy.signal
    import torch
    rng = np.random.default_rng(100 + n)
    for batch in (1, 5, 64, 1029):
        x = rng.standard_normal((batch, n)).astype(np.float32)
        z = vdev.hilbert(torch.from_numpy(x).cuda()).cpu().numpy()
        ref = scipy.signal.hilbert(x.astype(np.float64), axis=1)
        assert _normwise(z, ref) <= 2e-6 * max(1.0, np.log2(n)), (n, batch, _normwise(z, ref))
        np.testing.assert_allclose(z.real, x, rtol=0, atol=0)   # the real part is the input itself


@pytest.mark.parametrize("n", [2, 4, 16, 32, 40, 64, 128, 256, 400, 512, 1000, 1024, 2048, 4096, 8192])
def test_dct2_batched_device(vdev, n):
    """DCT-II over a batch of rows (two rows per complex FFT where the FFT can
    be mirror-paired) vs scipy.fft.dct(type 2)/2 in f64 (dct.c:21-30)."""
    import scipy.fft
    import torch
    rng = np.random.default_rng(200 + n)
    for batch in (1, 3, 64, 1029):
        x = rng.standard_normal((batch, n)).astype(np.float32)
        y = vdev.dct(torch.from_numpy(x).cuda()).cpu().numpy()
        ref = scipy.fft.dct(x.astype(np.float64), 2, axis=1) / 2
        assert _normwise(y, ref) <= 2e-6 * max(1.0, np.log2(n)), (n, batch, _normwise(y, ref))


@pytest.mark.parametrize("policy", [0, 1, 2, 3])
def test_dct_nan_policy_matches_reference(amd, ref, policy):
    """NaN/Inf handling of vv_dsp_dct_execute (dct.c:98,130, nan_policy.c):
    same status as the reference, same non-finite pattern, finite values within
    tolerance -- for the single-pass (1024; 256 with its mirror bins through LDS)
    and the multi-pass (1000) paths."""
    import ctypes as C
    for n in (1024, 256, 1000):
        rng = np.random.default_rng(n + policy)
        x = rng.standard_normal(n).astype(np.float32)
        x[[3, 77]] = np.nan
        if policy != 3:
            # clamp maps +-Inf to +-FLT_MAX, whose FFT-based transform overflows where the
            # reference's O(n^2) f32 sums do not: only NaN is compared under clamp
            x[n // 2 - 12] = np.inf
        outs = []
        for lib in (amd, ref):
            lib.lib.vv_dsp_set_nan_policy.argtypes = [C.c_int]
            lib.lib.vv_dsp_set_nan_policy(policy)
            try:
                outs.append(lib.dct_status(x, 2, False))
            finally:
                lib.lib.vv_dsp_set_nan_policy(0)
        (st_a, y_a), (st_r, y_r) = outs
        assert st_a == st_r, (n, policy, st_a, st_r)
        if st_a == 0:
            fa, fr = np.isfinite(y_a), np.isfinite(y_r)
            assert np.array_equal(fa, fr) and np.array_equal(np.isnan(y_a), np.isnan(y_r))
            np.testing.assert_allclose(y_a[fa], y_r[fr], rtol=1e-4, atol=1e-2)


# ---------------------------------------------------------------- host-buffer pipeline
@pytest.mark.parametrize("chunk_mb", ["1", "3"])
def test_stft_host_pipeline_matches_device(amd, vdev, orc, chunk_mb, knob):
    """vv_dsp_stft_spectrogram with host buffers above the pipeline threshold runs
    frame chunks on two lanes (shim.hip run_lanes); chunks start on even frames, so
    every frame pair is the one a single launch forms and the rows are
    bit-identical to the one-launch host call; within one f32 ulp of the
    device-pointer call (whose unaligned channel stride sends the zero-padded
    tail pair through the register-load kernel variant), and within the harness
    bound of the reference restatement."""
    import torch
    rng = np.random.default_rng(11)
    n = 10 * 48000 + 333                       # 1874 frames, ragged tail
    x = rng.uniform(-1, 1, n).astype(np.float32)
    knob("HOST_CHUNK_MB", "1024")
    one = amd.spectrogram(x, 1024, 256)
    knob("HOST_CHUNK_MB", chunk_mb)
    mag = amd.spectrogram(x, 1024, 256)
    dev = vdev.Stft(1024, 256).spectrogram(torch.from_numpy(x).cuda()).cpu().numpy()
    assert mag.shape == one.shape == dev.shape == (1 + (n - 1024 + 256) // 256, 1024)
    assert np.array_equal(mag, one)
    np.testing.assert_allclose(mag, dev, rtol=2.5e-7, atol=0)
    ref = orc.spectrogram(x[: 48000 * 2], 1024, 256)   # first 2 s: a bounded oracle sample
    close(mag[: ref.shape[0] - 4], ref[: ref.shape[0] - 4], factor=2.0)


def test_fft_host_pipeline_matches_device(amd_lib_path, vdev, knob):
    """A batched plan executed on host buffers (vv_dsp_fft_make_plan_many +
    vv_dsp_fft_execute) in 1 MiB chunks on two lanes equals the device call."""
    import ctypes as C
    import torch
    knob("HOST_CHUNK_MB", "1")
    L = C.CDLL(amd_lib_path)
    L.vv_dsp_fft_make_plan_many.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    L.vv_dsp_fft_execute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.vv_dsp_fft_destroy.argtypes = [C.c_void_p]
    rng = np.random.default_rng(12)
    for kind, n, b in ((C2C, 1024, 301), (R2C, 2048, 257), (C2C, 1 << 16, 5)):
        if kind == C2C:
            x = (rng.random((b, n)) - 0.5 + 1j * (rng.random((b, n)) - 0.5)).astype(np.complex64)
            y = np.empty_like(x)
        else:
            x = (rng.random((b, n)) - 0.5).astype(np.float32)
            y = np.empty((b, n // 2 + 1), np.complex64)
        p = C.c_void_p()
        assert L.vv_dsp_fft_make_plan_many(n, kind, FWD, b, C.byref(p)) == OK
        try:
            assert L.vv_dsp_fft_execute(p, x.ctypes.data, y.ctypes.data) == OK
        finally:
            L.vv_dsp_fft_destroy(p)
        d = vdev.FftPlan(n, vdev.C2C if kind == C2C else vdev.R2C, vdev.FWD, batch=b)(
            torch.from_numpy(x).cuda()).cpu().numpy()
        assert np.array_equal(y, d), (kind, n, b)


def test_dct_error_policy_input_nan_leaves_output(amd, ref):
    """ERROR policy with a NaN input: status NAN and the output buffer untouched,
    as the reference returns before writing it (dct.c:96-100); with finite input
    but an overflowing output the output IS written (dct.c:128-131)."""
    import ctypes as C
    x = np.ones(64, np.float32)
    x[5] = np.nan
    for lib in (amd, ref):
        lib.lib.vv_dsp_set_nan_policy.argtypes = [C.c_int]
        lib.lib.vv_dsp_set_nan_policy(2)
        try:
            y = np.full(64, 7.0, np.float32)
            fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
            assert lib.lib.vv_dsp_dct_forward(64, 2, fp(x), fp(y)) == 5
            assert np.all(y == 7.0)
        finally:
            lib.lib.vv_dsp_set_nan_policy(0)


def test_nan_policy_is_per_thread(amd):
    """nan_policy.c:11-31 keeps the policy _Thread_local: another thread's setting
    does not leak into this one."""
    import ctypes as C
    import threading
    L = amd.lib
    L.vv_dsp_set_nan_policy.argtypes = [C.c_int]
    L.vv_dsp_get_nan_policy.restype = C.c_int
    L.vv_dsp_set_nan_policy(0)
    seen = []

    def other():
        L.vv_dsp_set_nan_policy(2)
        seen.append(L.vv_dsp_get_nan_policy())
    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == [2] and L.vv_dsp_get_nan_policy() == 0


def test_device_wrappers_check_shapes(vdev):
    """The Python device API checks tensors against the plan before handing
    pointers to the kernels (a wrong dtype or a short tensor would be read or
    written past its allocation)."""
    import torch
    p = vdev.FftPlan(1024, vdev.C2C, vdev.FWD, batch=4)
    with pytest.raises(vdev.VvError):
        p(torch.zeros(4, 1024, device="cuda"))                        # float32 into a C2C plan
    with pytest.raises(vdev.VvError):
        p(torch.zeros(3, 1024, dtype=torch.complex64, device="cuda"))   # too few rows
    with pytest.raises(vdev.VvError):
        p(torch.zeros(4, 1024, dtype=torch.complex64, device="cuda"),
          out=torch.zeros(4, 1000, dtype=torch.complex64, device="cuda"))
    st = vdev.Stft(1024, 256)
    with pytest.raises(vdev.VvError):
        st.reconstruct(torch.zeros(5, 1024, dtype=torch.complex64, device="cuda"),
                       torch.zeros(100, device="cuda"))
    with pytest.raises(vdev.VvError):
        st.spectrogram(torch.zeros(2, 4096, device="cuda"), out=torch.zeros(2, 3, 1024, device="cuda"))
