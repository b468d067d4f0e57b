"""CPU tests: the oracle (oracle/vv_oracle.c, our restatement of the reference)
is pinned bit-for-bit against the reference's own compiled sources
(oracle/_ref/libvvref.so) and against the committed golden vectors, and the
golden vectors themselves are checked against NumPy/SciPy f64 with the
reference harness tolerances (python/test_fft.py:37-38,62; test_filters.py:32-33)."""
import numpy as np
import pytest

from vvapi import C2C, R2C, C2R, FWD, BWD

SIZES = [1, 2, 3, 4, 5, 7, 8, 12, 16, 17, 31, 64, 100, 128, 256, 1024, 4096]


def test_oracle_fft_bitexact_vs_reference(orc, ref):
    rng = np.random.default_rng(11)
    for n in SIZES:
        x = (rng.random(n) + 1j * rng.random(n)).astype(np.complex64)
        for d in (FWD, BWD):
            assert np.array_equal(orc.fft(x, C2C, d), ref.fft(x, C2C, d)), (n, d)
        xr = rng.standard_normal(n).astype(np.float32)
        assert np.array_equal(orc.fft(xr, R2C), ref.fft(xr, R2C)), n
        if n <= 1024:
            X = np.fft.rfft(xr).astype(np.complex64)
            assert np.array_equal(orc.fft(X, C2R, BWD, n=n), ref.fft(X, C2R, BWD, n=n)), n


def test_oracle_stft_hilbert_dct_fir_bitexact(orc, ref):
    rng = np.random.default_rng(12)
    x = rng.uniform(-1, 1, 20000).astype(np.float32)
    for nfft, hop in [(1024, 256), (512, 128), (64, 64), (256, 1), (100, 30)]:
        assert np.array_equal(orc.spectrogram(x[:5000], nfft, hop), ref.spectrogram(x[:5000], nfft, hop))
    for n in [1, 2, 7, 8, 255, 256, 1024]:
        s = rng.standard_normal(n).astype(np.float32)
        assert np.array_equal(orc.hilbert(s), ref.hilbert(s)), n
        for t in (2, 3, 4):
            for inv in (False, True):
                assert np.array_equal(orc.dct(s, t, inv), ref.dct(s, t, inv)), (n, t, inv)
    for taps in [1, 2, 7, 33, 257]:
        for wk in (0, 1, 2, 3):
            a, b = orc.fir_design_lowpass(taps, 0.25, wk), ref.fir_design_lowpass(taps, 0.25, wk)
            assert np.array_equal(a, b, equal_nan=True), (taps, wk)
        h = orc.fir_design_lowpass(taps, 0.25, 2)
        assert np.array_equal(orc.fir_apply(h, x[:3000]), ref.fir_apply(h, x[:3000]), equal_nan=True)
        assert np.array_equal(orc.fir_apply(h, x[:400], fft=True), ref.fir_apply(h, x[:400], fft=True),
                              equal_nan=True)


def _sine_analytic(n, fs, f0, ref):
    """the reference hilbert_tests.c:16-48 input: a bin-centred sine's analytic signal"""
    t = np.arange(n) / fs
    return ref.hilbert(np.sin(2 * np.pi * f0 * t).astype(np.float32))


def test_oracle_inst_phase_freq_bitexact(orc, ref):
    """hilbert.c:77-113 restated: phase (f64 increments summed left to right) and
    frequency (f64 difference x fs/2pi) bit-identical to the compiled reference."""
    rng = np.random.default_rng(21)
    cases = [_sine_analytic(256, 1000.0, 31 * 1000.0 / 256, ref), _sine_analytic(16384, 48000.0, 440.0, ref)]
    for n in (1, 2, 3, 255, 4096, 20000):
        cases.append((rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64))
    z = np.zeros(64, np.complex64)   # atan2(0, 0) = 0 increments
    z[10] = 1 + 1j
    cases.append(z)
    for z in cases:
        pa, pb = orc.inst_phase(z), ref.inst_phase(z)
        assert np.array_equal(pa, pb), len(z)
        for fs in (1000.0, 48000.0, 1.0):
            assert np.array_equal(orc.inst_freq(pa, fs), ref.inst_freq(pb, fs)), (len(z), fs)
    # the reference test's acceptance (hilbert_tests.c:40-43): mean frequency within 0.5 Hz of f0
    f0 = 31 * 1000.0 / 256
    fr = orc.inst_freq(orc.inst_phase(_sine_analytic(256, 1000.0, f0, ref)), 1000.0)
    assert abs(fr[1:].astype(np.float64).mean() - f0) < 0.5


MEL_CASES = [(512, 26, 16000.0, 0.0, 8000.0), (1024, 40, 48000.0, 20.0, 20000.0), (2048, 128, 44100.0, 0.0,
                                                                                   22050.0), (256, 10, 8000.0, 300.0, 3400.0)]


def test_oracle_mel_mfcc_bitexact(orc, ref):
    """src/features/mel.c restated: conversions, filterbank, log-mel and MFCC
    bit-identical to the reference compiled in place (oracle/_ref)."""
    for hz in (0.0, 1.0, 440.0, 1000.0, 8000.0, 24000.0, -5.0):
        assert orc.hz_to_mel(hz) == ref.hz_to_mel(hz)
        assert orc.mel_to_hz(hz) == ref.mel_to_hz(hz)
    rng = np.random.default_rng(21)
    for n_fft, n_mels, sr, fmin, fmax in MEL_CASES:
        st_o, fb_o = orc.mel_filterbank(n_fft, n_mels, sr, fmin, fmax)
        st_r, fb_r = ref.mel_filterbank(n_fft, n_mels, sr, fmin, fmax)
        assert st_o == st_r == 0
        assert np.array_equal(fb_o, fb_r)
        power = (rng.random((7, n_fft // 2 + 1)) ** 2).astype(np.float32)
        lm_o, lm_r = orc.log_mel(power, fb_o, 1e-10), ref.log_mel(power, fb_r, 1e-10)
        assert np.array_equal(lm_o, lm_r)
        nc = min(13, n_mels)
        for ncoef, lifter in ((nc, 22.0), (n_mels, 0.0)):
            assert np.array_equal(orc.mfcc(lm_o, ncoef, lifter), ref.mfcc(lm_r, ncoef, lifter))
        assert np.array_equal(ref.mfcc_pipeline(power, n_fft, n_mels, nc, sr, fmin, fmax, 22.0, 1e-10),
                              orc.mfcc(orc.log_mel(power, fb_o, 1e-10), nc, 22.0))
    # argument validation is the reference's (mel.c:78-98)
    assert orc.mel_filterbank(512, 300, 16000.0, 0.0, 8000.0)[0] == ref.mel_filterbank(512, 300, 16000.0, 0.0,
                                                                                        8000.0)[0] == 2
    assert orc.mel_filterbank(512, 26, 16000.0, 0.0, 9000.0)[0] == ref.mel_filterbank(512, 26, 16000.0, 0.0,
                                                                                       9000.0)[0] == 3


def test_oracle_matches_golden(orc, golden):
    g = golden("fft_testpy_n1024")
    assert np.array_equal(orc.fft(g["x"], C2C, FWD), g["c2c_fwd_kiss"])
    assert np.array_equal(orc.fft(g["x"], C2C, BWD), g["c2c_bwd_kiss"])
    assert np.array_equal(orc.fft(g["xr"], R2C), g["r2c_kiss"])
    assert np.array_equal(orc.fft(g["X"], C2R, BWD, n=1024), g["c2r_kiss"])
    g = golden("fft_batch64_n1024")
    for i in range(0, 64, 9):
        assert np.array_equal(orc.fft(g["x"][i], C2C, FWD), g["kiss"][i])
    g = golden("stft_48000_n1024_h256")
    assert np.array_equal(orc.window(1, 1024), g["window"])
    assert np.array_equal(orc.spectrogram(g["x"], 1024, 256), g["kiss"])
    for n in (1024, 255):
        g = golden(f"hilbert_n{n}")
        assert np.array_equal(orc.hilbert(g["x"]), g["kiss"])
    for n in (64, 1024):
        g = golden(f"dct2_n{n}")
        assert np.array_equal(orc.dct(g["x"], 2, False), g["kiss"])
        assert np.array_equal(orc.dct(g["kiss"], 2, True), g["inv_kiss"])
    g = golden("fir_257_n16384")
    assert np.array_equal(orc.fir_design_lowpass(257, 0.25, 2), g["h"])
    assert np.array_equal(orc.fir_apply(g["h"], g["x"]), g["kiss"])
    g = golden("firfft_257_n1500")
    assert np.array_equal(orc.fir_apply(g["h"], g["x"], fft=True), g["kiss"])
    g = golden("mel_512_26")
    assert np.array_equal(orc.mel_filterbank(512, 26, 16000.0, 0.0, 8000.0)[1], g["fb"])
    assert np.array_equal(orc.log_mel(g["power"], g["fb"], 1e-10), g["log_mel_kiss"])
    assert np.array_equal(orc.mfcc(g["log_mel_kiss"], 13, 22.0), g["mfcc_kiss"])
    np.testing.assert_allclose(g["log_mel_kiss"], g["log_mel_np64"], rtol=1e-5, atol=1e-5)


def _err_over_tol(y, ref, rtol, atol):
    return float(np.max(np.abs(y - ref) / (atol + rtol * np.abs(ref))))


def test_golden_kiss_accuracy_profile(golden):
    """The reference's own accuracy vs f64: C2C/R2C pass the
    harness tolerance at n=1024, its O(n^2) C2R does not (1.22x)."""
    g = golden("fft_testpy_n1024")
    assert _err_over_tol(g["c2c_fwd_kiss"], g["c2c_fwd_np64"], 5e-5, 5e-5) < 1.0
    assert _err_over_tol(g["r2c_kiss"], g["r2c_np64"], 5e-5, 5e-5) < 1.0
    assert _err_over_tol(g["c2r_kiss"], g["c2r_np64"], 5e-5, 5e-5) > 1.0
    g = golden("fft_testpy_n16")
    for k in ("c2c_fwd", "c2c_bwd", "r2c", "c2r"):
        assert _err_over_tol(g[k + "_kiss"], g[k + "_np64"], 5e-5, 5e-5) < 1.0, k
    g = golden("stft_48000_n1024_h256")
    assert _err_over_tol(g["kiss"], g["np64"], 5e-5, 5e-5) < 1.0
    g = golden("fir_257_n16384")
    np.testing.assert_allclose(g["kiss"], g["np64"], rtol=3e-3, atol=3e-3)
    for n in (1024, 255):
        g = golden(f"hilbert_n{n}")
        assert np.max(np.abs(g["kiss"] - g["np64"])) < 1e-4


# ---- CZT and cepstrum family (src/spectral/czt.c, src/envelope/cepstrum.c, minphase.c) ----
CZT_CASES = [(8, 8), (32, 32), (100, 64), (257, 300), (1000, 17), (1, 5), (5, 1)]


def test_oracle_czt_bitexact_vs_reference(orc, ref):
    """czt.c:22-178 restated (float chirps, Kiss FFTs of P = next_pow2(N+M-1)):
    bit-identical to the compiled reference for complex and real input, DFT and
    zoom parameters."""
    rng = np.random.default_rng(31)
    for n, m in CZT_CASES:
        x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        for w, a in ((np.exp(-2j * np.pi / n), 1.0 + 0j), (np.exp(-2j * np.pi * 0.37 / m), np.exp(0.3j)),
                     (1.001 * np.exp(-0.05j), 0.999 * np.exp(0.2j))):
            assert np.array_equal(orc.czt(x, m, w, a), ref.czt(x, m, w, a), equal_nan=True), (n, m, w, a)
            xr = x.real.astype(np.float32)
            assert np.array_equal(orc.czt(xr, m, w, a), ref.czt(xr, m, w, a), equal_nan=True), (n, m)
    for args in ((800.0, 1200.0, 64, 48000.0), (0.0, 24000.0, 1024, 48000.0), (-100.0, 100.0, 3, 1000.0)):
        assert orc.czt_params(*args) == ref.czt_params(*args)
    assert ref.czt_params(0.0, 1.0, 0, 1000.0)[0] == orc.czt_params(0.0, 1.0, 0, 1000.0)[0] == 2
    assert ref.czt_params(0.0, 1.0, 4, 0.0)[0] == orc.czt_params(0.0, 1.0, 4, 0.0)[0] == 2


def test_reference_czt_known_answers(ref):
    """czt_tests.c:10-39 (impulse -> ones at DFT parameters, 1e-3) and the
    reference's python/test_czt.py cases against scipy.signal.czt at its
    rtol = atol = 2e-4 (N = M = 32 and the 800-1200 Hz zoom of a 1 kHz tone)."""
    from scipy.signal import czt
    n = 8
    x = np.zeros(n, np.complex64)
    x[0] = 1
    X = ref.czt(x, n, np.exp(-2j * np.pi / n), 1.0 + 0j)
    assert np.allclose(X, 1.0, atol=1e-3)
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(32) + 1j * rng.standard_normal(32)).astype(np.complex64)
    w = complex(np.complex64(np.exp(-2j * np.pi / 32)))
    np.testing.assert_allclose(ref.czt(x, 32, w, 1.0 + 0j), czt(x.astype(np.complex128), m=32, w=w, a=1.0),
                               rtol=2e-4, atol=2e-4)
    fs, f0 = 48000.0, 1000.0
    xr = np.cos(2 * np.pi * f0 * np.arange(32) / fs).astype(np.float32)
    W = np.exp(-1j * 2 * np.pi * ((1200.0 - 800.0) / 64) / fs)
    A = np.exp(-1j * 2 * np.pi * 800.0 / fs)
    Wf, Af = complex(np.complex64(W)), complex(np.complex64(A))
    np.testing.assert_allclose(ref.czt(xr, 64, Wf, Af), czt(xr.astype(np.float64), m=64, w=Wf, a=Af),
                               rtol=2e-4, atol=2e-4)


def test_oracle_cepstrum_family_bitexact_vs_reference(orc, ref):
    """cepstrum.c:7-78 and minphase.c:7-31 restated: bit-identical (NaN/inf where
    the reference's expf overflows compare equal too)."""
    rng = np.random.default_rng(32)
    for n in (1, 2, 3, 16, 17, 64, 100, 1024):
        x = rng.standard_normal(n).astype(np.float32)
        assert np.array_equal(orc.cepstrum(x), ref.cepstrum(x), equal_nan=True), n
        for c in (x, (0.05 * x).astype(np.float32)):
            assert np.array_equal(orc.icepstrum_minphase(c), ref.icepstrum_minphase(c), equal_nan=True), n
            assert np.array_equal(orc.minphase_from_cepstrum(c), ref.minphase_from_cepstrum(c), equal_nan=True), n


def test_reference_envelope_known_answers(ref):
    """envelope_tests.c:9-23: an impulse's cepstrum is ~0 (c0 1e-3, others 1e-2)
    and its minimum-phase inverse starts at ~1."""
    x = np.zeros(16, np.float32)
    x[0] = 1
    c = ref.cepstrum(x)
    assert abs(c[0]) < 1e-3 and np.all(np.abs(c[1:]) < 1e-2)
    assert abs(ref.icepstrum_minphase(c)[0] - 1.0) < 1e-2
    assert np.all(np.isfinite(ref.minphase_from_cepstrum(c).view(np.float32)))


def test_oracle_spectral_utils_bitexact_vs_reference(orc, ref):
    """utils.c:5-73 restated: shifts (real and complex, even and odd n), phase wrap
    and unwrap (float accumulation) bit-identical; spectral_tests.c:71-81's
    fftshift/ifftshift round trip; n = 0 codes.  For odd n the reference rotates
    by n/2 rounded down in the fftshift direction (utils.c:8-12), i.e. NumPy's
    ifftshift: kept as the reference has it."""
    rng = np.random.default_rng(41)
    for n in (1, 2, 5, 8, 9, 1024, 1001):
        x = rng.standard_normal(n).astype(np.float32)
        z = (x + 1j * rng.standard_normal(n)).astype(np.complex64)
        for f in ("fftshift", "ifftshift"):
            assert np.array_equal(getattr(orc, f)(x), getattr(ref, f)(x)), (f, n)
            assert np.array_equal(getattr(orc, f)(z), getattr(ref, f)(z)), (f, n)
            if n % 2 == 0:   # odd n: the reference's fftshift is NumPy's ifftshift and vice versa
                assert np.array_equal(getattr(orc, f)(x), getattr(np.fft, f)(x)), (f, n)
        ph = (rng.standard_normal(n) * 20).astype(np.float32)
        assert np.array_equal(orc.phase_wrap(ph), ref.phase_wrap(ph)), n
        steps = np.cumsum(rng.uniform(-3, 3, n)).astype(np.float32)
        w = ref.phase_wrap(steps)
        assert np.array_equal(orc.phase_unwrap(w), ref.phase_unwrap(w)), n
    a = np.arange(5, dtype=np.float32)
    assert np.array_equal(ref.ifftshift(ref.fftshift(a)), a)
    assert ref._util("fftshift", np.zeros(0, np.float32))[0] == 2
    assert ref._util("phase_unwrap", np.zeros(0, np.float32))[0] == 2
    assert ref._util("phase_wrap", np.zeros(0, np.float32))[0] == 0


def test_oracle_czt_cepstrum_golden(orc, golden):
    """The committed CZT / cepstrum fixtures (tests/golden/make_golden.py section 8):
    the restatement reproduces the reference outputs bit for bit, and those sit
    within the reference harness tolerance of SciPy / NumPy f64 (rtol = atol =
    2e-4 for CZT, python/test_czt.py)."""
    g = golden("czt_testpy_n32")
    w = complex(g["w"][0])
    assert np.array_equal(orc.czt(g["x"], 32, w, 1.0 + 0j), g["kiss"])
    np.testing.assert_allclose(g["kiss"], g["np64"], rtol=2e-4, atol=2e-4)
    g = golden("czt_zoom_n32_m64")
    W, A = complex(g["w"][0]), complex(g["a"][0])
    assert np.array_equal(orc.czt(g["x"], 64, W, A), g["kiss"])
    np.testing.assert_allclose(g["kiss"], g["np64"], rtol=2e-4, atol=2e-4)
    g = golden("cepstrum_n64")
    assert np.array_equal(orc.cepstrum(g["x"]), g["ceps_kiss"])
    assert np.array_equal(orc.icepstrum_minphase(g["c"]), g["iceps_kiss"])
    assert np.array_equal(orc.minphase_from_cepstrum(g["c"]), g["minph_kiss"])
    for k in ("ceps", "iceps", "minph"):
        np.testing.assert_allclose(g[k + "_kiss"], g[k + "_np64"], rtol=1e-4, atol=1e-4)


def test_oracle_filtfilt_bitexact_vs_reference(orc, ref):
    """Zero-phase FIR (filter/common.c:6-80): the restatement against the
    reference compiled from its own sources, bit for bit -- long signals, signals
    shorter than the padding (the reflection clamps), a single tap -- and the
    reference test's case (filter_tests.c:62-80: 9-tap Hamming lowpass on a
    square wave, centre mean below 0.2)."""
    rng = np.random.default_rng(31)
    for taps, n in [(9, 64), (1, 10), (2, 1), (5, 3), (33, 20), (257, 4000), (64, 1000), (1000, 300)]:
        h = rng.standard_normal(taps).astype(np.float32) * 0.2
        x = rng.uniform(-1, 1, n).astype(np.float32)
        st, yr = ref.filtfilt(h, x)
        assert st == 0
        assert np.array_equal(orc.filtfilt(h, x), yr), (taps, n)
    h = ref.fir_design_lowpass(9, 0.25, 1)
    x = np.where(np.arange(64) % 8 < 4, 1.0, -1.0).astype(np.float32)
    y = orc.filtfilt(h, x)
    assert abs(float(np.mean(y[9:55]))) < 0.2


def test_oracle_round2_golden(orc, golden):
    """Round-2 fixtures (tests/golden/make_golden.py round2_sets): the
    restatement reproduces the reference's zero-phase FIR, its O(n^2) DFT at the
    7-smooth lengths 400 / 480 and its STFT with 400-sample frames bit for bit,
    and the float64 counterparts sit where the reference's own f32 arithmetic
    puts them (filtfilt within 1e-5; the f32 DFT within 2e-3 at these sizes)."""
    g = golden("filtfilt")
    assert np.array_equal(orc.filtfilt(g["h9"], g["xq"]), g["yq_kiss"])
    assert np.array_equal(orc.filtfilt(g["h257"], g["xg"]), g["yg_kiss"])
    np.testing.assert_allclose(g["yq_kiss"], g["yq_np64"], atol=1e-5)
    np.testing.assert_allclose(g["yg_kiss"], g["yg_np64"], atol=1e-5)
    g = golden("fft_smooth_400_480")
    assert np.array_equal(orc.fft(g["x"], C2C, FWD), g["c2c_fwd_kiss"])
    assert np.array_equal(orc.fft(g["x"], C2C, BWD), g["c2c_bwd_kiss"])
    assert np.array_equal(orc.fft(g["xr"], R2C), g["r2c_kiss"])
    np.testing.assert_allclose(g["c2c_fwd_kiss"], g["c2c_fwd_np64"], atol=2e-3)
    g = golden("stft_16000_n400_h160")
    assert np.array_equal(orc.spectrogram(g["x"], 400, 160), g["kiss"])
    np.testing.assert_allclose(g["kiss"], g["np64"], atol=2e-3)


REGISTER_LENGTHS = (320, 400, 441, 480, 600, 640, 720, 800, 900, 960)


def test_oracle_register_golden(orc, golden):
    """The restatement reproduces the reference's outputs in the round-3
    fixtures bit for bit: c2c and R2C at every register-kernel length (the
    reference's O(n^2) DFT, fft_kiss.c:76-92 via :114-116, R2C :120-147), the
    spectrogram rows (stft.c:112-144) and the complex rows of
    vv_dsp_stft_process (stft.c:74-92: window, then C2C)."""
    for n in REGISTER_LENGTHS:
        g = golden(f"register_n{n}")
        assert np.array_equal(orc.fft(g["x"], C2C, FWD), g["c2c_fwd_kiss"]), n
        assert np.array_equal(orc.fft(g["x"], C2C, BWD), g["c2c_bwd_kiss"]), n
        hop = int(g["hop"][0])
        assert np.array_equal(orc.spectrogram(g["sig"], n, hop), g["stft_mag_kiss"]), n
        w = orc.window(1, n)
        pad = np.concatenate([g["sig"], np.zeros(n, np.float32)])
        for f in range(g["stft_cpx_kiss"].shape[0]):
            fr = (pad[f * hop: f * hop + n] * w).astype(np.complex64)
            assert np.array_equal(orc.fft(fr, C2C, FWD), g["stft_cpx_kiss"][f]), (n, f)
        # the reference's f32 O(n^2) DFT is itself ~1e-4 relative off f64 here
        np.testing.assert_allclose(g["c2c_fwd_kiss"], g["c2c_fwd_np64"], rtol=1e-3, atol=5e-3)
    g = golden("register_r2c")
    for key in (k for k in g if k.startswith("x")):
        n = int(key[1:])
        assert np.array_equal(orc.fft(g[key], R2C), g[f"kiss{n}"]), n


def test_perfect_reconstruction_known_answer(orc, ref):
    """tests/gtest/test_stft.cpp:452-519 (512/128 Hann, three tones, max error
    < 1e-3, RMS < 1e-5 over [512, 1536)) holds for the compiled reference
    through its own API and for the oracle's restatement: the known answer the
    GPU tests (test_gpu_parity.py::test_stft_perfect_reconstruction_*) assert."""
    import ctypes as C
    from test_gpu_parity import _pr_check, _pr_signal
    x, F, H = _pr_signal()
    fp = lambda a, off=0: a[off:].ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    st, h = ref.stft_create(F, H, 1)
    assert st == 0
    try:
        y, norm = np.zeros(len(x), np.float32), np.zeros(len(x), np.float32)
        for start in range(0, len(x) - F + 1, H):
            spec = np.ascontiguousarray(ref.stft_process(h, np.ascontiguousarray(x[start:start + F]), F).view(np.float32))
            assert ref.lib.vv_dsp_stft_reconstruct(h, fp(spec), fp(y, start), fp(norm, start)) == 0
        ref_err = _pr_check(x, y, norm, F)
    finally:
        ref.lib.vv_dsp_stft_destroy(h)
    w = orc.window(1, F)
    y, norm = np.zeros(len(x), np.float32), np.zeros(len(x), np.float32)
    for start in range(0, len(x) - F + 1, H):
        spec = orc.fft((x[start:start + F] * w).astype(np.complex64), C2C, FWD)
        row = np.ascontiguousarray(spec.view(np.float32))
        assert orc.lib.orc_stft_reconstruct(fp(w), F, fp(row), fp(y, start), fp(norm, start)) == 0
    assert _pr_check(x, y, norm, F) == ref_err   # the restatement reproduces the reference's errors exactly
